#!/bin/bash
# Bricked baked-statistics planes: GPU tests of the baked path, bench lines of
# baked frames (methods 1 and 7, C0 and C1), PMC traffic of the baked m1 frames.
# usage: bash tools/gpu_planes.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/planes && export TMPDIR=/tmp
O=gpurun_out/planes
timeout -k 10 600 python -u -m pytest tests/test_gpu_baked.py tests/test_gpu_random.py tests/test_gpu_bench.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for M in ${METHODS:-1 7}; do
  for CAM in C0 C1; do
    timeout -k 10 200 python -u bench.py --baked --method $M --camera $CAM --no-cpu-baseline --warmup 10 > $O/bench_m${M}_$CAM.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/bench_m${M}_$CAM.log').read().strip().splitlines()[-1]); print('baked m$M $CAM', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['config']['bake_ms'])"
  done
done
for CAM in C0 C1; do
  bash tools/gpu_pmc1.sh "1024x8|$CAM|m1|baked" planes/pmc_$CAM -- --baked --camera $CAM || exit 1
done
