#!/bin/bash
# Small full frames (BASELINE configs 1-2) on the ray-segmented march: GPU parity
# tests of the path choices, bench lines of both configs at C0 and C1.
# usage: bash tools/gpu_small.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/small && export TMPDIR=/tmp
O=gpurun_out/small
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_bench.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in 128x1 256x4; do
  for CAM in C0 C1; do
    timeout -k 10 200 python -u bench.py --config $C --camera $CAM --no-cpu-baseline --warmup 10 --steps 50 > $O/bench_${C}_$CAM.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/bench_${C}_$CAM.log').read().strip().splitlines()[-1]); print('$C $CAM', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
  done
done
