#!/bin/bash
# round 4, job v: N > 1 frames on two alternating render streams -- bench tests, frame loop cost
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py > $O/pytest_r4v.log 2>&1 || { tail -30 $O/pytest_r4v.log; exit 1; }
tail -1 $O/pytest_r4v.log
for N in 8 4; do
  timeout -k 10 400 python -u tools/host_cost.py --world $N --streams-only > $O/host_cost_N${N}_streams.log 2>&1 || { tail -20 $O/host_cost_N${N}_streams.log; exit 1; }
  grep -v amdgpu.ids $O/host_cost_N${N}_streams.log
done
timeout -k 10 400 python -u tools/host_cost.py --world 8 --camera C1 --streams-only > $O/host_cost_N8_C1_streams.log 2>&1 || exit 1
grep -v amdgpu.ids $O/host_cost_N8_C1_streams.log
echo done
