#!/bin/bash
# round 4, job h: tests incl. bench end-to-end (batched waits), host cost of the new loop, dispatch checks
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_bench.py > $O/pytest_r4h.log 2>&1 || { tail -30 $O/pytest_r4h.log; exit 1; }
tail -1 $O/pytest_r4h.log
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 4 > $O/host_cost_N4.log 2>&1 || exit 1
for A in "1024x16:C0:3" "512x8:C1:3" "256x4:C1:1" "256x4:C0:1"; do
  IFS=: read CFG CAM MTH <<< "$A"
  timeout -k 10 400 python -u bench.py --config $CFG --camera $CAM --method $MTH --no-cpu-baseline > $O/bench_${CFG}_${CAM}_m$MTH.log 2>&1 || exit 1
done
echo done
