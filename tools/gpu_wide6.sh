#!/bin/bash
# wide-record entropy through the quad march: parity, then m3 bench lines (VR_PATH=1: old LDS box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or isabel" > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for CFG in 1024x32 1024x16; do
  for CAM in C0 C1; do
    timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method 3 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/${CFG}_${CAM}_m3.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_m3.log; exit 1; }
    echo "$CFG $CAM m3 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m3.log) $(grep -o '"frac": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m3.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_m3.log)"
  done
done
