#!/bin/bash
# method 7 for wide records: parity (wide tests + bin counts + random sweep), bench m7 (VR_M7_WQ=0: k_march_m7)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or isabel or random or method7" > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for CFG in 1024x32 1024x16; do
  for CAM in C0 C1; do
    timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method 7 --no-cpu-baseline --steps 10 > gpurun_out/wide/${CFG}_${CAM}_m7.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_m7.log; exit 1; }
    echo "$CFG $CAM m7 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m7.log) $(grep -o '"value": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m7.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_m7.log)"
  done
done
