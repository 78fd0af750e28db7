#!/bin/bash
# wide-record marches: parity tests, then bench lines per kernel (VR_WIDE=1 lane-per-record, 0 quad)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wide or bin_counts or isabel" > gpurun_out/wide/pytest.log 2>&1 || { tail -30 gpurun_out/wide/pytest.log; exit 1; }
tail -2 gpurun_out/wide/pytest.log
for CFG in ${CFGS:-1024x32 1024x16 512x32}; do
  for CAM in C0 C1; do
    for W in ${WIDES:-0}; do
      VR_WIDE=$W timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method 1 --no-cpu-baseline --steps 10 > gpurun_out/wide/${CFG}_${CAM}_w$W.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_w$W.log; exit 1; }
      echo "$CFG $CAM w$W $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_w$W.log) $(grep -o '"frac": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_w$W.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_w$W.log)"
    done
  done
done
