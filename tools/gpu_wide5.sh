#!/bin/bash
# wide records: PMC of the quad march at 1024^3 x 32 C0; entropy / method-7 bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
KPAT=k_march_wq bash tools/gpu_wide_pmc.sh || exit 1
for CFG in 1024x32 1024x16; do
  for CAM in C0 C1; do
    for M in 3 7; do
      timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method $M --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/${CFG}_${CAM}_m$M.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_m$M.log; exit 1; }
      echo "$CFG $CAM m$M $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m$M.log) $(grep -o '"frac": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m$M.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_m$M.log)"
    done
  done
done
