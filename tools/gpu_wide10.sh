#!/bin/bash
# codec (methods 4/5/6) on 32-bin records: bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
for CFG in ${CFGS:-1024x32}; do
  for CAM in C0 C1; do
    for M in 4 5 6; do
      timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method $M --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/wide/${CFG}_${CAM}_m$M.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_${CAM}_m$M.log; exit 1; }
      echo "$CFG $CAM m$M $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m$M.log) $(grep -o '"frac": [0-9.]*' gpurun_out/wide/${CFG}_${CAM}_m$M.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_${CAM}_m$M.log)"
    done
  done
done
