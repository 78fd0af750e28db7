#!/bin/bash
# 32-bin records from baked statistics (basicDataProcessing): bench lines m1 / m3 / m7, C0 / C1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
for CAM in C0 C1; do
  for M in 1 3 7; do
    timeout -k 10 300 python -u bench.py --config 1024x32 --baked --camera $CAM --method $M --no-cpu-baseline --steps 10 > gpurun_out/wide/baked_${CAM}_m$M.log 2>&1 || { tail -5 gpurun_out/wide/baked_${CAM}_m$M.log; exit 1; }
    echo "1024x32 baked $CAM m$M $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/baked_${CAM}_m$M.log) $(grep -o '"bake_ms": [0-9.]*' gpurun_out/wide/baked_${CAM}_m$M.log) $(grep -o '"value": [0-9.]*' gpurun_out/wide/baked_${CAM}_m$M.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/baked_${CAM}_m$M.log)"
  done
done
