#!/bin/bash
# Wide records (16 / 32 bins, the reference's own histogram width): bench lines C0 / C1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wide && export TMPDIR=/tmp
for CFG in 512x32 1024x16 1024x32; do
  for CAM in C0 C1; do
    timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --no-cpu-baseline --steps 10 > gpurun_out/wide/${CFG}_$CAM.log 2>&1 || { tail -5 gpurun_out/wide/${CFG}_$CAM.log; exit 1; }
    echo "$CFG $CAM $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/wide/${CFG}_$CAM.log) $(grep -o '"frac": [0-9.]*' gpurun_out/wide/${CFG}_$CAM.log) $(grep -o '"value": [0-9.]*' gpurun_out/wide/${CFG}_$CAM.log) $(grep -o '"kernel": "[^"]*"' gpurun_out/wide/${CFG}_$CAM.log)"
  done
done
