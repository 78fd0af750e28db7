#!/bin/bash
# Bench lines of the wide-record configs (16 / 32 bins, the reference's own
# record width) on the current build, no CPU baseline (a 128 GiB volume).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/wide; mkdir -p $O
for W in "1024x32 C0 1" "1024x32 C1 1" "1024x32 C0 3" "1024x16 C0 1" "1024x16 C1 1" "512x32 C0 1" "512x32 C1 1"; do
  read CFG CAM M <<< "$W"
  timeout -k 10 300 python -u bench.py --config $CFG --camera $CAM --method $M --no-cpu-baseline > $O/bench_${CFG}_${CAM}_m$M.log 2>&1 || { tail -20 $O/bench_${CFG}_${CAM}_m$M.log; exit 1; }
  echo "$CFG $CAM m$M $(grep -o '"value": [0-9.]*' $O/bench_${CFG}_${CAM}_m$M.log | head -1) $(grep -o '"kernel": "[^"]*", "kernel_ms": [0-9.]*' $O/bench_${CFG}_${CAM}_m$M.log)"
done
