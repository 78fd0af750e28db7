#!/bin/bash
# round 4, job w: frame loop speed-up (full frame / loop period, gather + unscatter included),
# one vs two alternating render streams
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4w; mkdir -p $O
for CN in C0:8 C0:4 C1:8 C1:4 S:8 S:4; do
  IFS=: read CAM N <<< "$CN"
  timeout -k 10 300 python -u tools/host_cost.py --world $N --camera $CAM --streams-only > $O/host_cost_${CAM}_N${N}_streams.log 2>&1 || { tail -20 $O/host_cost_${CAM}_N${N}_streams.log; exit 1; }
  grep "rank 0 of\|full frame\|live" $O/host_cost_${CAM}_N${N}_streams.log
done
echo done
