#!/bin/bash
# round 4, job x: frame loop on 1-4 alternating render streams (C0 N = 4 / 8)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4x; mkdir -p $O
for N in 4 8; do
  timeout -k 10 300 python -u tools/host_cost.py --world $N --camera C0 --streams-only > $O/host_cost_C0_N${N}_streams.log 2>&1 || { tail -20 $O/host_cost_C0_N${N}_streams.log; exit 1; }
  grep "rank 0 of\|full frame\|live" $O/host_cost_C0_N${N}_streams.log
done
echo done
