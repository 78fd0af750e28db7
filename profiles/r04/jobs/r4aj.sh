#!/bin/bash
# round 4, job aj: multi-GPU simulations on the final build (rank lists, frame loop)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4aj; mkdir -p $O
for CAM in C0 C1 S; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM --worlds 2,4,8 --modes cost --host-ms 0.017 > $O/rank_sim_$CAM.log 2>&1 || { tail -20 $O/rank_sim_$CAM.log; exit 1; }
done
for CN in C0:8 C0:4 C1:8 C1:4 S:8 S:4; do
  IFS=: read CAM N <<< "$CN"
  timeout -k 10 300 python -u tools/host_cost.py --world $N --camera $CAM --streams-only > $O/host_cost_${CAM}_N${N}.log 2>&1 || { tail -20 $O/host_cost_${CAM}_N${N}.log; exit 1; }
  grep "rank 0 of\|full frame\|streams=2\]\|ring=8\]:" $O/host_cost_${CAM}_N${N}.log
done
echo done
