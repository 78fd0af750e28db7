#!/bin/bash
# rank_sim at C0 m1 for the seg-lane variants (VR_SEG: S lanes per ray, negative = pipelined)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/seg3 && export TMPDIR=/tmp
O=gpurun_out/seg3
for s in 4 -4 8 -8 2 -2; do
  timeout -k 10 200 env VR_SEG=$s python -u tools/rank_sim.py --reps 5 > $O/s$s.log 2>&1 || { cat $O/s$s.log; exit 1; }
  echo "== VR_SEG=$s"; grep "cost N=8\|cost N=4" $O/s$s.log
done
