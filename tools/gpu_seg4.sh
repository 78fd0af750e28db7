#!/bin/bash
# rank_sim with the pipelined 2-lane / 1-lane segmented march at every rank count, and the
# full frame with the same variants (bench_variants)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/seg4 && export TMPDIR=/tmp
O=gpurun_out/seg4
for s in -2 -1; do
  timeout -k 10 200 env VR_SEG=$s VR_SEG_RAYS=3000000 python -u tools/rank_sim.py --reps 5 > $O/s$s.log 2>&1 || { cat $O/s$s.log; exit 1; }
  echo "== VR_SEG=$s all ranks"; grep "cost N=" $O/s$s.log
done
timeout -k 10 300 python -u tools/bench_variants.py --rounds 4 --cameras C0,C1 --env "" VR_PATH=7,VR_SEG=-2 VR_PATH=7,VR_SEG=-1 VR_PATH=7,VR_SEG=-4 > $O/full.log 2>&1 || { cat $O/full.log; exit 1; }
cat $O/full.log
