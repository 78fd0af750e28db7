#!/bin/bash
# round 4, job ak: N = 4 frame loop on two streams -- 2-lane windows vs the one-lane march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4ak; mkdir -p $O
for ENV in "" "VR_SEG_RAYS=0" "VR_SEG=-4"; do
  timeout -k 10 300 python -u tools/host_cost.py --world 4 --camera C0 --streams-only --env "$ENV" > $O/h.log 2>&1 || { tail -20 $O/h.log; exit 1; }
  echo "env [$ENV]"; grep "full frame\|streams=2\]\|ring=8\]:" $O/h.log
done
echo done
