#!/bin/bash
# rank_sim: default kernel choice vs one-lane pipe everywhere (VR_SEG_RAYS=1) vs seg everywhere
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/segthr && export TMPDIR=/tmp
O=gpurun_out/segthr
timeout -k 10 300 env VR_SEG_RAYS=1 python -u tools/rank_sim.py > $O/pipe.log 2>&1 || { cat $O/pipe.log; exit 1; }
grep -v amdgpu.ids $O/pipe.log
timeout -k 10 300 env VR_SEG_RAYS=2000000 python -u tools/rank_sim.py > $O/seg.log 2>&1 || { cat $O/seg.log; exit 1; }
grep -v amdgpu.ids $O/seg.log
