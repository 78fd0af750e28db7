#!/bin/bash
# rank_sim with estimate vs cost-dealt tile lists, C0 and C1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cost && export TMPDIR=/tmp
O=gpurun_out/cost
for cam in C0 C1; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $cam > $O/rank_$cam.log 2>&1 || { tail -20 $O/rank_$cam.log; exit 1; }
  grep -v amdgpu.ids $O/rank_$cam.log
done
