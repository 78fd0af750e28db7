#!/bin/bash
# round 4, job s: N = 4 rank lists -- march variants (C0, S)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 500 python -u tools/rank_sim.py --camera C0 --worlds 4 --modes cost --host-ms 0.017 --envs "" "VR_SEG=-4" "VR_SEG=2" "VR_SEG_RAYS=0" "VR_PATH=1" "VR_HEAD=64,VR_HEAD_SEG=-8" > $O/rank_sim_C0_N4_paths.log 2>&1 || exit 1
grep -v amdgpu.ids $O/rank_sim_C0_N4_paths.log
timeout -k 10 500 python -u tools/rank_sim.py --camera S --worlds 4,8 --modes cost --host-ms 0.017 --envs "" "VR_SEG=-4" "VR_HEAD=128" "VR_SEG_RAYS=0" > $O/rank_sim_S_paths.log 2>&1 || exit 1
grep -v amdgpu.ids $O/rank_sim_S_paths.log
echo done
