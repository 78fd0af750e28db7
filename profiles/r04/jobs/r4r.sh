#!/bin/bash
# round 4, job r: N = 4 / 8 rank lists -- cost-dealing block shapes and head slots
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 500 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --blocks 1x4,2x4,1x8,2x2,4x4 --host-ms 0.017 > $O/rank_sim_C0_blocks.log 2>&1 || exit 1
grep -v amdgpu.ids $O/rank_sim_C0_blocks.log
timeout -k 10 500 python -u tools/rank_sim.py --camera C0 --worlds 4 --modes cost --host-ms 0.017 --envs "" "VR_HEAD=64" "VR_HEAD=128" "VR_HEAD=256" "VR_HEAD=512" > $O/rank_sim_C0_N4_head.log 2>&1 || exit 1
grep -v amdgpu.ids $O/rank_sim_C0_N4_head.log
timeout -k 10 500 python -u tools/rank_sim.py --camera C1 --worlds 4,8 --modes cost --blocks 1x4,2x4,2x2 --host-ms 0.017 > $O/rank_sim_C1_blocks.log 2>&1 || exit 1
grep -v amdgpu.ids $O/rank_sim_C1_blocks.log
echo done
