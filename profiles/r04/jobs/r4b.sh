#!/bin/bash
# round 4, job b: unconditional seg decode (143 VGPRs), head splits with pipe / segp2 tails, host cost loop variants
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
ENVS=("" "VR_HEAD=64" "VR_HEAD=32,VR_HEAD_TAIL=1" "VR_HEAD=64,VR_HEAD_TAIL=1" "VR_HEAD=128,VR_HEAD_TAIL=1" "VR_HEAD=64,VR_HEAD_SEG=-2,VR_HEAD_TAIL=1" "VR_HEAD=128,VR_HEAD_SEG=-2,VR_HEAD_TAIL=1")
timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0_main.log 2>&1 || exit 1
E2=("" "VR_SEG_RAYS=2000000" "VR_SEG_RAYS=2000000,VR_HEAD=64,VR_HEAD_TAIL=1" "VR_SEG_RAYS=2000000,VR_HEAD=128,VR_HEAD_TAIL=1" "VR_SEG_RAYS=2000000,VR_HEAD=128,VR_HEAD_SEG=-2,VR_HEAD_TAIL=1")
timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 2 --modes cost --envs "${E2[@]}" > $O/rank_sim_C0_N2.log 2>&1 || exit 1
VRDD_LIB=tools/build/variants/segw4/libvr.so timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "" "VR_HEAD=64" "VR_HEAD=64,VR_HEAD_TAIL=1" > $O/rank_sim_C0_segw4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rank_sim.py --camera S --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_S_main.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8.log 2>&1 || exit 1
echo done
