#!/bin/bash
# round 4, job a: rank-list head split / unconditional-gather variants + host cost
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4a; mkdir -p $O
ENVS=("" "VR_HEAD=64" "VR_HEAD=128" "VR_HEAD=256" "VR_HEAD=64,VR_HEAD_SEG=-8" "VR_HEAD=128,VR_HEAD_SEG=-8")
timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0_main.log 2>&1 || exit 1
VRDD_LIB=tools/build/variants/uncond/libvr.so timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0_uncond.log 2>&1 || exit 1
VRDD_LIB=tools/build/variants/uncw3/libvr.so timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "" "VR_HEAD=128" > $O/rank_sim_C0_uncw3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 4 > $O/host_cost_N4.log 2>&1 || exit 1
echo done
