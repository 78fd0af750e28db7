#!/bin/bash
# round 4, job c: head-split sweep on the unconditional-gather build, host cost of the new loop, wave timelines
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layout.py tests/test_gpu_parity.py -k "layout or head or segmented or axis or tile_split or every_kernel or environment" > $O/pytest_r4.log 2>&1 || { tail -30 $O/pytest_r4.log; exit 1; }
tail -2 $O/pytest_r4.log
ENVS=("" "VR_HEAD=32" "VR_HEAD=64" "VR_HEAD=96" "VR_HEAD=128" "VR_HEAD=32,VR_HEAD_SEG=-8" "VR_HEAD=64,VR_HEAD_SEG=-8")
timeout -k 10 300 python -u tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/rank_sim.py --camera S --worlds 4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_S.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 > $O/host_cost_N8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 8 --env VR_HEAD=64 > $O/host_cost_N8_head64.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_cost.py --world 4 > $O/host_cost_N4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wave_timeline.py --camera C0 --world 8 --cost --ranks 0 --env "" > $O/wave_timeline_N8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wave_timeline.py --camera C0 --world 8 --cost --ranks 0 --env VR_HEAD=64 > $O/wave_timeline_N8_head64.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wave_timeline.py --camera C0 --world 4 --cost --ranks 0 --env "" > $O/wave_timeline_N4.log 2>&1 || exit 1
echo done
