#!/bin/bash
# round 4, job f: two-stream head/tail split for rank lists
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_layout.py > $O/pytest_r4f.log 2>&1 || { tail -30 $O/pytest_r4f.log; exit 1; }
ENVS=("" "VR_HEAD=64,VR_HEAD_STREAM=1" "VR_HEAD=128,VR_HEAD_STREAM=1" "VR_HEAD=256,VR_HEAD_STREAM=1" "VR_HEAD=128,VR_HEAD_STREAM=1,VR_HEAD_TAILPATH=7" "VR_HEAD=64,VR_HEAD_STREAM=1,VR_HEAD_SEG=-8" "VR_HEAD=128,VR_HEAD_STREAM=1,VR_HEAD_SEG=-2")
timeout -k 10 400 python -u tools/rank_sim.py --camera C0 --worlds 2,4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0_split.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --rounds 5 --env "" "VR_PATH=7,VR_SEG=-2" "VR_PATH=7,VR_SEG=-4" > $O/variants_256x4.log 2>&1 || exit 1
echo done
