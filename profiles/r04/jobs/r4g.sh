#!/bin/bash
# round 4, job g: entropy dispatch after the reverts; two-stream head split; config 2 segmented; tests
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_layout.py > $O/pytest_r4g.log 2>&1 || { tail -30 $O/pytest_r4g.log; exit 1; }
tail -1 $O/pytest_r4g.log
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=0" "VR_PATH=4" > $O/variants_1024x8_m3.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=0" > $O/variants_512x8_m3.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x16 --cameras C0,C1 --method 3 --rounds 2 --env "" "VR_PATH=1" > $O/variants_1024x16_m3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --rounds 5 --env "" "VR_PATH=7,VR_SEG=-2" "VR_PATH=7,VR_SEG=-4" > $O/variants_256x4.log 2>&1 || exit 1
ENVS=("" "VR_HEAD=64,VR_HEAD_STREAM=1" "VR_HEAD=128,VR_HEAD_STREAM=1" "VR_HEAD=256,VR_HEAD_STREAM=1" "VR_HEAD=128,VR_HEAD_STREAM=1,VR_HEAD_TAILPATH=7" "VR_HEAD=64,VR_HEAD_STREAM=1,VR_HEAD_SEG=-8")
timeout -k 10 400 python -u tools/rank_sim.py --camera C0 --worlds 2,4,8 --modes cost --envs "${ENVS[@]}" > $O/rank_sim_C0_split.log 2>&1 || exit 1
echo done
