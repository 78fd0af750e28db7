# round 6 (session 2): 16x4 pixel blocks for the one-lane method-7 marches and the 16-bin row march
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b9; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "block_map or codec" > $O/pytest_map.log 2>&1 || { tail -30 $O/pytest_map.log; exit 1; }
tail -1 $O/pytest_map.log
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1,S --method 7 --rounds 3 --reps 3 --env "" "VR_M7_MAP=1" > $O/m7_1024x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --cameras C0,C1 --method 7 --rounds 3 --reps 3 --env "" "VR_M7_MAP=1" > $O/m7_512x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x4@1920x1080 --cameras C0,C1 --method 7 --rounds 3 --reps 3 --env "" "VR_M7_MAP=1" > $O/m7_1024x4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --method 7 --rounds 3 --reps 3 --env "" "VR_M7_MAP=1" > $O/m7_256x4.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x16@1920x1080 --cameras C0 --method 1 --rounds 3 --reps 3 --env "VR_PATH=2" "VR_PATH=2,VR_WIDE_MAP=1" "" > $O/wide_1024x16.log 2>&1 || exit 1
grep -E "median" $O/m7_*.log $O/wide_*.log
echo ok
