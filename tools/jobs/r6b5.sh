# round 6 (session 2): compact pixel blocks per wave for the segmented / one-lane pipelined marches (VR_SEG_MAP=1)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6b5; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_baked.py -k "every_kernel_path or baked_paths or plane8" > $O/pytest_map.log 2>&1 || { tail -30 $O/pytest_map.log; exit 1; }
tail -1 $O/pytest_map.log
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --baked --cameras C1,C0 --method 1 --rounds 5 --reps 5 --env "" "VR_SEG_MAP=1" "VR_PATH=2" "VR_PATH=2,VR_SEG_MAP=1" > $O/map_baked_1024x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 512x8 --baked --cameras C1 --method 1 --rounds 5 --reps 5 --env "" "VR_SEG_MAP=1" > $O/map_baked_512x8.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --method 1 --rounds 5 --reps 5 --env "" "VR_SEG_MAP=1" > $O/map_256x4.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 128x1 --cameras C0,C1 --method 1 --rounds 5 --reps 5 --env "" "VR_SEG_MAP=1" > $O/map_128x1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C0,C1 --method 1 --rounds 3 --reps 3 --env "VR_PATH=7,VR_SEG=-2" "VR_PATH=7,VR_SEG=-2,VR_SEG_MAP=1" "VR_PATH=7,VR_SEG=4" "VR_PATH=7,VR_SEG=4,VR_SEG_MAP=1" > $O/map_1024x8_seg.log 2>&1 || exit 1
grep -E "median" $O/map_*.log
echo ok
