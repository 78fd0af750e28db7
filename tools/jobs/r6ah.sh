# round 6: dispatch changes (wide side/top views and coarse oblique entropy on the box; 2/4-bin entropy on the pipelined march)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ah; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "wide" > $O/pytest_fullsize_wide.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x4@1920x1080 --cameras C0,C1 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=0" > $O/m3_1024x4.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x2@1920x1080 --cameras C0,C1 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=1" "VR_PATH=2" "VR_PATH=0" > $O/m3_1024x2.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 512x32@1920x1080 --cameras C1,S --method 3 --rounds 2 --reps 2 > $O/m3_512x32_after.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 256x4 --cameras C0,C1 --method 3 --rounds 2 --reps 3 > $O/m3_256x4_after.log 2>&1 || exit 1
echo ok
