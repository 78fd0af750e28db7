# round 6: row-aligned 1-4-bin entropy on the pipelined march -- tests, timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6ai; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_multi.py tests/test_gpu_io.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x1@1920x1080 --cameras C0 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=4" "VR_PATH=1" "VR_PATH=7" > $O/m3_1024x1.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_variants.py --config 1024x2@1920x1080 --cameras C0 --method 3 --rounds 2 --reps 2 --env "" "VR_PATH=4" > $O/m3_1024x2_after.log 2>&1 || exit 1
echo ok
