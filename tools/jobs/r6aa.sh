# round 6: 8-bin side-view entropy routed to the LDS-box march -- tests, timing
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "S" > $O/pytest_fullsize_S.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x8 --cameras S,C0 --method 3 --rounds 3 > $O/side_m3.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_variants.py --config 1024x4@1920x1080 --cameras S --method 3 --rounds 3 --env "" "VR_PATH=1" "VR_PATH=0" > $O/side_m3_nb4.log 2>&1 || exit 1
echo ok
