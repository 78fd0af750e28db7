# round 6: entropy terms in chunks of 4 -- parity, and the codec entropy frame (method 6) against the committed build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baked.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config 1024x8 --method 6 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_m6_main.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config 1024x8 --method 3 --camera C1 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_m3C1_main.log 2>&1 || exit 1
cp tools/build/variants/prev/libvr.so volume-rendering-based-on-distribution-data_amd/csrc/build/libvr.so
timeout -k 10 600 python -u bench.py --config 1024x8 --method 6 --no-cpu-baseline --steps 10 --warmup 3 > $O/bench_m6_prev.log 2>&1 || exit 1
echo ok
