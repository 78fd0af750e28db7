# round 6 session 3: config-5 at-size parity over the WHOLE 3840x2160 frame (one-off; the suite checks every 8th row),
# then the baked C1 frame timed by bench.py at a longer warm-up / more frames beside tools/bench_variants.py
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6f4; mkdir -p $O
( while sleep 50; do date >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
VR_CONFIG5_ROW_STEP=1 timeout -k 10 1000 python -u -m pytest tests/test_gpu_gmm.py -k config5_at_size -x -v -s --durations=0 --timeout 950 --timeout-method thread > $O/pytest_config5_full.log 2>&1; rc=$?; tail -3 $O/pytest_config5_full.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config 1024x8 --camera C1 --baked --steps 200 --warmup 50 --no-cpu-baseline --no-issue-bounds > $O/bench_baked_C1_long.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_variants.py --config 1024x8 --cameras C1,C0 --method 1 --baked --rounds 3 > $O/variants_baked.log 2>&1 || exit 1
echo ok
