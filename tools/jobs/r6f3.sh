# round 6 session 3: config-5 at-size parity on every 8th row, then the remaining 1024^3 workloads on the HEAD build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6f3; mkdir -p $O
( while sleep 50; do date >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gmm.py -k config5_at_size -x -v -s --durations=0 --timeout 500 --timeout-method thread > $O/pytest_config5.log 2>&1; rc=$?; tail -3 $O/pytest_config5.log; [ $rc -ne 0 ] && exit $rc
RANKSIM=0 bash tools/gpu_round.sh r6f3 1024x8:C1 1024x8:S 1024x8:C0::3 gmm1024:C0 || exit 1
echo ok
