#!/bin/bash
# The whole -m gpu suite and smoke() on the tree as it is (what the driver runs at round end).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; mkdir -p $O
# heartbeat under gpurun_out: a test that runs bench.py as a subprocess prints
# nothing for a minute or more (each test still has its --timeout)
( while sleep 50; do date >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=20 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -n "FAILED\|Error" $O/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; exit $rc
