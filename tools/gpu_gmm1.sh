#!/bin/bash
# GMM path: GPU parity tests + first timings.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/gmm1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_gmm.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -30 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/gmm_time.py --dim 512 > $O/time512.log 2>&1; rc=$?; cat $O/time512.log; exit $rc
