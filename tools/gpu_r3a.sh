cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3a && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --maxfail=30 --timeout 300 --timeout-method thread > gpurun_out/r3a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/r3a/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r3a/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3a/bench.log; exit 1; }
grep '^{' gpurun_out/r3a/bench.log
