#!/bin/bash
# GPU parity tests, then an in-process sweep (args passed to bench_variants.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/bench_variants.py "$@" > gpurun_out/sweep.log 2> gpurun_out/sweep.err; rc=$?
echo "sweep rc=$rc"; exit $rc
