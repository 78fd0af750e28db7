#!/bin/bash
# Tuning sweep: all variant builds x env knobs, interleaved in one process.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_variants.py "$@" > gpurun_out/sweep.log 2> gpurun_out/sweep.err; rc=$?
echo "rc=$rc"; exit $rc
