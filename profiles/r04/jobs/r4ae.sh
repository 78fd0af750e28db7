#!/bin/bash
# round 4, job ae: GPU suite after the mid-size box rule, and config 2's bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r4ae || exit 1
O=gpurun_out/r4ae
timeout -k 10 600 python -u bench.py --config 256x4 > $O/bench_256x4.log 2>&1 || { tail -20 $O/bench_256x4.log; exit 1; }
tail -1 $O/bench_256x4.log | cut -c1-400
echo done
