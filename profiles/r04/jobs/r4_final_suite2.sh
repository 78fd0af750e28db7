#!/bin/bash
# round 4 final tree: the whole -m gpu suite + smoke, then bench.py with the driver's
# default arguments (the N = 1 headline line as the driver runs it)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
bash tools/gpu_suite.sh r4suite2 || exit 1
O=gpurun_out/r4suite2
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-300
echo done
