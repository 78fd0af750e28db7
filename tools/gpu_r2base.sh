#!/bin/bash
# Round-2 baseline on a fresh box: GPU tests + C0/C1 bench lines.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r02base; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py > $O/bench_C0.log 2>&1 || { tail -20 $O/bench_C0.log; exit 1; }
tail -1 $O/bench_C0.log | cut -c1-400
timeout -k 10 300 python -u bench.py --camera C1 --no-cpu-baseline > $O/bench_C1.log 2>&1 || { tail -20 $O/bench_C1.log; exit 1; }
tail -1 $O/bench_C1.log | cut -c1-400
