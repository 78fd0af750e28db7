#!/bin/bash
# Round-end rehearsal: all GPU tests, smoke(), default bench line.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python -u bench.py --method 7 --camera C1 --no-cpu-baseline > $O/bench_m7c1.log 2>&1 || { tail $O/bench_m7c1.log; exit 1; }
grep -o '"kernel_ms": [0-9.]*' $O/bench_m7c1.log
