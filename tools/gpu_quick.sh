#!/bin/bash
# full GPU test suite + rank_sim (C0) + default bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/q && export TMPDIR=/tmp
O=gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/rank_sim.py > $O/rank_C0.log 2>&1 || { cat $O/rank_C0.log; exit 1; }
grep -v amdgpu.ids $O/rank_C0.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log
