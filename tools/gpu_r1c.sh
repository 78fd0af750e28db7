#!/bin/bash
# GPU suite + rank_sim (estimate vs cost-dealt lists) + default bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r1c && export TMPDIR=/tmp
O=gpurun_out/r1c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|error" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/rank_sim.py > $O/rank_C0.log 2>&1 || { cat $O/rank_C0.log; exit 1; }
grep -v amdgpu.ids $O/rank_C0.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
tail -1 $O/bench.log
