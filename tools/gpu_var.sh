#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/var && export TMPDIR=/tmp
O=gpurun_out/var
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in 2 1; do timeout -k 10 300 python -u tools/bench_variants.py --cameras C0,C1 --rounds 4 --method $m > $O/ab_m$m.log 2>&1 || { tail -30 $O/ab_m$m.log; exit 1; }; grep -v amdgpu.ids $O/ab_m$m.log | tail -4; done
