#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fin && export TMPDIR=/tmp
O=gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in 1 2 3 7; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --method $m > $O/bench_m$m.log 2>&1 || { tail -20 $O/bench_m$m.log; exit 1; }; tail -1 $O/bench_m$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('m$m', d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], r['traffic'])"; done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --camera C1 > $O/bench_C1.log 2>&1 || { tail -20 $O/bench_C1.log; exit 1; }; tail -1 $O/bench_C1.log | cut -c1-200
timeout -k 10 300 python -u tools/rank_sim.py > $O/rank_C0.log 2>&1 || { cat $O/rank_C0.log; exit 1; }
grep -v amdgpu.ids $O/rank_C0.log | grep -v longest
