#!/bin/bash
# Baked statistics: parity, rank split (seg vs pipe for short lists), bench + rocprof
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/baked3; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_baked.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for E in "" "VR_PATH=2"; do
echo "== rank_sim baked C0 env '$E'"
timeout -k 10 300 python -u tools/rank_sim.py --baked --camera C0 --env "$E" > $O/rank_C0_$E.log 2>&1 || { tail -20 "$O/rank_C0_$E.log"; exit 1; }
grep "full frame\|N=" "$O/rank_C0_$E.log"
done
timeout -k 10 300 python -u bench.py --baked --no-cpu-baseline > $O/bench_C0.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench_C0.json
timeout -k 10 300 python -u bench.py --baked --no-cpu-baseline --camera C1 > $O/bench_C1.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench_C1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --baked --no-cpu-baseline --steps 20 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv"
timeout -k 10 300 python -u tools/rank_sim.py --baked --camera C1 > $O/rank_C1.log 2>&1 || { tail -20 $O/rank_C1.log; exit 1; }
grep "full frame\|N=" $O/rank_C1.log
