#!/bin/bash
# host issue overhead per bench step (small config) + rank_sim two-pass
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/host && export TMPDIR=/tmp
O=gpurun_out/host
timeout -k 10 300 python -u bench.py --config 256x4 --steps 400 --no-cpu-baseline > $O/bench_small.log 2>&1 || { cat $O/bench_small.log; exit 1; }
tail -1 $O/bench_small.log | cut -c1-400
timeout -k 10 300 python -u tools/rank_sim.py > $O/rank_C0.log 2>&1 || { cat $O/rank_C0.log; exit 1; }
grep -v amdgpu.ids $O/rank_C0.log
