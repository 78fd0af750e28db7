#!/bin/bash
# Round-3: rank simulation with compact band dealing, bench issue bounds of the smaller configs.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/${1:-r3d}; mkdir -p $O
guard() { rc=$1; if [ $rc -ne 0 ]; then echo "$2 failed rc=$rc"; tail -20 $3; exit $rc; fi; }
for CAM in C1 C0; do
  timeout -k 10 300 python -u tools/rank_sim.py --camera $CAM > $O/rank_sim_$CAM.log 2>&1; guard $? rank-$CAM $O/rank_sim_$CAM.log
  grep -v amdgpu $O/rank_sim_$CAM.log | grep "N=8\|steady"
done
for CFG in 128x1 256x4 512x8; do
  timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline > $O/bench_$CFG.log 2>&1; guard $? bench-$CFG $O/bench_$CFG.log
  grep -o '"kernel_ms": [0-9.]*\|"issue_bounds": {[^}]*}' $O/bench_$CFG.log
done
echo done
