#!/bin/bash
# round 4, job t: fabric traffic of the N = 4 / 8 C0 rank lists against the full frame
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4t; mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$C -o p -- python tools/rank_sim.py --camera C0 --worlds 4,8 --modes cost --reps 2 > $O/rank_sim_$C.log 2>&1 || { tail -20 $O/rank_sim_$C.log; exit 1; }
done
python tools/rank_pmc.py $O/FETCH_SIZE/p_counter_collection.csv $O/WRITE_SIZE/p_counter_collection.csv > $O/rank_pmc_C0.log || exit 1
cat $O/rank_pmc_C0.log
echo done
