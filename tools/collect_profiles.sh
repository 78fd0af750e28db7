#!/bin/bash
# Copy a gpu_round.sh run (gpurun_out/<TAG>) into profiles/<DEST> and refresh
# profiles/traffic.json.  usage: tools/collect_profiles.sh TAG DEST
set -e
cd "$(dirname "$0")/.."
R=gpurun_out/$1; D=profiles/$2
mkdir -p $D/pmc
for c in C0 C1; do
  cp $R/ktrace/${c}_kernel_stats.csv $D/kernel_stats_1024x8_$c.csv
  grep '^{' $R/bench_1024x8_$c.log > $D/bench_1024x8_$c.json
  for p in 1 2 3; do cp $R/pmc_$c/p$p/p${p}_counter_collection.csv $D/pmc/${c}_p$p.csv; done
done
if [ -f $R/bench_1024x8_C0_baked.log ]; then
  grep '^{' $R/bench_1024x8_C0_baked.log > $D/bench_1024x8_C0_baked.json
  cp $R/ktrace/C0_baked_kernel_stats.csv $D/kernel_stats_1024x8_C0_baked.csv
  for p in 1 2 3; do cp $R/pmc_C0_baked/p$p/p${p}_counter_collection.csv $D/pmc/C0_baked_p$p.csv; done
fi
if [ -f $R/bench_1024x8_C1_baked.log ]; then
  grep '^{' $R/bench_1024x8_C1_baked.log > $D/bench_1024x8_C1_baked.json
  for p in 1 2 3; do cp $R/pmc_C1_baked/p$p/p${p}_counter_collection.csv $D/pmc/C1_baked_p$p.csv; done
fi
[ -f $R/pytest_gpu.log ] && cp $R/pytest_gpu.log $D/pytest_gpu.log
for c in C0 C1; do [ -f $R/rank_sim_$c.log ] && grep -v amdgpu.ids $R/rank_sim_$c.log > $D/rank_sim_1024x8_$c.log; done
cp $R/traffic.json profiles/traffic.json
ls $D
