#!/bin/bash
# Copy a tools/gpu_round.sh run (gpurun_out/<TAG>) into profiles/<DEST> and
# profiles/traffic.json.  usage: tools/collect_profiles.sh TAG DEST
set -e
cd "$(dirname "$0")/.."
R=gpurun_out/$1; D=profiles/$2
mkdir -p $D/pmc
for f in $R/bench_*.log; do
  n=$(basename $f .log); n=${n#bench_}
  grep '^{' $f > $D/bench_$n.json
  [ -f $R/ktrace/${n}_kernel_stats.csv ] && cp $R/ktrace/${n}_kernel_stats.csv $D/kernel_stats_$n.csv
  for p in 1 2 3 4; do
    c=$(ls $R/pmc_$n/p$p/*counter_collection.csv 2>/dev/null | head -1)
    [ -n "$c" ] && cp $c $D/pmc/${n}_p$p.csv
  done
done
for c in C0 C1; do [ -f $R/rank_sim_$c.log ] && grep -v amdgpu.ids $R/rank_sim_$c.log > $D/rank_sim_1024x8_$c.log; done
[ -f $R/pytest_gpu.log ] && cp $R/pytest_gpu.log $D/pytest_gpu.log
[ -f $R/traffic.json ] && python3 - "$R/traffic.json" <<'PY'
import json, sys
new = json.load(open(sys.argv[1]))
db = json.load(open("profiles/traffic.json"))
db.update(new)
json.dump(db, open("profiles/traffic.json", "w"), indent=1, sort_keys=True)
print("traffic.json:", sorted(new))
PY
ls $D
true
