#!/bin/bash
# round 4, job y: config 3 fabric traffic, one vs two samples per box (same build, same process)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES"; do
  T=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$T -o p -- python tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 2 --reps 2 --env "VR_DUO=0" "" "VR_DUO=3" > $O/variants_$T.log 2>&1 || { tail -20 $O/variants_$T.log; exit 1; }
done
python tools/rank_pmc.py $O/FETCH_SIZE/p_counter_collection.csv $O/WRITE_SIZE/p_counter_collection.csv > $O/pmc_duo.log || exit 1
cat $O/pmc_duo.log
python - <<'PY' >> $O/pmc_duo.log
import csv, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/r4y/SQ_INSTS_VMEM_RD/p_counter_collection.csv")):
    if "vr::k_march" in r["Kernel_Name"]:
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k[0][:50], k[1], sum(v) / len(v))
PY
tail -8 $O/pmc_duo.log
echo done
