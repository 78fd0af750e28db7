#!/bin/bash
# round 4, job aa: config 3 -- occupancy caps on the two-sample box march, L2 hit rates
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4aa; mkdir -p $O
timeout -k 10 600 python -u tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 5 --env "VR_DUO=0" "" "VR_WG_PER_CU=3" "VR_WG_PER_CU=2" "VR_DUO=0,VR_WG_PER_CU=3" "VR_BOX_MAP=0" > $O/variants_512x8_caps.log 2>&1 || exit 1
grep -v "round\|amdgpu.ids" $O/variants_512x8_caps.log
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $O/tcc -o p -- python tools/bench_variants.py --config 512x8 --cameras C0 --method 1 --rounds 2 --reps 2 --env "VR_DUO=0" "" "VR_WG_PER_CU=3" > $O/pmc_tcc.log 2>&1 || { tail -20 $O/pmc_tcc.log; exit 1; }
python - <<'PY' > $O/tcc_summary.log
import csv, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/r4aa/tcc/p_counter_collection.csv")):
    if "vr::k_march" in r["Kernel_Name"] and int(r["Grid_Size"]) == 2073600:
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k[0][:50]:50s} {k[1]:14s} mean {sum(v) / len(v):14.0f} over {len(v)}")
PY
cat $O/tcc_summary.log
echo done
