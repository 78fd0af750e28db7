"""Average PMC counters per dispatch of the march kernel (tooling).
usage: python tools/pmc_summary.py gpurun_out/pmc/<TAG> [kernel-substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_march<8, 1, false>"
vals = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
            per[r["Dispatch_Id"]]["_dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    for d, cs in per.items():
        for c, v in cs.items():
            vals[c].append(v)
for c, v in sorted(vals.items()):
    print(f"{c:40s} {sum(v) / len(v):14.4e}  (n={len(v)})")
