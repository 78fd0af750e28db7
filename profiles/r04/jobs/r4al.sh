#!/bin/bash
# round 4, job al: kernel trace of rank 0's N = 8 frame loop on two render streams --
# consecutive renders overlap (start of frame f+1 before the end of frame f)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4al; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o k -- python tools/host_cost.py --world 8 --camera C0 --streams-only --frames 100 > $O/host_cost.log 2>&1 || { tail -20 $O/host_cost.log; exit 1; }
python - <<'PY' | tee $O/overlap_trace.log
import csv, glob
rows = [r for r in csv.DictReader(open(glob.glob("gpurun_out/r4al/kt/*kernel_trace.csv")[0]))
        if "k_march_seg_head" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# runs of consecutive renders; a gap > 1 ms separates the loop variants
runs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 1_000_000:
        runs.append(cur); cur = []
    cur.append(b)
runs.append(cur)
for i, run in enumerate(runs):
    if len(run) < 50:
        continue
    ov = [int(a["End_Timestamp"]) - int(b["Start_Timestamp"]) for a, b in zip(run, run[1:])]
    n_ov = sum(1 for x in ov if x > 0)
    dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in run) / len(run) / 1e6
    span = (int(run[-1]["End_Timestamp"]) - int(run[0]["Start_Timestamp"])) / (len(run) - 1) / 1e6
    print(f"run {i}: {len(run)} renders, mean kernel {dur:.4f} ms, period {span:.4f} ms, "
          f"{n_ov} of {len(ov)} start before the previous one ends "
          f"(mean overlap {sum(x for x in ov if x > 0) / max(n_ov, 1) / 1e6:.4f} ms)")
PY
echo done
