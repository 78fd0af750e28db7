#!/usr/bin/env python3
"""Per-rank HBM traffic of an N-rank bench.py split, for its N > 1 line (tooling).

bench.py at N > 1 deals the tiles by measured cost (balanced_lists); the
integer cost sums make that deal reproducible in ONE process on one GPU
(bench.emulated_rank_lists).  `run` builds the bench's volume, derives the
lists of a `--world` split, and renders every rank's list `--reps` times in
rank order under the caller's `rocprofv3 --pmc` pass; `fold` reads the passes
(FETCH_SIZE, WRITE_SIZE: one process each), takes the last world x reps march
dispatches in dispatch order (the balancing renders come first), and writes
the traffic.json entry bench.py looks up: key "<config>|<camera>|m<method>|N<world>",
per_rank_hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE per launch of each rank's
list (tools/pmc_traffic.py's gfx950 correction), with the build's sha16 and
the lists' sha16 -- bench.py uses it only for that same build and deal.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/f -o f -- \
      python tools/rank_traffic.py run --world 8 > D/run.json
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/w -o w -- \
      python tools/rank_traffic.py run --world 8
  python tools/rank_traffic.py fold OUT.json D/run.json D/f D/w
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[a.config]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    pkg.set_stream(stream)
    pkg.synthesize((n, n, n), nb, bench.SEED)
    m = bench.camera_matrix(pkg, a.camera)
    lists = bench.emulated_rank_lists(pkg, torch, a.world, W, H, m, a.method, dev, stream)
    n_slots = lists.shape[1]
    kernels = []
    with torch.cuda.stream(stream):
        buf = torch.zeros(n_slots * 256, dtype=torch.int32, device=dev)
        for r in range(a.world):
            tl = torch.from_numpy(lists[r].view(np.int32).copy()).to(dev)
            d = pkg.make_desc(buf, W, H, m, query_method=a.method, d_tile_list=tl, n_tiles=n_slots)
            for _ in range(a.reps):
                pkg.render(d)
            torch.cuda.synchronize()
            kernels.append(pkg.last_kernel())
    print(json.dumps({"config": a.config, "camera": a.camera, "method": a.method,
                      "world": a.world, "reps": a.reps, "lists_sha16": bench.lists_sha16(lists),
                      "kernels": kernels, "lib_sha16": bench.lib_sha16(pkg.LIB_PATH)}), flush=True)


def march_dispatches(d):
    """(dispatch id, counter value) of the march launches of a pass, in order"""
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "vr::k_march" in r["Kernel_Name"]:
                rows[int(r["Dispatch_Id"])] = rows.get(int(r["Dispatch_Id"]), 0.0) + float(
                    r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def fold(a):
    meta = json.loads([ln for ln in open(a.run_json) if ln.startswith("{")][-1])
    world, reps = meta["world"], meta["reps"]
    fetch, write = march_dispatches(a.fetch_dir), march_dispatches(a.write_dir)
    need = world * reps
    if len(fetch) < need or len(write) < need:
        raise SystemExit(f"{len(fetch)} / {len(write)} march dispatches, need {need}")
    fetch, write = fetch[-need:], write[-need:]
    per_rank = []
    for r in range(world):
        # a rank's later renders (its own list again, as in the bench's frame
        # loop); the first follows the previous rank's list
        lo = r * reps + (1 if reps > 1 else 0)
        f = float(np.mean(fetch[lo:(r + 1) * reps]))
        w = float(np.mean(write[lo:(r + 1) * reps]))
        per_rank.append(int((2.0 * f + w) * 1024))  # KiB -> bytes, 2 x FETCH_SIZE + WRITE_SIZE
    key = f"{meta['config']}|{meta['camera']}|m{meta['method']}|N{world}"
    entry = {"kernel": meta["kernels"][0], "kernels": meta["kernels"],
             "lib_sha16": meta["lib_sha16"], "lists_sha16": meta["lists_sha16"],
             "per_rank_hbm_bytes": per_rank, "reps": reps,
             "measured": os.environ.get("PMC_TAG", "")}
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    db[key] = entry
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
    print(json.dumps({key: entry}))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--config", default="1024x8")
    r.add_argument("--camera", default="C0")
    r.add_argument("--method", type=int, default=1)
    r.add_argument("--world", type=int, required=True)
    r.add_argument("--reps", type=int, default=4)
    f = sub.add_parser("fold")
    f.add_argument("out")
    f.add_argument("run_json")
    f.add_argument("fetch_dir")
    f.add_argument("write_dir")
    a = ap.parse_args()
    run(a) if a.cmd == "run" else fold(a)


if __name__ == "__main__":
    main()
