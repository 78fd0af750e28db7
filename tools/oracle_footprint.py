#!/usr/bin/env python3
"""U of SURVEY.md 8(d) at a BASELINE config counted by the CPU oracle (tooling).

The bench's algorithmic bytes are U * S_rec + W*H*4 with U counted on the GPU by
vr_count_footprint; this counts the same U with the oracle's own march
(orc_count_footprint) on the same synthetic volume, so the headline's roofline
numerator is pinned at its own size, not only at test sizes.  Needs the volume
in host RAM (32 GiB at 1024^3 x 8).

  python tools/oracle_footprint.py --config 1024x8 --cameras C0,C1 [--threads 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--cameras", default="C0,C1")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import bench
    import __graft_entry__ as graft
    orc = graft.load_oracle()
    pkg = graft.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    t0 = time.perf_counter()
    vol = orc.synth_volume(n, n, n, nb, bench.SEED, args.threads)
    t_synth = time.perf_counter() - t0
    for cam in args.cameras.split(","):
        m = bench.camera_matrix(pkg, cam)
        t0 = time.perf_counter()
        u = orc.count_footprint(vol, orc.make_params(W, H, m, query_method=args.method),
                                args.threads)
        print(json.dumps({"config": args.config, "camera": cam, "method": args.method,
                          "U_records": u, "alg_bytes": u * nb * 4 + W * H * 4,
                          "oracle_s": round(time.perf_counter() - t0, 1),
                          "synth_s": round(t_synth, 1), "seed": bench.SEED}), flush=True)


if __name__ == "__main__":
    main()
