#!/usr/bin/env python3
"""Render a few frames of one view under given tuning knobs (tooling).

For PMC passes of a variant (rocprofv3 --pmc ... -- python tools/pmc_frames.py
...): the frames run with the knobs set through vr_set_tuning; the last one is
compared bit for bit with a frame of the default dispatch (the default's
parity with the oracle is what the GPU tests and bench lines check).

  python tools/pmc_frames.py --config 512x8 --camera C0 --method 1 --tune VR_DUO=0 --frames 3
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="512x8")
    ap.add_argument("--camera", default="C0")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--tune", nargs="*", default=[])
    ap.add_argument("--frames", type=int, default=3)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    pkg.synthesize((n, n, n), nb, bench.SEED)
    m = bench.camera_matrix(pkg, args.camera)
    ref = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.render(pkg.make_desc(ref, W, H, m, query_method=args.method))
    base_kernel = pkg.last_kernel()
    for kv in args.tune:
        k, v = kv.split("=")
        pkg.set_tuning(k, v)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    d = pkg.make_desc(out, W, H, m, query_method=args.method)
    for _ in range(args.frames):
        out.zero_()
        pkg.render(d)
    torch.cuda.synchronize()
    same = bool(torch.equal(out, ref))
    print(f"default {base_kernel}  tuned {pkg.last_kernel()} {args.tune}  "
          f"frame identical to the default: {same}", flush=True)
    if not same:
        diff = int((out != ref).sum())
        print(f"MISMATCH: {diff} pixels differ", flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()
