"""Kernel-choice cliff: frame time over view rotations (tooling).

The march kernel is chosen on the view (vr_api.cpp fill_params): when the
screen x axis runs along the voxel rows (|invViewMatrix[0]| >= threshold) the
per-ray pipelined march, else the quad-cooperative march.  For the display()
camera (C:225-246) m00 = cos(ry), so a yaw sweep crosses that threshold.  For
each (rx, ry) this times the default dispatch and each candidate forced through
vr_set_tuning (VR_PATH 2 = per-ray pipelined, 0 = quad).

  python tools/rot_sweep.py [--config 1024x8] [--method 1] [--rx 0,30] [--step 5]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--rx", default="0,30")
    ap.add_argument("--step", type=float, default=5.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--paths", default="2,0", help="forced VR_PATH values to time beside the default")
    ap.add_argument("--knob", default="VR_ZROWS=0",
                    help="one more column: the default dispatch under this tuning knob")
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")

    def timed(desc):
        for _ in range(3):  # the 1st frame of a view records tile costs, the 2nd re-deals
            pkg.render(desc)
        torch.cuda.synchronize()
        ev = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pkg.render(desc)
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        return float(np.median([a.elapsed_time(b) for a, b in ev])), pkg.last_kernel()

    paths = [p for p in args.paths.split(",") if p]
    print(f"{args.config} m{args.method} {W}x{H}: median kernel ms over {args.reps} frames")
    kk, kv = args.knob.split("=") if args.knob else (None, None)
    print(f"{'rx':>4} {'ry':>5} {'m00':>6}  {'default':>8} kernel" +
          "".join(f"   VR_PATH={p:>2}" for p in paths) + (f"   {args.knob}" if kk else ""))
    for rx in (float(v) for v in args.rx.split(",")):
        for ry in np.arange(0.0, 90.0 + 1e-6, args.step):
            m = pkg.camera.display_inv_view((rx, float(ry)))
            desc = pkg.make_desc(out, W, H, m, query_method=args.method)
            pkg.clear_tuning()
            t_def, k_def = timed(desc)
            row = f"{rx:4.0f} {ry:5.1f} {m[0]:6.3f}  {t_def:8.3f} {k_def:26s}"
            for p in paths:
                pkg.set_tuning("VR_PATH", p)
                t, _ = timed(desc)
                row += f"   {t:8.3f}"
            pkg.clear_tuning()
            if kk:
                pkg.set_tuning(kk, kv)
                t, _ = timed(desc)
                row += f"   {t:8.3f}"
                pkg.clear_tuning()
            print(row, flush=True)


if __name__ == "__main__":
    main()
