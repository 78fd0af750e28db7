"""Consecutive frames on one vs two alternating streams (tooling).

A frame's launch starts on an empty GPU (ramp) and ends with its last waves
(tail); on one stream the next frame's launch waits for that tail.  Frames
issued alternately on two streams (double-buffered outputs, no dependency
between consecutive frames) let the next launch start while the previous one
drains.  This times the frame period both ways -- wall clock over F frames
after a warm-up -- for the full frame (N = 1) and for the slowest rank's
cost-dealt list at N = 2 / 4 / 8, as bench.py would render them.

  python tools/overlap_sim.py --camera C0 --worlds 1,4,8
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--camera", default="C0")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--worlds", default="1,4,8")
    ap.add_argument("--frames", type=int, default=200)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    m = bench.camera_matrix(pkg, args.camera)
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    full = torch.zeros(W * H, dtype=torch.int32, device=dev)
    steps = torch.full((W * H,), -1, dtype=torch.int32, device=dev)
    pkg.render(pkg.make_desc(full, W, H, m, query_method=args.method, d_steps=steps))
    cost = pkg.tiles.tile_costs_from_frame(steps.cpu().numpy(), W, H)
    torch.cuda.synchronize()

    def period(descs, outs, nstreams, zero):
        def frame(f):
            s = streams[f % nstreams]
            pkg.set_stream(s)
            with torch.cuda.stream(s):
                if zero:
                    outs[f % 2].zero_()  # C:208
                pkg.render(descs[f % 2])
        for f in range(40):
            frame(f)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(args.frames):
            frame(f)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / args.frames

    for world in [int(w) for w in args.worlds.split(",")]:
        if world == 1:
            outs = [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(2)]
            descs = [pkg.make_desc(o, W, H, m, query_method=args.method) for o in outs]
            zero = True
            what = "full frame"
        else:
            lists = pkg.tiles.tile_lists_by_cost(W, H, world, cost)
            slots = lists.shape[1]
            # the slowest rank: its list rendered alone, one stream
            per = []
            for r in range(world):
                dl = torch.from_numpy(lists[r].view(np.int32).copy()).to(dev)
                o = [torch.zeros(slots * 256, dtype=torch.int32, device=dev) for _ in range(2)]
                d = [pkg.make_desc(x, W, H, m, query_method=args.method, d_tile_list=dl,
                                   n_tiles=slots) for x in o]
                per.append((period(d, o, 1, False), r, d, o, dl))
            _, r, descs, outs, _ = max(per, key=lambda p: p[0])
            zero = False
            what = f"N={world} rank {r} list ({slots} slots)"
        p1 = period(descs, outs, 1, zero)
        k1 = pkg.last_kernel()
        p2 = period(descs, outs, 2, zero)
        p1b = period(descs, outs, 1, zero)
        print(f"{args.config} {args.camera} m{args.method} {what} [{k1}]: one stream "
              f"{p1:.4f} / {p1b:.4f} ms per frame, two alternating streams {p2:.4f} ms "
              f"({(min(p1, p1b) - p2) / min(p1, p1b) * 100:+.1f} %)", flush=True)
    pkg.set_stream(None)


if __name__ == "__main__":
    main()
