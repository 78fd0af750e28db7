"""Sweep the hybrid march (VR_HYB leading slots ray-segmented with VR_SEG lanes)
over the ranks of a multi-GPU tile split, each rank's list rendered alone on
one GPU as in tools/rank_sim.py (tooling).

  python tools/hyb_sweep.py [--camera C0] [--world 8] [--seg 4,8] [--hyb 0,64,128]
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
    ap.add_argument("--camera", default="C0")
    ap.add_argument("--world", default="8")
    ap.add_argument("--seg", default="4,8")
    ap.add_argument("--hyb", default="0,32,64,128,256")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--method", type=int, default=1)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    m = (pkg.camera.single_test_inv_view() if args.camera == "C0"
         else pkg.camera.display_inv_view((30.0, 45.0)))

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    dfull = pkg.make_desc(full, W, H, m, query_method=args.method)
    t1 = timed(lambda: pkg.render(dfull))
    print(f"{args.config} {args.camera} m{args.method}: full frame {t1:.3f} ms ({pkg.last_kernel()})",
          flush=True)
    for world in (int(w) for w in args.world.split(",")):
        lists = pkg.tiles.tile_lists(W, H, world, m)
        slots = lists.shape[1]
        packed = torch.zeros((world, slots * 256), dtype=torch.int32, device="cuda")
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        descs = [pkg.make_desc(packed[r], W, H, m, query_method=args.method, d_tile_list=dl[r],
                               n_tiles=slots) for r in range(world)]
        frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        for S in args.seg.split(","):
            for K in (int(k) for k in args.hyb.split(",")):
                if K == 0:
                    os.environ.pop("VR_HYB", None)
                    os.environ["VR_PATH"] = "2" if S == "pipe" else "7"
                else:
                    os.environ.pop("VR_PATH", None)
                    os.environ["VR_HYB"] = str(K)
                os.environ["VR_SEG"] = "4" if S == "pipe" else S
                packed.zero_()
                per = [timed(lambda d=d: pkg.render(d)) for d in descs]
                kern = pkg.last_kernel()
                frame.zero_()
                pkg.unscatter_tiles(packed, dl, world, slots, frame, W, H)
                torch.cuda.synchronize()
                ok = torch.equal(frame, full)
                print(f"  N={world} S={S:>4} K={K:4d} [{kern}]: per-rank "
                      f"{' '.join(f'{x:.3f}' for x in per)}  max {max(per):.3f} -> "
                      f"{t1 / max(per):.2f}x  {'identical' if ok else 'DIFFERS'}", flush=True)
                if K == 0 and S != "pipe":
                    pass
        os.environ.pop("VR_HYB", None)
        os.environ.pop("VR_PATH", None)
        os.environ.pop("VR_SEG", None)


if __name__ == "__main__":
    main()
