"""Per-rank render time of the multi-GPU tile split, simulated on one GPU (tooling).

For N in 1, 2, 4, 8 every rank's tile list is rendered in turn into its packed
buffer (the work one GPU does at world size N), then rank 0's unscatter of
all N buffers is timed.  max over ranks + unscatter approximates the N-GPU
frame time without the RCCL gather.

  python tools/rank_sim.py [--config 1024x8] [--camera C0] [--reps 5]
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--no-lpt", action="store_true", help="tile lists without longest-first order")
    ap.add_argument("--baked", action="store_true", help="bake the statistics planes first")
    ap.add_argument("--env", default="", help="tuning knobs NAME=VALUE[,NAME=VALUE] (vr_set_tuning) for the renders")
    ap.add_argument("--envs", nargs="*", default=None,
                    help="several knob sets (each NAME=VALUE[,...]; '' = defaults) timed in turn "
                         "on the same lists, so variants share one process and one GPU state")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--modes", default="est,cost")
    ap.add_argument("--blocks", default="1x4",
                    help="cost-dealing block shapes (tiles, WxH) to compare, e.g. 1x4,2x4,4x4")
    ap.add_argument("--host-ms", type=float, default=0.0,
                    help="per-frame host issue cost of the N > 1 frame loop (tools/host_cost.py); "
                         "reported as a second, conservative speed-up with it added")
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    if args.baked:
        pkg.bake_stats()
    def knobs(spec):
        pkg.clear_tuning()
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            pkg.set_tuning(k, v)  # tuning knobs: the library reads no environment
    knobs(args.env)
    m = (pkg.camera.single_test_inv_view() if args.camera == "C0"
         else pkg.camera.display_inv_view((0.0, 90.0) if args.camera == "S" else (30.0, 45.0)))

    def timed(fn, warm=3):
        for _ in range(warm):  # a full frame's 2nd render re-deals its tiles (adaptive order)
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
    # steady state: the clocks and address translation need ~15-20 frames of a
    # running frame loop (profiles/r02/loop_timing.log); the speedups below are
    # against this steady full frame, measured again after the rank lists
    t1 = timed(lambda: pkg.render(dfull), warm=30)
    print(f"{args.config} {args.camera} m{args.method}: steady full frame {t1:.3f} ms "
          f"({pkg.last_kernel()})")
    # latency floor: k centre-most tiles alone on the GPU
    lists1 = pkg.tiles.tile_lists(W, H, 1, m)[0]
    for k in (1, 64, 512, 1024):
        sel = torch.from_numpy(lists1[:k].view(np.int32).copy()).cuda()
        pk = torch.zeros(k * 256, dtype=torch.int32, device="cuda")
        dk = pkg.make_desc(pk, W, H, m, query_method=args.method, d_tile_list=sel, n_tiles=k)
        print(f"  {k:5d} longest tiles alone: {timed(lambda dk=dk: pkg.render(dk)):.3f} ms")
    # measured per-tile costs of this view (steps of the full frame) for the
    # cost-dealt lists (tiles.tile_lists_by_cost, what bench.py uses at N > 1)
    steps = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    pkg.render(pkg.make_desc(full, W, H, m, query_method=args.method, d_steps=steps))
    cost = pkg.tiles.tile_costs_from_frame(steps.cpu().numpy(), W, H)
    worlds = [int(w) for w in args.worlds.split(",")]
    blocks = [tuple(int(v) for v in b.split("x")) for b in args.blocks.split(",")]
    modes = [(md, w, bl) for md in args.modes.split(",") for w in worlds
             for bl in (blocks if md == "cost" else [None])]
    envs = args.envs if args.envs is not None else [args.env]
    for mode, world, bl in modes:
        if mode == "est":
            lists = pkg.tiles.tile_lists(W, H, world, None if args.no_lpt else m)
        else:
            lists = pkg.tiles.tile_lists_by_cost(W, H, world, cost, block=bl)
        slots = lists.shape[1]
        packed = torch.zeros((world, slots * 256), dtype=torch.int32, device="cuda")
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        descs = [pkg.make_desc(packed[r], W, H, m, query_method=args.method, d_tile_list=dl[r],
                               n_tiles=slots) for r in range(world)]
        for spec in envs:
            knobs(spec)
            packed.zero_()
            # two passes over the ranks, the second reported (the first pass's rank 0
            # ran right after a different launch shape)
            for _ in range(2):
                per = [timed(lambda d=d: pkg.render(d), warm=10) for d in descs]
            kern = pkg.last_kernel()
            frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            tu = timed(lambda: pkg.unscatter_tiles(packed, dl, world, slots, frame, W, H))
            torch.cuda.synchronize()
            ok = torch.equal(frame, full)
            host = (f"  + host {args.host_ms:.3f} -> {t1 / (max(per) + tu + args.host_ms):.2f}x"
                    if args.host_ms > 0 else "")
            tag = mode if bl is None or bl == (1, 4) else f"{mode} {bl[0]}x{bl[1]}"
            print(f"  {tag:4s} N={world} [{spec or 'defaults'}] {kern}: per-rank ms "
                  f"{' '.join(f'{x:.3f}' for x in per)}  max {max(per):.3f}"
                  f"  unscatter {tu:.3f}  -> est. speedup {t1 / (max(per) + tu):.2f}x{host}"
                  f"  frame {'identical' if ok else 'DIFFERS'}", flush=True)
    knobs(args.env)
    t2 = timed(lambda: pkg.render(dfull), warm=30)
    print(f"steady full frame again: {t2:.3f} ms (speedups above use {t1:.3f})")


if __name__ == "__main__":
    main()
