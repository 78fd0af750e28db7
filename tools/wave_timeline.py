"""Wave occupancy timeline of the per-ray pipelined and quad marches (tooling).

Runs a full frame and the tile lists of a multi-GPU split (each rank's list
rendered alone, as tools/rank_sim.py does) with vr_debug_wave_clock on, and
prints for each launch: span, live waves over time (per XCD), when the live
count falls below 90 / 50 / 10 % of its peak, and wave-duration statistics.

  python tools/wave_timeline.py [--camera C0] [--world 8] [--ranks 0,1] [--env VR_PATH=2] [--cost]

--cost deals the rank lists by the measured per-tile costs of a full frame
(tiles.tile_lists_by_cost, what bench.py uses at N > 1) instead of the estimate.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(name, clk, hits, ms=None):
    """clk: (n_waves, 3) uint64 {start, end, smid}; hits: mask of waves that ran"""
    c = clk[hits]
    t0, t1 = c[:, 0].astype(np.int64), c[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0   # 100 MHz -> us
    span = e.max()
    sm = c[:, 2].astype(np.int64)
    xcc = sm >> 7 if len(np.unique(sm >> 7)) == 8 else sm >> 6
    bins = np.arange(0.0, span + 1.0, 1.0)
    live = np.zeros(len(bins))
    for a, b in zip(s, e):
        i0, i1 = int(a), int(b)
        live[i0:i1 + 1] += 1
    peak = live.max()
    def first_below(fr):
        idx = np.nonzero(live >= fr * peak)[0]
        return bins[idx[-1]] if len(idx) else 0.0
    dur = e - s
    print(f"{name}: event ms {ms:.3f}" if ms else name)
    print(f"   waves {len(c)}  span {span:.1f} us  peak live {peak:.0f}  "
          f"mean live {live.mean():.0f} ({live.mean() / peak:.0%})")
    print(f"   last time >=90% peak {first_below(0.9):.1f} us, >=50% {first_below(0.5):.1f}, "
          f">=10% {first_below(0.1):.1f}")
    print(f"   wave us: mean {dur.mean():.1f}  p50 {np.median(dur):.1f}  p99 "
          f"{np.percentile(dur, 99):.1f}  max {dur.max():.1f};  first start spread "
          f"{np.sort(s)[min(len(s) - 1, 2047)]:.1f} us for the first 2048 waves")
    fin = [e[xcc == x].max() for x in np.unique(xcc)]
    print("   per-XCD end us " + " ".join(f"{f:.0f}" for f in fin) +
          "   per-XCD waves " + " ".join(str(int((xcc == x).sum())) for x in np.unique(xcc)))
    # live-wave profile in 10 % slices of the span
    sl = [live[(bins >= span * k / 10) & (bins < span * (k + 1) / 10)].mean() for k in range(10)]
    print("   live by tenth of span: " + " ".join(f"{v:.0f}" for v in sl))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--camera", default="C0")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--env", default="VR_PATH=2",
                    help="tuning knobs NAME=VALUE[,NAME=VALUE] (vr_set_tuning)")
    ap.add_argument("--cost", action="store_true", help="cost-dealt rank lists")
    ap.add_argument("--baked", action="store_true", help="bake the statistics planes first")
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    for kv in filter(None, args.env.split(",")):
        k, v = kv.split("=")
        pkg.set_tuning(k, v)
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    if args.baked:
        pkg.bake_stats()
    m = (pkg.camera.single_test_inv_view() if args.camera == "C0"
         else pkg.camera.display_inv_view((30.0, 45.0)))
    steps = torch.zeros(W * H, dtype=torch.int32, device="cuda")

    def run(desc, nslots, name):
        buf = torch.zeros(nslots * 48, dtype=torch.int64, device="cuda")  # <= 16 waves per slot
        pkg.render(desc)
        torch.cuda.synchronize()
        pkg.debug_wave_clock(buf)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pkg.render(desc)
        e1.record()
        torch.cuda.synchronize()
        pkg.debug_wave_clock(None)
        clk = buf.view(-1, 3).cpu().numpy().view(np.uint64)
        analyse(f"{name} [{pkg.last_kernel()}]", clk, clk[:, 1] != 0, e0.elapsed_time(e1))

    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    tx, ty = pkg.tiles.tiles_x(W), pkg.tiles.tiles_y(H)
    run(pkg.make_desc(full, W, H, m), tx * ty, f"{args.config} {args.camera} full frame")
    if args.cost:
        st = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
        pkg.render(pkg.make_desc(full, W, H, m, d_steps=st))
        torch.cuda.synchronize()
        cost = pkg.tiles.tile_costs_from_frame(st.cpu().numpy(), W, H)
        lists = pkg.tiles.tile_lists_by_cost(W, H, args.world, cost)
    else:
        lists = pkg.tiles.tile_lists(W, H, args.world, m)
    slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in (int(x) for x in args.ranks.split(",")):
        pk = torch.zeros(slots * 256, dtype=torch.int32, device="cuda")
        d = pkg.make_desc(pk, W, H, m, d_tile_list=dl[r], n_tiles=slots)
        run(d, slots, f"N={args.world} rank {r}")
    del steps


if __name__ == "__main__":
    main()
