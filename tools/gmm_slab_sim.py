"""BASELINE config 5 on one GPU: the z-slab chain of an N-rank run, slab by slab.

Each slab's slices (+ halo) of the synthetic GMM volume are generated in HBM
(the previous slab is released first: a 2048^3 x 16 slab is 207 GB), the
previous slab's alive rays stay in HBM, and the slab's march is timed with HIP
events on the library stream.  Per slab: kernel ms, rays in / out, and the
alive-list bytes an N-rank run sends to the next rank over xGMI.  The frame
assembled from all slabs is the N-rank frame; --check also renders the whole
volume (when it fits) and requires bit-identical frames.
usage: python tools/gmm_slab_sim.py [--dim 2048] [--K 16] [--W 3840 --H 2160] [--slabs 8]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=2048)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--slabs", type=int, default=8)
    ap.add_argument("--camera", default="C0", choices=["C0", "C1"])
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--balance", action="store_true",
                    help="after the equal slabs, re-cut them by the measured per-slab cost "
                         "(slabs.bounds_by_cost, capped at this GPU's HBM) and run again")
    a = ap.parse_args()
    import numpy as np
    import torch
    pkg = g.load_package()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    pkg.set_stream(s)
    n, K, W, H = a.dim, a.K, a.W, a.H
    m = pkg.camera.single_test_inv_view() if a.camera == "C0" else pkg.camera.display_inv_view()
    direction = pkg.slabs.march_direction(m, W, H)
    bounds = pkg.slabs.slab_bounds(n, a.slabs, direction)
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    desc = pkg.make_desc(frame, W, H, m, query_method=a.method, volume_size=(1, 1, 1))
    rays = [torch.zeros((W * H, pkg.slabs.RAY_WORDS), dtype=torch.int32, device="cuda") for _ in range(2)]
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    rows = run_chain(a, pkg, torch, np, s, bounds, n, K, W, H, desc, rays, cnt, frame, "equal")
    if a.balance:
        pkg.free_gmm()
        free, _ = torch.cuda.mem_get_info()
        cap = pkg.slabs.max_slices_for(n, n, K, free)
        nb = pkg.slabs.bounds_by_cost(n, a.slabs, direction, bounds,
                                      [r["kernel_ms"] for r in rows], cap)
        print(json.dumps({"balanced_bounds": nb, "max_slices": cap}), flush=True)
        frame.zero_()
        run_chain(a, pkg, torch, np, s, nb, n, K, W, H, desc, rays, cnt, frame, "cost-balanced")
    if a.check:
        got = frame.clone()
        pkg.synthesize_gmm((n, n, n), K, 20261015)
        frame.zero_()
        with torch.cuda.stream(s):
            pkg.render_gmm(desc)
        torch.cuda.synchronize()
        same = torch.equal(got, frame)
        print(json.dumps({"check_whole_volume_identical": bool(same)}), flush=True)
        if not same:
            sys.exit(1)


def run_chain(a, pkg, torch, np, s, bounds, n, K, W, H, desc, rays, cnt, frame, label):
    n_in, rows = 0, []
    for i, (z_lo, z_hi) in enumerate(bounds):
        zb, ns = pkg.slabs.resident_slices(z_lo, z_hi, n)
        t0 = time.time()
        pkg.synthesize_gmm((n, n, n), K, 20261015, z_base=zb, nslices=ns)
        t_syn = time.time() - t0
        rin, rout = (rays[(i + 1) % 2], rays[i % 2])
        ms = []
        with torch.cuda.stream(s):
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                pkg.render_gmm(desc, pkg.gmm_slab(z_lo, z_hi, rout, cnt,
                                                  d_rays_in=rin if i else None, n_rays_in=n_in))
                e1.record(s)
                e1.synchronize()
                ms.append(e0.elapsed_time(e1))
        n_out = int(cnt.item())
        r = {"slabs": label, "slab": i, "z": [z_lo, z_hi], "resident_GB": round(n * n * ns * 12 * K / 1e9, 1),
             "synth_s": round(t_syn, 2), "kernel_ms": round(float(np.median(ms)), 4),
             "kernel_ms_min": round(float(min(ms)), 4), "rays_in": n_in if i else W * H,
             "rays_out": n_out, "handoff_MB": round(n_out * 48 / 1e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
        n_in = n_out
    assert n_in == 0, "the last slab must end every ray"
    tot = sum(r["kernel_ms"] for r in rows)
    mx = max(r["kernel_ms"] for r in rows)
    print(json.dumps({"summary": f"{n}^3 x {K} GMM, {W}x{H}, {a.camera} m{a.method}, "
                                 f"{a.slabs} {label} slabs",
                      "sum_kernel_ms": round(tot, 3), "max_kernel_ms": round(mx, 3),
                      "one_gpu_out_of_core_Mrays_s_excl_streaming": round(W * H / tot / 1e3, 1),
                      "pipelined_ranks_Mrays_s_upper": round(W * H / mx / 1e3, 1),
                      "max_handoff_MB": max(r["handoff_MB"] for r in rows)}), flush=True)
    return rows


if __name__ == "__main__":
    main()
