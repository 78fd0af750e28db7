#!/usr/bin/env python3
"""LDS-box bound check of the staged marches (tooling).

Run against a -DVR_BOX_CHECK build of libvr.so (tools/build_variants.sh
boxcheck:-DVR_BOX_CHECK; VRDD_LIB points the package at it): every frame of
k_march (VR_DUO=0) and k_march_duo (VR_DUO=2/3/4 samples per box), methods 1-3,
is rendered with the library's violation counters on (vr_debug_box_check) and
compared with the default dispatch's frame of the same view.  A violating read
is counted and skipped by the checking build, never performed.  Also printed:
the box voxels and lane slots the frame decoded, as multiples of U (the
distinct voxels under the footprints, vr_count_footprint).

  VRDD_LIB=tools/build/variants/boxcheck/libvr.so python tools/box_check.py
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="512x8:C0,512x8:C1,256x4:C0,1024x8:C0")
    ap.add_argument("--methods", default="1,2,3")
    ap.add_argument("--duos", default="0,2,3,4",
                    help="VR_DUO values; a value NAME=V,... sets those knobs instead")
    ap.add_argument("--any-build", action="store_true",
                    help="also run on a default build (frames compared, nothing counted)")
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    L = pkg._lib.load()
    ctr = torch.zeros(6, dtype=torch.int64, device="cuda")
    checking = L.vr_debug_box_check(ctypes.c_void_p(ctr.data_ptr()))
    print(f"library {pkg.LIB_PATH}: checking build {bool(checking)}", flush=True)
    if not checking and not args.any_build:
        raise SystemExit("not a -DVR_BOX_CHECK build: nothing would be counted")
    bad_total = 0
    us = {}
    for spec in args.configs.split(","):
        cfg, cam = spec.split(":")
        n, nb, W, H = bench.CONFIGS[cfg]
        pkg.synthesize((n, n, n), nb, bench.SEED)
        m = bench.camera_matrix(pkg, cam)
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        for method in (int(v) for v in args.methods.split(",")):
            pkg.clear_tuning()
            ctr.zero_()
            out.zero_()
            pkg.render(pkg.make_desc(out, W, H, m, query_method=method))
            torch.cuda.synchronize()
            ref = out.clone()
            ref_kernel = pkg.last_kernel()
            for duo in args.duos.split(","):
                pkg.clear_tuning()
                pkg.set_tuning("VR_PATH", "1")
                if "=" in duo:
                    for kv in duo.split("+"):
                        k, v = kv.split("=")
                        pkg.set_tuning(k, v)
                else:
                    pkg.set_tuning("VR_DUO", duo)
                ctr.zero_()
                out.zero_()
                pkg.render(pkg.make_desc(out, W, H, m, query_method=method))
                torch.cuda.synchronize()
                c = ctr.cpu().tolist()
                same = torch.equal(out, ref)
                ndiff = int((out != ref).sum().item())
                if ndiff:
                    import numpy as np
                    a = out.cpu().numpy().view(np.uint8).reshape(-1, 4).astype(int)
                    b = ref.cpu().numpy().view(np.uint8).reshape(-1, 4).astype(int)
                    bad = np.nonzero(np.any(a != b, axis=1))[0]
                    print(f"    differing pixels: max |dRGBA8| {np.abs(a - b).max()}, first "
                          f"{[(int(i % W), int(i // W)) for i in bad[:6]]}, rows "
                          f"{int(bad.min() // W)}-{int(bad.max() // W)}", flush=True)
                bad_total += c[0] + c[2] + (0 if same else 1)
                u = us.get((cfg, cam, method))
                if u is None:
                    u = us[(cfg, cam, method)] = pkg.count_footprint(
                        pkg.make_desc(out, W, H, m, query_method=method))
                print(f"{cfg} {cam} m{method} VR_DUO={duo} {pkg.last_kernel():28s} "
                      f"violations {c[0]} (worst over {c[1]}) boxes outside the volume {c[2]} "
                      f"frame {'identical to' if same else f'DIFFERS ({ndiff} px) from'} {ref_kernel}; "
                      f"decoded {c[3] / u:.3f} U, slots {c[4] / u:.3f} U (U = {u})",
                      flush=True)
        pkg.clear_tuning()
    L.vr_debug_box_check(None)
    print(f"total: {bad_total} violations / differing frames")
    return 1 if bad_total else 0


if __name__ == "__main__":
    sys.exit(main())
