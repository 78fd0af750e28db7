#!/usr/bin/env python3
"""A/B timing of libvr tuning builds in ONE process, interleaved rounds (tooling).

Every variant library (tools/build/variants/*/libvr.so, plus the in-tree build
as 'main') adopts the same device volume; each (variant, env) configuration is
timed with HIP events, rounds interleaved, median and min reported.

  python tools/bench_variants.py --config 1024x8 --rounds 5 [--env VR_BOX_MAX=0 ...]
"""
import argparse
import ctypes
import glob
import itertools
import re
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cameras", default="C0,C1")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--variants", default="")
    ap.add_argument("--codec", action="store_true",
                    help="synthesize a codec volume (methods 4/5/6; the in-tree build only)")
    ap.add_argument("--baked", action="store_true",
                    help="bake the statistics planes (basicDataProcessing) before timing")
    ap.add_argument("--pads", nargs="*", default=[""],
                    help="VR_PAD layouts to synthesize in turn, e.g. '' '4,0' '4,64'")
    ap.add_argument("--env", nargs="*", default=[""],
                    help="tuning knobs (vr_set_tuning) to sweep, e.g. 'VR_BOX_MAX=0' 'VR_WG_PER_CU=4,VR_BOX_MAX=0'")
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    if args.config in bench.CONFIGS:
        n, nb, W, H = bench.CONFIGS[args.config]
    else:  # ad-hoc shape for sweeps: N x B @ W x H, e.g. 256x8@512x512
        vol, img = args.config.split("@")
        n, nb = (int(v) for v in vol.split("x"))
        W, H = (int(v) for v in img.split("x"))
    paths = {"main": pkg.LIB_PATH}
    for p in sorted(glob.glob(os.path.join(ROOT, "tools/build/variants/*/libvr.so"))):
        paths[os.path.basename(os.path.dirname(p))] = p
    if args.codec:
        args.variants = "main"
    if args.variants:
        keep = set(args.variants.split(","))
        paths = {k: v for k, v in paths.items() if k in keep}
    libs = {}
    for name, p in paths.items():
        L = ctypes.CDLL(p)
        L.vr_render.argtypes = [ctypes.POINTER(pkg._lib.RenderDesc)]
        L.vr_init_distribution.argtypes = [ctypes.c_void_p, pkg._lib.Extent, ctypes.c_int,
                                           ctypes.c_int]
        L.vr_synthesize.argtypes = [pkg._lib.Extent, ctypes.c_int, ctypes.c_uint64]
        L.vr_volume_info.argtypes = [ctypes.POINTER(pkg._lib.Extent),
                                     ctypes.POINTER(ctypes.c_int),
                                     ctypes.POINTER(ctypes.c_void_p)]
        L.vr_last_error.restype = ctypes.c_char_p
        L.vr_last_kernel.restype = ctypes.c_char_p
        L.vr_set_tuning.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        libs[name] = L
    torch.cuda.set_device(0)
    for pad in args.pads:
        run_pad(args, pkg, libs, pad, n, nb, W, H, torch, bench)


def run_pad(args, pkg, libs, pad, n, nb, W, H, torch, bench):
    first = next(iter(libs.values()))
    ext = pkg._lib.Extent(n, n, n)
    if args.codec:  # the package's own library instance is "main"
        pkg.synthesize_codec((n, n, n), nb, bench.CODEC_TEMPLATES, bench.CODEC_SLOTS, bench.SEED)
        return run_timed(args, pkg, libs, pad, n, nb, W, H, torch, bench)
    first.vr_set_tuning(b"VR_PAD", pad.encode() if pad else None)
    assert first.vr_synthesize(ext, nb, bench.SEED) == 0
    first.vr_set_tuning(b"VR_PAD", None)
    ptr = ctypes.c_void_p()
    first.vr_volume_info(None, None, ctypes.byref(ptr))
    for L in list(libs.values())[1:]:  # other variants adopt the same (dense) volume
        assert L.vr_init_distribution(ptr, ext, nb, 2) == 0
    if args.baked:
        for L in libs.values():
            assert L.vr_bake_stats() == 0, L.vr_last_error()
    return run_timed(args, pkg, libs, pad, n, nb, W, H, torch, bench)


def run_timed(args, pkg, libs, pad, n, nb, W, H, torch, bench):
    if args.codec and args.baked:
        for L in libs.values():
            assert L.vr_bake_stats() == 0, L.vr_last_error()
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    cams = {c: bench.camera_matrix(pkg, c) for c in ("C0", "C1", "S")}
    cams["T"] = pkg.camera.display_inv_view((90.0, 90.0))  # top view: screen x along y
    descs = {c: pkg.make_desc(out, W, H, cams[c], query_method=args.method,
                              volume_size=(n, n, n)) for c in args.cameras.split(",")}
    envs = []
    for e in args.env:
        d = {}
        for kv in filter(None, re.split(r",(?=[A-Z_]+=)", e)):
            k, v = kv.split("=")
            d[k] = v
        envs.append(d)
    configs = list(itertools.product(libs.keys(), envs, descs.keys()))
    times = {i: [] for i in range(len(configs))}
    kern = {}
    for rnd in range(args.rounds):
        for i, (name, env, cam) in enumerate(configs):
            L = libs[name]
            L.vr_clear_tuning()
            for k, v in env.items():  # knobs (vr_set_tuning): the library reads no environment
                L.vr_set_tuning(k.encode(), v.encode())
            d = descs[cam]
            # two untimed frames: a changed env re-keys the frame order, whose first
            # frame records tile costs and whose second re-deals by them (host sync)
            for _ in range(2):
                assert L.vr_render(ctypes.byref(d)) == 0, L.vr_last_error()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            bad = 0
            for _ in range(args.reps):
                bad += L.vr_render(ctypes.byref(d)) != 0
            e1.record()
            torch.cuda.synchronize()
            # a launch failing only under some env setting must not be logged as fast
            assert bad == 0, f"{name} {env}: {bad} failed renders: {L.vr_last_error()}"
            assert L.vr_render(ctypes.byref(d)) == 0, L.vr_last_error()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / args.reps)
            kern[i] = L.vr_last_kernel().decode()
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    for L in libs.values():
        L.vr_clear_tuning()
    print(f"config {args.config} method {args.method} pad '{pad}'"
          + (" baked" if args.baked else ""))
    for i, (name, env, cam) in enumerate(configs):
        t = np.array(times[i])
        envs_s = ",".join(f"{k}={v}" for k, v in env.items()) or "-"
        print(f"{name:10s} {envs_s:34s} {cam}  median {np.median(t):7.3f} ms  min {t.min():7.3f}"
              f"  ({W * H / np.median(t) / 1e3:8.1f} Mrays/s)  {kern[i]}")


if __name__ == "__main__":
    main()
