"""Parity margin against the readings the reference leaves open (CPU, tooling).

The oracle fixes one canonical reading of arithmetic the reference does not pin
(DESIGN.md section 3): texture filter weights rounded to 8 fractional bits,
rsqrtf as the correctly rounded 1/sqrtf, the float log as (float)log((double)x).
Real NVIDIA output may differ in any of them.  This renders the BASELINE
configs with each alternative reading (oracle/vr_oracle.c orc_set_reading) and
compares the frames with the canonical oracle frame: how far the 1e-4 bar and
the bit-identical RGBA8 claim would move if the hardware read it that way.

Variants: weights truncated instead of rounded (K:601/619/683); rsqrtf +-1,
+-2 ulp (helper_math normalize, K:295); per-bin logf +-1 ulp (entropy, K:766,
method 3 only).

  python tools/parity_margin.py [--configs 128x1,256x4,512x8,1024x8] [--stride 4]
      [--json profiles/r04/parity_margin.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = {"128x1": (128, 1, 256, 256), "256x4": (256, 4, 512, 512),
         "512x8": (512, 8, 1920, 1080), "1024x8": (1024, 8, 1920, 1080)}
VARIANTS = {  # name: (w_trunc, rsqrt_ulps, log_ulps), methods it applies to
    "weights truncated": ((1, 0, 0), (1, 3)),
    "rsqrtf +1 ulp": ((0, 1, 0), (1, 3)),
    "rsqrtf -1 ulp": ((0, -1, 0), (1, 3)),
    "rsqrtf +2 ulp": ((0, 2, 0), (1,)),
    "rsqrtf -2 ulp": ((0, -2, 0), (1,)),
    "logf +1 ulp": ((0, 0, 1), (3,)),
    "logf -1 ulp": ((0, 0, -1), (3,)),
}


def camera(cam):
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "vr_camera", os.path.join(ROOT, "volume-rendering-based-on-distribution-data_amd",
                                  "camera.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.single_test_inv_view() if cam == "C0" else mod.display_inv_view((30.0, 45.0))


def compare(ref, got):
    r8, rf, rn = ref
    g8, gf, gn = got
    hit = rn >= 0
    d = np.abs(gf - rf)
    byte = np.abs(g8.view(np.uint8).astype(np.int16) - r8.view(np.uint8).astype(np.int16))
    return {
        "pixels": int(r8.size), "hit": int(hit.sum()),
        "rgba8_mismatch": int(np.sum(g8 != r8)),
        "max_byte_diff": int(byte.max()) if byte.size else 0,
        "max_abs": float(d.max()) if d.size else 0.0,
        "over_1e-4": int(np.sum(np.any(d > 1e-4, axis=-1))),
        "steps_mismatch": int(np.sum(gn != rn)),
    }


def run(orc, cfg, stride, cams, threads, log=print):
    n, nb, W, H = SIZES[cfg]
    t0 = time.perf_counter()
    vol = orc.synth_volume(n, n, n, nb, 20261015, threads)
    log(f"{cfg}: volume {n}^3 x {nb} synthesized in {time.perf_counter() - t0:.1f} s", flush=True)
    rows = []
    for cam in cams:
        m = camera(cam)
        for method in (1, 3):
            p = orc.make_params(W, H, m, query_method=method)
            orc.set_reading()
            ref = orc.render(vol, p, row_stride=stride, nthreads=threads, want_float=True,
                             want_steps=True)[:3]
            for name, (rd, methods) in VARIANTS.items():
                if method not in methods:
                    continue
                orc.set_reading(*rd)
                got = orc.render(vol, p, row_stride=stride, nthreads=threads, want_float=True,
                                 want_steps=True)[:3]
                orc.set_reading()
                sel = slice(0, None, stride)
                c = compare(tuple(a[sel] for a in ref), tuple(a[sel] for a in got))
                c.update(config=cfg, camera=cam, method=method, variant=name, row_stride=stride)
                rows.append(c)
                log(f"  {cam} m{method} {name:18s}: rgba8 {c['rgba8_mismatch']:7d} / {c['hit']:7d} hit"
                    f"  max byte {c['max_byte_diff']:3d}  max|d| {c['max_abs']:.3e}"
                    f"  >1e-4 {c['over_1e-4']:7d}  steps {c['steps_mismatch']:6d}", flush=True)
    del vol
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="128x1,256x4,512x8,1024x8")
    ap.add_argument("--cameras", default="C0,C1")
    ap.add_argument("--stride", type=int, default=4, help="row stride at 1080p (1 below)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import __graft_entry__ as g
    orc = g.load_oracle()
    out = []
    for cfg in args.configs.split(","):
        stride = args.stride if SIZES[cfg][3] >= 1080 else 1
        out += run(orc, cfg, stride, args.cameras.split(","), args.threads)
    if args.json:
        os.makedirs(os.path.dirname(args.json), exist_ok=True)
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
