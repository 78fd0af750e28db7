"""Per-phase cycle breakdown of k_march_wg (tooling; needs the VR_WG_PROF variant).

  bash tools/build_variants.sh wgprof:-DVR_WG_PROF
  python tools/wg_prof.py [--config 1024x8] [--cameras C0,C1]
Counters are thread 0 of every workgroup (clock64 cycles), summed over the grid.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WS_PHASES = ["footprint+reduce", "-", "row atomics", "-", "compaction+scan", "marks+rows",
             "(E overflow)", "(rows overflow)", "(records overflow)", "load+decode",
             "blend+composite"]
PHASES = ["footprint+reduce", "B1 wait", "row atomics", "B2 wait", "compaction+scan",
          "B2b wait", "compact write", "B3 wait", "load+decode", "B4 wait", "blend+composite"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--cameras", default="C0,C1")
    ap.add_argument("--lib", default=os.path.join(ROOT, "tools/build/variants/wgprof/libvr.so"))
    args = ap.parse_args()
    os.environ["VRDD_LIB"] = args.lib
    os.environ.setdefault("VR_PATH", "3")
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    L = pkg._lib.load()
    L.vr_wg_prof_read.argtypes = [ctypes.c_void_p]
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    buf = (ctypes.c_ulonglong * 16)()
    for cam in args.cameras.split(","):
        m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
        d = pkg.make_desc(out, W, H, m, query_method=1)
        pkg.render(d)
        torch.cuda.synchronize()
        L.vr_wg_prof_read(buf)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pkg.render(d)
        e1.record()
        torch.cuda.synchronize()
        L.vr_wg_prof_read(buf)
        v = list(buf)
        steps, staged = max(v[11], 1), max(v[12], 1)
        print(f"{cam}: {e0.elapsed_time(e1):.3f} ms, kernel {pkg.last_kernel()}; workgroup-steps "
              f"{v[11]}, staged {v[12]} ({100.0 * v[12] / steps:.1f} %), rows/step "
              f"{v[13] / staged:.1f}, records/step {v[14] / staged:.1f}, "
              f"load batches/step (thread 0) {v[15] / staged:.2f}")
        ws = os.environ["VR_PATH"] == "4"
        names = WS_PHASES if ws else PHASES
        tot = sum(v[k] for k in range(11) if not (ws and 6 <= k <= 8))
        for k, name in enumerate(names):
            if ws and 6 <= k <= 8:
                print(f"   {name:18s} {v[k]} steps")
                continue
            print(f"   {name:18s} {v[k] / steps:9.1f} cycles/step  {100.0 * v[k] / max(tot, 1):5.1f} %")


if __name__ == "__main__":
    main()
