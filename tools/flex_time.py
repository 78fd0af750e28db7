"""Time the flexible-block path (methods 8/9/0) at the reference's sizes (tooling):
the dataProcessing pre-pass on a 64^3 span set with 6-voxel blocks and 64 bins
(K:1735-1796; the reference's own run took 194 s, ver1.9.6.txt:9), then a
1920x1080 frame per method at camera C0 and C1.

  python tools/flex_time.py [--reps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import __graft_entry__ as g
    pkg = g.load_package()
    orc = g.load_oracle()
    t = orc.synth_flex(64, 6, 64, ntemplates=469, seed=11, extra=0, dup=False)
    pkg.init_flex(t)
    pkg.flex_process(6)  # warm-up (module load, first-touch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        pkg.flex_process(6)
    torch.cuda.synchronize()
    print(f"dataProcessing (64^3, 6-voxel blocks, 64 bins): "
          f"{(time.perf_counter() - t0) / 5 * 1e3:.3f} ms per pre-pass (synchronous)")
    W, H = 1920, 1080
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for cam in ("C0", "C1"):
        m = (pkg.camera.single_test_inv_view() if cam == "C0"
             else pkg.camera.display_inv_view((30.0, 45.0)))
        for method in (8, 9, 0):
            d = pkg.make_desc(out, W, H, m, query_method=method, volume_size=(64, 64, 64))
            for _ in range(3):
                pkg.render(d)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                pkg.render(d)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            print(f"  {cam} method {method}: {ms:.3f} ms/frame  {W * H / ms / 1e3:.1f} Mrays/s "
                  f"({pkg.last_kernel()})")


if __name__ == "__main__":
    main()
