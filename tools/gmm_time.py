"""Time the GMM march (config-5 record type) on one GPU: whole-volume renders of a
synthetic K-component GMM volume, HIP events on the library stream, algorithmic
bytes from the footprint count (U x 8K for the mean, U x 12K for the variance).
usage: python tools/gmm_time.py [--dim 512] [--K 16] [--W 1920 --H 1080]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--methods", default="1,2")
    ap.add_argument("--cams", default="C0,C1")
    a = ap.parse_args()
    import torch
    pkg = g.load_package()
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    pkg.set_stream(s)
    t0 = time.time()
    pkg.synthesize_gmm((a.dim,) * 3, a.K)
    print(f"synth {a.dim}^3 x K{a.K}: {time.time() - t0:.1f} s", flush=True)
    out = torch.zeros(a.W * a.H, dtype=torch.int32, device="cuda")
    for cam in a.cams.split(","):
        m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
        for method in (int(x) for x in a.methods.split(",")):
            d = pkg.make_desc(out, a.W, a.H, m, query_method=method, volume_size=(1, 1, 1))
            with torch.cuda.stream(s):
                for _ in range(2):
                    pkg.render_gmm(d)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    pkg.render_gmm(d)
                e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            u = pkg.gmm_count_footprint(d)
            alg = u * (8 if method == 1 else 12) * a.K + a.W * a.H * 4
            print(f"{cam} m{method}: {ms:.3f} ms  {a.W * a.H / ms / 1e3:.1f} Mrays/s  U={u}  "
                  f"alg {alg / 1e9:.2f} GB  {alg / ms / 1e6:.0f} GB/s ({alg / ms / 8e9:.3f} of 8 TB/s)"
                  f"  {pkg.last_kernel()}", flush=True)


if __name__ == "__main__":
    main()
