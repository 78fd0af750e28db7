"""Out-of-core GMM frames on one GPU: host-pinned slabs streamed through HBM (tooling).

The volume (generated on the device slab by slab, copied into pinned host
memory) never sits in HBM whole: stream.GmmStream copies slab i+1 while slab i
marches.  Prints one JSON line per frame set: frame ms, Mrays/s, the
host->device GB/s the frame achieved, and the march-only ms of the same slabs
(from HIP events around each slab's launch is not separable from the copy
waits, so the in-core march of the whole volume is timed beside it when it
fits, --incore).  --check compares the streamed frame with the whole-volume
render (bit-identical).

  python tools/gmm_stream_bench.py --dim 512 --K 16 --W 3840 --H 2160 --slab 64
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as g  # noqa: E402

SEED = 20261015


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=512)
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--slab", type=int, default=64, help="slices per streamed slab")
    ap.add_argument("--camera", default="C0", choices=["C0", "C1"])
    ap.add_argument("--method", type=int, default=1, choices=[1, 2])
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--incore", action="store_true", help="also time the whole volume in HBM")
    a = ap.parse_args()
    import numpy as np
    import torch
    pkg = g.load_package()
    torch.cuda.set_device(0)
    n, K, W, H = a.dim, a.K, a.W, a.H
    hip = ctypes.CDLL("libamdhip64.so")
    # host volume, pinned: generated on the device in chunks, copied down
    t0 = time.time()
    wm = torch.empty((n, n, n, K, 2), dtype=torch.float32, pin_memory=True)
    sg = torch.empty((n, n, n, K), dtype=torch.float32, pin_memory=True)
    chunk = max(1, min(n, int(8e9 // (n * n * K * 12))))
    for zb in range(0, n, chunk):
        ns = min(chunk, n - zb)
        pkg.synthesize_gmm((n, n, n), K, SEED, z_base=zb, nslices=ns)
        _, _, _, _, pw, ps = pkg.gmm_info()
        torch.cuda.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(wm[zb].data_ptr()), ctypes.c_void_p(pw),
                             ctypes.c_size_t(ns * n * n * K * 8), 2) == 0
        assert hip.hipMemcpy(ctypes.c_void_p(sg[zb].data_ptr()), ctypes.c_void_p(ps),
                             ctypes.c_size_t(ns * n * n * K * 4), 2) == 0
    pkg.free_gmm()
    t_gen = time.time() - t0
    m = pkg.camera.single_test_inv_view() if a.camera == "C0" else pkg.camera.display_inv_view()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    desc = pkg.make_desc(frame, W, H, m, query_method=a.method, volume_size=(1, 1, 1))
    s = torch.cuda.Stream()
    st = pkg.stream.GmmStream(wm, sg, a.slab)
    info = st.render(desc, s)  # warm-up (allocates the alive lists)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.frames):
        frame.zero_()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        info = st.render(desc, s)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t1)
    t = float(np.median(ts))
    out = {"volume": [n, n, n], "K": K, "image": [W, H], "camera": a.camera, "method": a.method,
           "slab_slices": a.slab, "slabs": info["slabs"], "host_volume_GB": round(n ** 3 * K * 12 / 1e9, 2),
           "frame_ms": round(t * 1e3, 2), "Mrays_s": round(W * H / t / 1e6, 2),
           "streamed_GB": round(info["bytes_streamed"] / 1e9, 2),
           "h2d_GBps": round(info["bytes_streamed"] / t / 1e9, 1),
           "rays_handed_on": info["rays_handed_on"], "generate_s": round(t_gen, 1)}
    streamed = frame.clone()
    if a.incore or a.check:
        free, _ = torch.cuda.mem_get_info()
        if n ** 3 * K * 12 < 0.9 * free:
            pkg.init_gmm(wm.cuda(), sg.cuda(), adopt=False)
            torch.cuda.synchronize()
            pkg.set_stream(s)
            with torch.cuda.stream(s):
                frame.zero_()
                pkg.render_gmm(desc)  # warm-up
            ms = []
            for _ in range(a.frames):
                with torch.cuda.stream(s):
                    frame.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                pkg.render_gmm(desc)
                e1.record(s)
                e1.synchronize()
                ms.append(e0.elapsed_time(e1))
            out["incore_march_ms"] = round(float(np.median(ms)), 3)
            if a.check:
                out["check_identical_to_incore"] = bool(torch.equal(frame, streamed))
            pkg.free_gmm()
    print(json.dumps(out), flush=True)
    if a.check and not out.get("check_identical_to_incore", False):
        sys.exit(1)


if __name__ == "__main__":
    main()
