"""Frame-loop timing variants of the bench's timed region (tooling): per-step
frame zeroing and per-render events vs a plain loop of renders (runSingleTest,
C:1049-1063, clears the output once, C:1022)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import __graft_entry__ as g
import bench

pkg = g.load_package()
baked = "--baked" in sys.argv
n, nb, W, H = bench.CONFIGS["1024x8"]
pkg.synthesize((n, n, n), nb, bench.SEED)
if baked:
    pkg.bake_stats()
s = torch.cuda.Stream()
pkg.set_stream(s)
frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
d = pkg.make_desc(frame, W, H, pkg.camera.single_test_inv_view(), query_method=1)
K = 40
with torch.cuda.stream(s):
    for _ in range(5):
        pkg.render(d)
torch.cuda.synchronize()
res = {}
for mode in ("zero+events", "events", "plain", "zero+events", "events", "plain"):
    with torch.cuda.stream(s):
        ev = []
        torch.cuda.synchronize()
        a0 = torch.cuda.Event(enable_timing=True); a1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a0.record(s)
        for _ in range(K):
            if mode.startswith("zero"):
                frame.zero_()
            if "events" in mode:
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
            pkg.render(d)
            if "events" in mode:
                e1.record(s)
                ev.append((e0, e1))
        a1.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K * 1e3
    kern = float(np.mean([x.elapsed_time(y) for x, y in ev])) if ev else None
    res.setdefault(mode, []).append({"wall_ms": round(wall, 4), "span_ms": round(a0.elapsed_time(a1) / K, 4),
                                      "kernel_ms": round(kern, 4) if kern else None})
print(json.dumps({"baked": baked, "kernel": pkg.last_kernel(), **res}))
