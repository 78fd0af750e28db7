"""Per-frame kernel time over a long run of frames (tooling): how many frames the
GPU takes to reach its steady frame time (clock / translation warm-up)."""
import os, sys, json
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
torch.cuda.synchronize()
ev = []
with torch.cuda.stream(s):
    for _ in range(300):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s); pkg.render(d); e1.record(s); ev.append((e0, e1))
torch.cuda.synchronize()
t = np.array([a.elapsed_time(b) for a, b in ev])
print(json.dumps({"baked": baked, "first10": [round(x, 3) for x in t[:10]],
                  "mean_by_20": [round(float(t[i:i + 20].mean()), 4) for i in range(0, 300, 20)]}))
