"""Samples per pixel of the 1024^3 x 8 bench frames (C0, C1) -> gpurun_out/steps_<cam>.npy (tooling)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS["1024x8"]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    steps = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for cam in ("C0", "C1"):
        m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
        pkg.render(pkg.make_desc(out, W, H, m, d_steps=steps))
        torch.cuda.synchronize()
        np.save(os.path.join(ROOT, "gpurun_out", f"steps_{cam}.npy"),
                steps.cpu().numpy().reshape(H, W))


if __name__ == "__main__":
    main()
