"""Multi-GPU (RCCL over xGMI) end to end: only where >= 2 devices are visible.

bench.py with the NCCL (= RCCL) backend, one rank per GPU: the image-tile
split (tile gather to rank 0 + k_unscatter) and the GMM z-slab chain (alive
rays handed rank to rank by send/recv, frames reduced on rank 0) must assemble
exactly the single-GPU frame.  The one-GPU boxes of this pool skip it; the
gloo rehearsals of the same code paths run in test_gpu_bench.py."""
import pytest

from test_gpu_bench import _run

pytestmark = pytest.mark.gpu


def _devices():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.parametrize("args,shape", [
    (["--config", "256x4", "--camera", "C1"], (512, 512)),
    (["--config", "gmm96"], (256, 256)),
])
def test_rccl_ranks_assemble_the_single_gpu_frame(gpu, tmp_path, args, shape):
    if _devices() < 2:
        pytest.skip("needs >= 2 GPUs (RCCL ranks on distinct devices)")
    import sys
    import numpy as np
    common = args + ["--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    f1 = str(tmp_path / "n1.npy")
    out1 = _run([sys.executable, "bench.py", *common, "--dump-frame", f1], tmp_path)
    f2 = str(tmp_path / "n2.npy")
    out2 = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", "29541",
                 "bench.py", "--gpus", "2", *common, "--dump-frame", f2], tmp_path)
    assert out1["n_gpus"] == 1 and out2["n_gpus"] == 2
    a, b = np.load(f1), np.load(f2)
    assert a.shape == shape and np.count_nonzero(a) > 0
    assert np.array_equal(a, b), f"{int(np.sum(a != b))} pixels differ between 1 and 2 GPUs"
    if out2.get("parity") is not None:
        assert out2["parity"]["rgba8_mismatch"] == 0
