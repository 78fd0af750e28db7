"""bench.py end to end on the GPU: the JSON contract at N = 1, and the N > 1 tile
path (2 ranks sharing the one GPU, tile gather staged through gloo) assembling
exactly the single-rank frame."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "256x4", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]


def _run(cmd, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_single_and_two_rank_frames_agree(gpu, tmp_path):
    f1 = str(tmp_path / "f1.npy")
    out1 = _run([sys.executable, "bench.py", *ARGS, "--dump-frame", f1], tmp_path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in out1, k
    assert out1["n_gpus"] == 1 and out1["value"] > 0
    rf = out1["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["kernel"].startswith("k_march")
    # the measured read ceiling streams the whole resident 256^3 x 4 volume
    rc = rf["read_ceiling"]
    assert rc["bytes"] == 256 ** 3 * 4 * 4 and rc["GBps"] > 100 and rc["ms"] <= rc["mean_ms"]
    assert rf["frac_of_read_ceiling"] > 0 and rf["gather_bytes_per_launch"] > 0
    f2 = str(tmp_path / "f2.npy")
    # bench.py starts its own 2 ranks (no external launcher), as the driver's
    # `python bench.py --gpus N` does
    # (with the CPU baseline: at N > 1 rank 0 compares the ASSEMBLED frame with
    # the oracle's)
    args2 = [a for a in ARGS if a != "--no-cpu-baseline"]
    out2 = _run([sys.executable, "bench.py", "--gpus", "2", *args2, "--dist-backend", "gloo",
                 "--dump-frame", f2], tmp_path)
    assert out2["n_gpus"] == 2 and out2["physical_gpus"] == 1
    assert out2["rehearsal_shared_gpus"] is True and out2["scaling"] is None
    cpu = out2["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["kind"] == "port" and cpu["cores"] >= 1
    par = out2["parity"]
    assert "assembled" in par["frame"] and par["against"].startswith("oracle")
    assert par["pixels"] > 0 and par["rgba8_mismatch"] == 0
    assert par["steps_mismatch"] == 0 and par["max_abs"] <= 1e-4
    rf2 = out2["roofline"]
    agg = rf2["aggregate"]
    assert agg["ranks"] == 2 and agg["peak"] == 16000.0 and len(agg["per_rank"]) == 2
    assert sum(r["pixels"] for r in agg["per_rank"]) >= 512 * 512
    assert rf2["frac"] == agg["frac"] and 0 < agg["frac"] < 1
    assert agg["render_ms_max_over_ranks"] == max(r["render_ms"] for r in agg["per_rank"])
    assert rf2["traffic"] is None and rf2["traffic_source"]
    assert rf2["rank0"]["kernel_ms"] > 0
    # the deal the two ranks made (all_reduce of integer costs) is the one
    # tools/rank_traffic.py derives in one process for its per-rank PMC passes
    import importlib.util
    import torch
    import __graft_entry__ as g
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pkg = g.load_package()
    n, nb, W, H = bench.CONFIGS["256x4"]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    dev = torch.device("cuda", 0)
    lists = bench.emulated_rank_lists(pkg, torch, 2, W, H, bench.camera_matrix(pkg, "C0"), 1,
                                      dev, torch.cuda.current_stream())
    assert bench.lists_sha16(lists) == out2["config"]["lists_sha16"]
    pkg.freeCudaBuffers()
    a, b = np.load(f1), np.load(f2)
    assert a.shape == (512, 512) and np.count_nonzero(a) > 0
    assert np.array_equal(a, b), f"{int(np.sum(a != b))} pixels differ between N=1 and N=2"


def test_bench_gmm_single_and_two_slab_frames_agree(gpu, tmp_path):
    """GMM mode: the whole-volume frame (N = 1) equals the 2-rank z-slab chain's
    (alive rays handed rank to rank, frames summed on rank 0; gloo staging)"""
    args = ["--config", "gmm96", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    f1 = str(tmp_path / "g1.npy")
    out1 = _run([sys.executable, "bench.py", *args, "--dump-frame", f1], tmp_path)
    assert out1["n_gpus"] == 1 and out1["value"] > 0
    assert out1["roofline"]["kernel"].startswith("k_march_gmm") and 0 < out1["roofline"]["frac"] < 1
    f2 = str(tmp_path / "g2.npy")
    out2 = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", "29534",
                 "bench.py", "--gpus", "2", *args, "--dist-backend", "gloo",
                 "--dump-frame", f2], tmp_path)
    assert out2["n_gpus"] == 2 and out2["config"]["parallelism"].startswith("z-slabs x2")
    a, b = np.load(f1), np.load(f2)
    assert a.shape == (256, 256) and np.count_nonzero(a) > 0
    assert np.array_equal(a, b), f"{int(np.sum(a != b))} pixels differ between N=1 and N=2"
    # two z segments per rank (--segments 2: front + back, tick-scheduled chain),
    # ranks started by bench.py itself
    f3 = str(tmp_path / "g3.npy")
    out3 = _run([sys.executable, "bench.py", "--gpus", "2", *args, "--dist-backend", "gloo",
                 "--segments", "2", "--dump-frame", f3], tmp_path)
    assert out3["n_gpus"] == 2 and "two segments" in out3["config"]["parallelism"]
    assert len(out3["config"]["segments"]) == 4
    c = np.load(f3)
    assert np.array_equal(a, c), f"{int(np.sum(a != c))} pixels differ (two segments per rank)"


def test_bench_gmm_slab_rehearsal(gpu, tmp_path):
    """--slab-rehearsal on one GPU: every segment of the chain generated and timed
    in turn, one and two segments per rank; the line is an estimate (value
    null): the slowest rank's march plus its hand-off and reduce"""
    for seg in ("1", "2"):
        out = _run([sys.executable, "bench.py", "--config", "gmm96", "--slab-rehearsal",
                    "--rehearsal-ranks", "3", "--segments", seg, "--steps", "2", "--warmup", "1",
                    "--no-cpu-baseline"], tmp_path)
        cfg = out["config"]
        assert out["n_gpus"] == 1 and out["scaling"] is None and out["rehearsal_shared_gpus"]
        assert len(cfg["slabs_balanced"]) == 3 * int(seg)
        assert out["value"] is None and out["ms_per_step"] is None
        assert abs(out["period_march_only_ms"] - max(cfg["rank_ms"])) < 1e-3
        assert out["period_estimate_ms"] > out["period_march_only_ms"]
        assert out["period_overlapped_ms"] <= out["period_estimate_ms"]
        assert len(cfg["handoff"]) == 3 and out["estimated_Mrays_s"] > 0
        assert cfg["slabs_balanced"][0]["rays_in"] == 256 * 256
