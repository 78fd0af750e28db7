"""bench.py's rank launcher (CPU): `python bench.py --gpus N` must start N ranks
itself when no launcher did, refuse a WORLD_SIZE that differs from --gpus, and
relay exactly rank 0's JSON line with the launcher's return code."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_plan_single_gpu_runs_in_process():
    b = _bench()
    assert b.launch_plan(1, ["--gpus", "1"], {}) == ("run", None)
    assert b.launch_plan(1, [], {"WORLD_SIZE": "1"}) == ("run", None)


def test_plan_external_launcher_must_match():
    b = _bench()
    assert b.launch_plan(8, [], {"WORLD_SIZE": "8"}) == ("run", None)
    what, why = b.launch_plan(8, [], {"WORLD_SIZE": "1"})
    assert what == "error" and "WORLD_SIZE 1" in why
    assert b.launch_plan(1, [], {"WORLD_SIZE": "4"})[0] == "error"


def test_plan_spawns_n_ranks_with_the_same_arguments():
    b = _bench()
    argv = ["--gpus", "4", "--config", "256x4", "--steps", "3"]
    what, cmd = b.launch_plan(4, argv, {})
    assert what == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    # a child that lost WORLD_SIZE must not launch again
    assert b.launch_plan(4, argv, {b.LAUNCHED_ENV: "1"})[0] == "error"


def test_relay_keeps_one_json_line_and_the_worst_rc(capfd):
    b = _bench()
    script = ("import sys, os; print('rank log'); print('{\"metric\": 1}'); "
              "sys.stderr.write('err\\n'); sys.exit(int(os.environ['" + b.LAUNCHED_ENV + "']) * 3)")
    rc = b.relay_ranks([sys.executable, "-c", script])
    out, err = capfd.readouterr()
    assert rc == 3
    assert out.strip().splitlines() == ['{"metric": 1}']
    assert "rank log" in err and "err" in err


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE 2" in r.stderr and not r.stdout.strip()


def test_self_launch_starts_ranks_with_world_size(tmp_path, capfd):
    """The spawned launcher really sets WORLD_SIZE/RANK in N fresh processes:
    run it on a stand-in script that reports its environment (no GPU)."""
    b = _bench()
    probe = tmp_path / "probe.py"
    probe.write_text("import os, json\n"
                     "if os.environ['RANK'] == '0':\n"
                     "    print(json.dumps({'ws': os.environ['WORLD_SIZE']}), flush=True)\n")
    what, cmd = b.launch_plan(2, [], {})
    cmd = [c if not c.endswith("bench.py") else str(probe) for c in cmd]
    rc = b.relay_ranks(cmd)
    out, _ = capfd.readouterr()
    assert rc == 0 and out.strip().splitlines() == ['{"ws": "2"}']


def test_self_launched_ranks_failing_fail_the_parent():
    """no GPU here: `bench.py --gpus 2` starts its 2 ranks, they fail (no device),
    and the parent exits non-zero with no JSON line instead of hanging or
    reporting a one-rank run"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--config", "128x1",
                        "--dist-backend", "gloo", "--no-cpu-baseline", "--steps", "1",
                        "--warmup", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "starting 2 ranks" in r.stderr


def test_plan_without_gpus_flag_follows_the_launcher():
    """`torchrun --nproc-per-node 8 bench.py` (no --gpus) runs 8 ranks;
    only an explicit --gpus that differs from WORLD_SIZE is refused"""
    b = _bench()
    assert b.launch_plan(None, [], {"WORLD_SIZE": "8"}) == ("run", None)
    assert b.launch_plan(None, [], {}) == ("run", None)
    assert b.launch_plan(2, [], {"WORLD_SIZE": "8"})[0] == "error"


def test_aggregate_roofline_sums_the_ranks():
    """N > 1 bench line: the node's algorithmic bytes are the ranks' sum, its peak
    N x 8 TB/s, against ms_per_step; the slowest rank's own fraction beside it"""
    b = _bench()
    # (alg bytes, U, render ms, pixels) of 4 ranks
    rows = [[1.0e9, 10, 0.50, 1000], [2.0e9, 20, 0.80, 2000],
            [1.5e9, 15, 0.60, 1500], [1.5e9, 15, 0.70, 1500]]
    a = b.aggregate_roofline(rows, ms_per_step=1.0)
    assert a["ranks"] == 4 and a["peak"] == 4 * 8000.0
    assert a["alg_bytes_per_frame"] == 6_000_000_000 and a["U_records"] == 60
    # 6 GB in 1 ms = 6000 GB/s of 32000
    assert a["achieved"] == 6000.0 and a["frac"] == round(6000 / 32000, 4)
    assert a["slowest_rank"] == 1 and a["render_ms_max_over_ranks"] == 0.8
    assert a["slowest_rank_frac"] == round(2e9 / 0.8e-3 / 1e9 / 8000, 4)
    assert a["frac_at_render_max"] == round(6e9 / 0.8e-3 / 1e9 / 32000, 4)
    assert [r["rank"] for r in a["per_rank"]] == [0, 1, 2, 3]
    # per-rank PMC traffic (tools/rank_traffic.py): the node's is the sum
    t = b.aggregate_roofline(rows, 1.0, rank_traffic=[1.2e9, 2.4e9, 1.8e9, 1.8e9])
    assert t["traffic"] == 7_200_000_000 and t["traffic_x_alg"] == 1.2
    assert t["traffic_GBps"] == 7200.0 and t["per_rank"][1]["traffic"] == 2_400_000_000
    assert t["per_rank"][1]["traffic_GBps"] == round(2.4e9 / 0.8e-3 / 1e9, 1)
    assert "traffic" not in a
    # a rank without a footprint count (U = -1) leaves the node's U unknown
    rows[2][1] = -1
    assert b.aggregate_roofline(rows, 1.0)["U_records"] is None


def test_assembled_parity_counts_every_pixel_of_the_oracle_rows():
    import numpy as np
    b = _bench()
    ref8 = np.arange(24, dtype=np.uint32).reshape(6, 4)
    got = ref8.copy()
    got[1, 0] += 1  # a row the oracle skipped at stride 2: not compared
    got[2, 3] += 1  # a compared row
    full = {"max_abs": 0.0, "tol": 1e-4, "steps_mismatch": 0}
    p = b.assembled_parity(got, (ref8, None, None), 2, 4, full)
    assert p["rows"] == 3 and p["pixels"] == 12 and p["rgba8_mismatch"] == 1
    assert p["row_stride"] == 2 and "4 ranks" in p["frame"]


def test_lists_sha_identifies_a_deal():
    import numpy as np
    b = _bench()
    x = np.arange(24, dtype=np.uint32).reshape(3, 8)
    y = x.copy()
    y[2, 7] = 0xFFFFFFFF
    assert b.lists_sha16(x) == b.lists_sha16(x.copy()) != b.lists_sha16(y)
    assert len(b.lists_sha16(x)) == 16
