#!/usr/bin/env python3
"""Benchmark of the d_render path on MI355X: Mrays/s + fps + HBM roofline fraction.

One step = one frame: clear the output, ray-cast every pixel of the frame (each
rank its own image tiles), and for N > 1 gather the tiles to rank 0 (RCCL over
xGMI) and assemble the frame.  For N > 1 frames are pipelined: frame f+1 renders
while frame f's gather and rank 0's assembly run on their own streams (double-
buffered tile buffers); the timed region ends when every frame is assembled.  The distribution volume is generated in HBM
before timing (synthetic, seeded) and replicated per GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1024x8]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment starts
its own N ranks: a child `python -m torch.distributed.run --nproc-per-node N
bench.py ...` (a fresh process; this one never touches the GPU), whose rank-0
JSON line it relays, exiting with the launcher's return code.  Under an external
launcher WORLD_SIZE must equal --gpus (a mismatch exits non-zero).

Prints ONE JSON line on rank 0 (contract in the task statement).  The metric
formula is the reference's own benchmark line, 1e-6*W*H/t (C:1065-1067); one
frame = one render_kernel (K:2387-2401), timed as runSingleTest does (C:1049-1067).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (volume edge, bins, W, H)
    "128x1": (128, 1, 256, 256),
    "256x4": (256, 4, 512, 512),
    "512x8": (512, 8, 1920, 1080),
    "1024x8": (1024, 8, 1920, 1080),
    # the reference's own records are 32-bin histograms (C:86-87): wide-record frames
    "512x32": (512, 32, 1920, 1080),
    "1024x16": (1024, 16, 1920, 1080),
    "1024x32": (1024, 32, 1920, 1080),
}
# GMM volumes: name -> (volume edge, components, W, H)
GMM_CONFIGS = {
    "gmm96": (96, 16, 256, 256),       # tests
    "gmm1024": (1024, 16, 1920, 1080),  # in-core on one GPU (206 GB)
    "gmm2048": (2048, 16, 3840, 2160),  # BASELINE config 5: z-slabs over 8 GPUs (207 GB each)
}
GMM_CPU_EDGE = 512  # CPU-baseline volume edge (a 1024^3 GMM exceeds the box's host-memory cap)
SEED = 20261015
CODEC_TEMPLATES, CODEC_SLOTS = 64, 4  # synthetic codec volume (methods 4/5/6)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md chip table


LAUNCHED_ENV = "VR_BENCH_RANKS_LAUNCHED"  # set by the self-launch in the ranks' environment


def launch_plan(gpus, argv, env):
    """What `bench.py --gpus N` does before any GPU call: ("run", None) = this
    process is the (only or one) rank; ("spawn", cmd) = start N ranks as fresh
    child processes with cmd; ("error", why) = refuse.  gpus None = the flag was
    not given: an external launcher's WORLD_SIZE decides (`torchrun
    --nproc-per-node 8 bench.py` runs 8 ranks), else one rank.  Only an explicit
    --gpus that differs from WORLD_SIZE is refused.  Pure, so the CPU tests cover
    every branch (tests/test_bench_launch.py)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if gpus is not None and int(ws) != gpus:
            return "error", (f"--gpus {gpus} but WORLD_SIZE {ws}: the launcher started a "
                             f"different number of ranks than asked for")
        return "run", None
    if gpus is None or gpus <= 1:
        return "run", None
    if env.get(LAUNCHED_ENV):
        return "error", "self-launched rank without WORLD_SIZE (launcher did not set it)"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__), *argv]
    return "spawn", cmd


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relay_ranks(cmd, env=None):
    """Run the rank launcher as a child process (never exec: this process may not
    replace itself) and stream its output: JSON lines (rank 0's result) to stdout,
    everything else to stderr, so the caller sees exactly one JSON line.  Returns
    the launcher's return code (non-zero when any rank failed)."""
    import signal
    import subprocess
    env = dict(os.environ if env is None else env)
    env[LAUNCHED_ENV] = "1"
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)

    def stop(signum, _frame):  # a killed parent takes its ranks with it
        p.terminate()  # torch.distributed.run forwards it to the ranks
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
        sys.exit(128 + signum)
    old = {sg: signal.signal(sg, stop) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        for line in p.stdout:
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()
        return p.wait()
    finally:
        for sg, h in old.items():
            signal.signal(sg, h)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: WORLD_SIZE under a launcher, else 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="1024x8", choices=sorted(CONFIGS) + sorted(GMM_CONFIGS))
    ap.add_argument("--method", type=int, default=1, choices=[1, 2, 3, 4, 5, 6, 7])
    ap.add_argument("--camera", default="C0", choices=["C0", "C1", "S"],
                    help="C0 runSingleTest (C:1024-1043), C1 display() at (30, 45) deg, "
                         "S display() at yaw 90 deg (screen x along the volume's z)")
    ap.add_argument("--baked", action="store_true",
                    help="basicDataProcessing first: frames filter the baked statistics "
                         "planes (vr_stats.hip) instead of decoding records per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-issue-bounds", action="store_true",
                    help="skip the untimed one-tile latency probe (roofline.compute): "
                         "profiling runs use it so a kernel's rocprofv3 average holds only "
                         "whole-frame launches")
    ap.add_argument("--render-streams", type=int, default=0, choices=[0, 1, 2],
                    help="N > 1: render streams consecutive frames alternate over "
                         "(0 = default: 2 at N > 1; N = 1 always 1)")
    ap.add_argument("--no-balance", action="store_true",
                    help="N > 1: keep the estimate-dealt tile lists (no measured-cost re-deal)")
    ap.add_argument("--dump-frame", default="",
                    help="rank 0 saves the last assembled frame (.npy) for checks")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo stages the tile gather through host memory (multi-rank "
                         "rehearsal on a single GPU; never for measurement)")
    ap.add_argument("--slab-rehearsal", action="store_true",
                    help="GMM volumes on ONE GPU: every rank's z-slab of the --rehearsal-ranks "
                         "chain generated in turn (untimed) and its march timed with HIP "
                         "events; reports per-slab ms and the pipeline-period estimate")
    ap.add_argument("--segments", type=int, default=1, choices=[1, 2],
                    help="GMM z-slab chains: z segments per rank (2: a thin front and a thick "
                         "back one, slabs.two_segment_bounds)")
    ap.add_argument("--rehearsal-ranks", type=int, default=8,
                    help="--slab-rehearsal: slabs (ranks) of the chain (BASELINE config 5: 8)")
    ap.add_argument("--link-gbs", type=float, default=153.0,
                    help="--slab-rehearsal: assumed xGMI point-to-point rate per link (GB/s) "
                         "for the alive-list hand-off and the frame reduce in the period")
    ap.add_argument("--rebalance", type=int, default=4,
                    help="GMM z-slabs (N > 1 and --slab-rehearsal): cost-balancing passes "
                         "after the equal cut (each: one untimed frame, slabs re-cut by its "
                         "per-slab costs and regenerated)")
    ap.add_argument("--cpu-row-stride", type=int, default=0,
                    help="CPU baseline renders every k-th row (0 = auto)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-measured HBM bytes per launch (tools/pmc_traffic.py) for "
                         "roofline.traffic; used only when the kernel matches")
    return ap.parse_args()


def camera_matrix(pkg, cam):
    if cam == "C0":
        return pkg.camera.single_test_inv_view()
    return pkg.camera.display_inv_view((0.0, 90.0) if cam == "S" else (30.0, 45.0))


def lib_sha16(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def traffic_entry(args, kernel, world, lists_sha=None, rank=0):
    """(PMC entry, where it comes from) of this workload from the committed
    passes (profiles/traffic.json), or (None, why not): only entries measured on
    this same libvr.so build (its sha256) and kernel count -- a rebuilt library
    needs a new PMC pass.  N = 1: a whole frame's HBM bytes per launch
    (tools/pmc_traffic.py).  N > 1: every rank's bytes per launch of its tile
    list, measured by tools/rank_traffic.py on one GPU for the very lists this
    run dealt (the entry's lists_sha16 must equal this run's)."""
    if not args.traffic_json or not os.path.exists(args.traffic_json):
        return None, None
    import __graft_entry__ as graft
    key = f"{args.config}|{args.camera}|m{args.method}" + ("|baked" if args.baked else "")
    if world > 1:
        key += f"|N{world}"
    with open(args.traffic_json) as f:
        entry = json.load(f).get(key)
    if not entry:
        return None, f"no PMC entry for {key}" + (" (per-rank lists: tools/rank_traffic.py)"
                                                  if world > 1 else "")
    sha = lib_sha16(graft.load_package().LIB_PATH)
    want = entry["kernels"][rank] if world > 1 and entry.get("kernels") else entry.get("kernel")
    if want != kernel or entry.get("lib_sha16") != sha:
        return None, (f"PMC entry {key} was measured on {want} of libvr.so "
                      f"{entry.get('lib_sha16')}, this run is {kernel} of {sha}")
    if world > 1 and entry.get("lists_sha16") != lists_sha:
        return None, (f"PMC entry {key} was measured on tile lists {entry.get('lists_sha16')}, "
                      f"this run dealt {lists_sha}")
    what = ("per rank, each rank's tile list rendered alone (tools/rank_traffic.py)"
            if world > 1 else "per launch")
    return entry, (
        f"{os.path.relpath(args.traffic_json, ROOT)}[{key}]: FETCH_SIZE x 2 + WRITE_SIZE {what}, "
        f"rocprofv3 --pmc on this libvr.so build ({sha}), {entry.get('measured', '')}")


VALU_ISSUE_CYCLES = 2      # SIMD cycles per f32 wave64 VALU instruction (f64 adds: ~4.4,
SIMDS, CLOCK_HZ = 1024, 2.4e9  # tools/valu_calib.hip); 256 CUs x 4 SIMDs at 2.4 GHz


def compute_bounds(pkg, torch, stream, W, H, m, method, kern_ms, pmc):
    """The bounds of a launch that is not HBM-bound:
    latency -- the frame cannot end before its longest tile's step chain does: the
    longest-ray tile rendered ALONE (one 64x4 tile, its list entry first in the
    longest-first order), min over 5 launches, as a fraction of the frame;
    valu -- f32-rate VALU issue: SQ_INSTS_VALU of the launch (committed PMC pass on
    this build) x 2 cycles over 1024 SIMDs x 2.4 GHz x kernel time (f64 decode
    instructions take ~2x that, so the true VALU busy lies between frac and ~2x)"""
    lst = pkg.tiles.tile_lists(W, H, 1, m)[0][:1]
    with torch.cuda.stream(stream):
        dl = torch.from_numpy(lst.view(np.int32).copy()).to(torch.cuda.current_device())
        buf = torch.zeros(256, dtype=torch.int32, device=dl.device)
        d = pkg.make_desc(buf, W, H, m, query_method=method, d_tile_list=dl, n_tiles=1)
        ts = []
        for _ in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            pkg.render(d)
            e1.record(stream)
            ts.append((e0, e1))
    torch.cuda.synchronize()
    t1 = min(a.elapsed_time(b) for a, b in ts[1:])
    out = {"latency": {"longest_tile_alone_ms": round(t1, 4), "frac": round(t1 / kern_ms, 4),
                       "kernel": pkg.last_kernel()}}
    if pmc and pmc.get("valu_insts"):
        busy = pmc["valu_insts"] * VALU_ISSUE_CYCLES / (SIMDS * CLOCK_HZ * kern_ms * 1e-3)
        out["valu"] = {"insts_per_launch": int(pmc["valu_insts"]),
                       "achieved": round(pmc["valu_insts"] / (kern_ms * 1e-3) / 1e12, 4),
                       "peak": round(SIMDS * CLOCK_HZ / VALU_ISSUE_CYCLES / 1e12, 4),
                       "unit": "T wave-instr/s", "frac": round(busy, 4)}
    return out


def host_threads():
    """CPU threads for the baseline and what the host grants: the OpenMP team is
    OMP_NUM_THREADS when set (the GPU box sets it to the job's CPU share, 16 per
    GPU), else every CPU in this process's affinity mask."""
    affinity = len(os.sched_getaffinity(0))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (env or affinity), {"nproc": os.cpu_count(), "affinity": affinity,
                               "omp_num_threads_env": env or None}


def cpu_baseline(pkg, cfg_name, m, method, row_stride):
    """The CPU oracle (C, OpenMP) ray-casting the same scene on this host's cores.
    Also returns the oracle's frame (packed RGBA8, float RGBA, samples per pixel)
    of a first, untimed pass for the parity check of the GPU frame."""
    import __graft_entry__ as graft
    orc = graft.load_oracle()
    n, nb, W, H = CONFIGS[cfg_name]
    threads, host = host_threads()
    if row_stride <= 0:
        row_stride = 1  # the whole frame
    codec = method in (4, 5, 6)
    if codec:
        cb, tp, er = orc.synth_codec_field(n, n, n, nb, CODEC_TEMPLATES, CODEC_SLOTS, SEED)
    else:
        vol = orc.synth_volume(n, n, n, nb, SEED, threads)
    print(f"cpu baseline: {n}^3 x {nb} volume in host RAM", file=sys.stderr, flush=True)
    p = orc.make_params(W, H, m, query_method=method, m7_dims=(n, n, n))

    def frame(want):
        if codec:
            return orc.render_codec(cb, tp, er, p, row_start=0, row_stride=row_stride,
                                    nthreads=threads)
        return orc.render(vol, p, row_start=0, row_stride=row_stride, nthreads=threads,
                          want_float=want, want_steps=want)
    ref = frame(True)[:3]  # untimed: the parity frame
    # repeat the frame until ~24 core-seconds of work have been timed
    frames, samples, dt = 0, 0, 0.0
    while frames == 0 or dt * threads < 24.0 and frames < 16:
        t0 = time.perf_counter()
        _, _, _, smp = frame(False)
        dt += time.perf_counter() - t0
        samples += smp
        frames += 1
        print(f"cpu baseline: frame {frames} ({dt:.1f} s)", file=sys.stderr, flush=True)
    rows = len(range(0, H, row_stride))
    rays = rows * W * frames
    omp = orc.max_threads()
    return {
        "value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
        "nproc": host["nproc"], "affinity_cpus": host["affinity"], "omp_max_threads": omp,
        "sample": (f"oracle/vr_oracle.c (-O3, OpenMP) on every {row_stride}th row of the "
                   f"{W}x{H} frame, {frames} frame(s) ({rays} rays, {samples} samples, "
                   f"{dt:.2f} s on {threads} threads = OMP_NUM_THREADS, the host's CPU share "
                   f"for this GPU; nproc {host['nproc']}, affinity {host['affinity']} CPUs, "
                   f"omp_get_max_threads {omp}), full {n}^3x{nb} "
                   f"{'codec ' if codec else ''}volume in host RAM"),
    }, (ref, row_stride)


def frame_parity(got8, got_f, got_n, kernel, ref, row_stride):
    """GPU frame vs the oracle's frame (rows 0, s, 2s, ... of the CPU baseline):
    the reference's own check compares its whole benchmark frame (C:1073-1077)"""
    r8, rf, rn = ref
    rows = slice(0, None, row_stride)
    g8, gf, gn, r8, rf, rn = got8[rows], got_f[rows], got_n[rows], r8[rows], rf[rows], rn[rows]
    hit = rn >= 0
    return {
        "against": "oracle frame of the cpu_baseline (same volume, camera, method)",
        "rows": int(g8.shape[0]), "pixels": int(g8.size), "hit_pixels": int(hit.sum()),
        "rgba8_mismatch": int(np.sum(g8 != r8)),
        "max_abs": float(np.max(np.abs(gf - rf))) if gf.size else 0.0,
        "tol": 1e-4,
        "steps_mismatch": int(np.sum(gn[hit] != rn[hit]) + np.sum(gn[~hit] != -1)),
        "kernel": kernel,
    }


def assembled_parity(frame8, ref, row_stride, world, full_render):
    """N > 1: the frame rank 0 assembled from every rank's gathered tiles (the
    last timed frame) against the oracle frame of the cpu_baseline, on the rows
    the oracle rendered (0, s, 2s, ...).  Misses: the oracle leaves them 0, the
    tiles write 0 (vr.h tile-list mode), so every pixel is compared.  The float
    RGBA and sample counts come from rank 0's whole-frame render of the same
    view (full_render, frame_parity): the tiles carry packed RGBA8 only."""
    rows = slice(0, None, row_stride)
    g8, r8 = frame8[rows], ref[0][rows]
    return {
        "against": "oracle frame of the cpu_baseline (same volume, camera, method)",
        "frame": f"assembled on rank 0 from the tiles of {world} ranks (last timed frame)",
        "rows": int(g8.shape[0]), "row_stride": row_stride, "pixels": int(g8.size),
        "rgba8_mismatch": int(np.sum(g8 != r8)),
        "max_abs": full_render["max_abs"], "tol": full_render["tol"],
        "steps_mismatch": full_render["steps_mismatch"],
        "float_and_steps_from": "rank 0's whole-frame render of the view",
        "full_frame_render": full_render,
    }


def aggregate_roofline(per_rank, ms_per_step, peak_gbs=HBM_PEAK_GBS, rank_traffic=None):
    """Whole-node roofline of an N-rank frame.  per_rank: one row per rank of
    (algorithmic bytes of its launch, U of its tile list or -1, its render ms
    alone, pixels it renders).  Every rank reads its own footprint from its own
    HBM, so the node's algorithmic bytes are the sum over ranks and its peak is
    N x 8 TB/s: frac = sum(alg) / ms_per_step / (N x peak).  Beside it the same
    bytes over the slowest rank's render alone (what the frame's compute could
    reach without the gather, the assembly and the host) and the slowest
    rank's own fraction.  rank_traffic (optional): every rank's PMC bytes per
    launch of its list (tools/rank_traffic.py): the node's fabric traffic per
    frame is their sum."""
    per_rank = np.asarray(per_rank, dtype=np.float64)
    n = per_rank.shape[0]
    alg, u, ms, px = per_rank.T
    total = float(alg.sum())
    node = total / (ms_per_step * 1e-3) / 1e9
    slow = int(np.argmax(ms))
    frac = lambda b, t, k: round(b / (t * 1e-3) / 1e9 / (k * peak_gbs), 4)
    out = {
        "ranks": n, "peak": n * peak_gbs, "unit": "GB/s",
        "alg_bytes_per_frame": int(total),
        "U_records": int(u.sum()) if np.all(u >= 0) else None,
        "achieved": round(node, 1), "frac": frac(total, ms_per_step, n),
        "of": "sum over ranks of the algorithmic bytes / ms_per_step / (N x 8 TB/s)",
        "render_ms_max_over_ranks": round(float(ms[slow]), 4),
        "frac_at_render_max": frac(total, ms[slow], n),
        "slowest_rank": slow, "slowest_rank_frac": frac(alg[slow], ms[slow], 1),
        "per_rank": [{"rank": r, "alg_bytes": int(alg[r]), "U_records": int(u[r]) if u[r] >= 0 else None,
                      "render_ms": round(float(ms[r]), 4), "pixels": int(px[r]),
                      "frac": frac(alg[r], ms[r], 1)} for r in range(n)],
    }
    if rank_traffic is not None:
        tr = [int(v) for v in rank_traffic]
        out["traffic"] = sum(tr)
        out["traffic_x_alg"] = round(sum(tr) / total, 4)
        out["traffic_GBps"] = round(sum(tr) / (ms_per_step * 1e-3) / 1e9, 1)
        for r, row in enumerate(out["per_rank"]):
            row["traffic"] = tr[r]
            row["traffic_GBps"] = round(tr[r] / (ms[r] * 1e-3) / 1e9, 1)
    return out


def rank_costs(pkg, torch, lst, W, H, m, method, dev, stream):
    """Per-tile costs (tiles.tile_costs_from_steps, int64) of one rank's tile list,
    rendered once with per-pixel sample counts (untimed)."""
    n_slots = lst.shape[0]
    n_tiles = pkg.tiles.tiles_x(W) * pkg.tiles.tiles_y(H)
    with torch.cuda.stream(stream):
        tl = torch.from_numpy(lst.view(np.int32).copy()).to(dev)
        buf = torch.zeros(n_slots * 256, dtype=torch.int32, device=dev)
        steps = torch.full((n_slots * 256,), -1, dtype=torch.int32, device=dev)
        pkg.render(pkg.make_desc(buf, W, H, m, query_method=method, d_tile_list=tl,
                                 n_tiles=n_slots, d_steps=steps))
    torch.cuda.synchronize()
    return pkg.tiles.tile_costs_from_steps(steps.cpu().numpy(), lst, n_tiles)


def deal_by_cost(pkg, world, W, H, cost):
    """The cost-dealt lists every rank derives from the summed per-tile costs;
    rank 0 takes a smaller share (it also receives and assembles the frame)."""
    share = np.ones(world)
    share[0] = pkg.tiles.rank0_share(world)
    return pkg.tiles.tile_lists_by_cost(W, H, world, np.asarray(cost), share=share)


def lists_sha16(lists):
    """Identity of a split's tile lists (keys the per-rank PMC traffic entries)."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(lists, dtype=np.uint32).tobytes()).hexdigest()[:16]


def balanced_lists(pkg, lists, world, rank, W, H, m, method, dev, stream, backend):
    """Re-deal the tiles by measured cost (untimed, once per view): every rank
    renders its estimate-ordered list once with per-pixel sample counts, the
    per-tile costs are summed over ranks (one all_reduce of a tiles-sized int64
    vector, 64 KB at 1080p) and every rank derives the same cost-dealt lists
    (tiles.tile_lists_by_cost): ranks and their XCDs get equal work, not only
    equal pixel counts.  The sums are integers, so emulated_rank_lists derives
    the very same lists in one process."""
    import torch
    import torch.distributed as dist
    cost = torch.from_numpy(rank_costs(pkg, torch, lists[rank], W, H, m, method, dev, stream))
    if backend == "nccl":
        cost = cost.to(dev)
    dist.all_reduce(cost)
    return deal_by_cost(pkg, world, W, H, cost.cpu().numpy())


def emulated_rank_lists(pkg, torch, world, W, H, m, method, dev, stream):
    """The cost-dealt lists of a `world`-rank bench run, derived in one process
    on one GPU (every rank's estimate list rendered in turn, the costs summed as
    the all_reduce would): tools/rank_traffic.py profiles each rank's list."""
    lists = pkg.tiles.tile_lists(W, H, world, m)
    cost = sum(rank_costs(pkg, torch, lists[r], W, H, m, method, dev, stream)
               for r in range(world))
    return deal_by_cost(pkg, world, W, H, cost)


def gmm_cpu_baseline(m, method, W, H, K):
    """The CPU oracle's GMM march (C) on this host's cores: a band of rows of the
    same frame, on a GMM_CPU_EDGE^3 volume held in host RAM."""
    import __graft_entry__ as graft
    orc = graft.load_oracle()
    n = GMM_CPU_EDGE
    threads, host = host_threads()
    wm, sg = orc.synth_gmm(n, n, n, K, SEED, nthreads=threads)
    rows = (H // 2 - 24, H // 2 + 24)  # the centre band: the longest rays
    p = orc.make_params(W, H, m, query_method=method)
    frames, rays, dt = 0, 0, 0.0
    while frames == 0 or dt * threads < 24.0 and frames < 8:
        t0 = time.perf_counter()
        orc.render_gmm_rows(wm, sg, (n, n, n), p, rows[0], rows[1], nthreads=threads)
        dt += time.perf_counter() - t0
        rays += (rows[1] - rows[0]) * W
        frames += 1
    return {
        "value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
        "nproc": host["nproc"], "affinity_cpus": host["affinity"],
        "omp_max_threads": orc.max_threads(),
        "sample": (f"oracle/vr_oracle.c GMM march (-O3, OpenMP) on the {rows[1] - rows[0]} centre rows of the "
                   f"{W}x{H} frame, {frames} pass(es) ({rays} rays, {dt:.2f} s on {threads} "
                   f"threads), {n}^3 x {K} GMM volume in host RAM (the GPU workload's "
                   f"volume is larger than the box's host-memory cap)"),
    }


def gmm_slab_rehearsal(args, pkg, torch, dev, stream, m, n, K, W, H, rec_bytes):
    """BASELINE config 5 rehearsed on one GPU.  The chain's R
    slabs (march order) are generated in HBM one at a time, untimed, as rank r
    holds slab r; each slab's march is timed with HIP events over --steps frames
    of its real input (slab 0: the camera rays; slab r: the alive list slab r - 1
    handed on, kept in HBM); its U is counted on the same input.  Passes: equal
    slabs, then --rebalance cost-balanced cuts as the N-rank run makes them
    (slabs.bounds_by_cost / two_segment_bounds), the best one re-measured.  The
    line is an ESTIMATE of the R-GPU pipeline period, not a measurement: the
    max over ranks of (alive lists received + march + sent + the frame into the
    reduce), the transfers priced at --link-gbs (slabs.period_with_handoff);
    value null, n_gpus 1, scaling null."""
    R = args.rehearsal_ranks
    direction = pkg.slabs.march_direction(m, W, H)
    frame = torch.zeros(W * H, dtype=torch.int32, device=dev)
    desc = pkg.make_desc(frame, W, H, m, query_method=args.method, volume_size=(1, 1, 1))
    bufs = [torch.zeros((W * H, pkg.slabs.RAY_WORDS), dtype=torch.int32, device=dev)
            for _ in range(2)]
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    # the library launches on `stream` (pkg.set_stream) and resets the alive-list
    # counter there itself; the events and cnt.item() below use the same stream
    assert torch.cuda.current_stream(dev) == stream

    def chain(bounds, label):
        rows, n_in = [], 0
        for i, (z_lo, z_hi) in enumerate(bounds):
            if i and n_in == 0:  # no ray reaches this slab: nothing to march
                rows.append({"slab": i, "z": [z_lo, z_hi], "rays_in": 0, "ms": 0.0,
                             "rays_out": 0, "U_records": 0})
                continue
            zb, ns = pkg.slabs.resident_slices(z_lo, z_hi, n)
            tg = time.perf_counter()
            pkg.synthesize_gmm((n, n, n), K, SEED, z_base=zb, nslices=ns)
            torch.cuda.synchronize()
            gen_s = time.perf_counter() - tg
            out, inp = bufs[i % 2], bufs[(i + 1) % 2]
            slab = pkg.gmm_slab(z_lo, z_hi, out, cnt, d_rays_in=inp if i else None, n_rays_in=n_in)
            u = pkg.gmm_count_footprint(desc, slab)
            ev = []
            for f in range(args.warmup + args.steps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                pkg.render_gmm(desc, slab)
                e1.record(stream)
                if f >= args.warmup:
                    ev.append((e0, e1))
            torch.cuda.synchronize()
            ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
            n_out = int(cnt.item())
            if n_out > (n_in if i else W * H):
                raise RuntimeError(f"slab {i}: {n_out} alive rays out of {n_in if i else W * H} in")
            # algorithmic bytes of the slab's launch: its footprint records, the
            # alive list in and out, the pixels of rays ending here
            ended = (W * H if i == 0 else n_in) - n_out
            alg = u * rec_bytes + (n_in + n_out) * pkg.slabs.RAY_WORDS * 4 + max(ended, 0) * 4
            rows.append({"slab": i, "z": [z_lo, z_hi], "resident_slices": ns,
                         "rays_in": n_in if i else W * H, "rays_out": n_out,
                         "ms": round(ms, 4), "U_records": int(u), "alg_bytes": int(alg),
                         "GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                         "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "generate_s": round(gen_s, 2)})
            print(f"slab rehearsal ({label}) slab {i} z [{z_lo}, {z_hi}): {ms:.3f} ms, "
                  f"{n_out} rays alive, U {u}", file=sys.stderr, flush=True)
            n_in = n_out
            pkg.free_gmm()
        return rows

    def owners(nseg):
        return list(range(nseg)) if nseg == R else pkg.slabs.segment_owner(nseg, R)

    def rank_period(rows):
        """max over ranks of the summed march time of the segments a rank holds"""
        per = [0.0] * R
        for r, row in zip(owners(len(rows)), rows):
            row["rank"] = r
            per[r] += row["ms"]
        return max(per), per

    def estimate(rows):
        """the period estimate with the hand-off (what a pass is judged by)"""
        return pkg.slabs.period_with_handoff(
            [r["ms"] for r in rows], [r["rays_out"] for r in rows], owners(len(rows)), R,
            W * H * 4, args.link_gbs)

    pkg.free_gmm()
    torch.cuda.empty_cache()
    bounds = pkg.slabs.slab_bounds(n, R, direction)
    rows_eq = rows = chain(bounds, "equal")
    free_now, _ = torch.cuda.mem_get_info(dev)
    cap = pkg.slabs.max_slices_for(n, n, K, free_now)
    passes = [estimate(rows)[0]]
    best = None  # the balanced cut with the shortest period (a run keeps that cut)
    for p in range(args.rebalance):
        costs = [r["ms"] for r in rows]
        if args.segments == 2:  # every rank a front and a back segment
            bounds = pkg.slabs.two_segment_bounds(n, R, direction, bounds, costs, cap)
        else:
            bounds = pkg.slabs.bounds_by_cost(n, R, direction, bounds, costs, cap)
        rows = chain(bounds, f"balanced {p + 1}")
        passes.append(estimate(rows)[0])
        if best is None or passes[-1] < best[0]:
            best = (passes[-1], bounds)
    rows_bal = rows
    if best is not None and args.rebalance > 1:
        # the kept cut measured again: its period is this fresh run's, not the
        # minimum over noisy passes
        rows_bal = chain(best[1], "kept cut")
    march_period, per_rank = rank_period(rows_bal)
    # the hand-off: every segment's alive list crosses one xGMI link to the next
    # rank (none between the two segments rank N-1 holds), every rank's frame
    # goes into the reduce; at the stated link rate (slabs.period_with_handoff)
    serial, overlap, handoff = estimate(rows_bal)
    for r in rows_bal:
        r["bytes_out"] = r["rays_out"] * pkg.slabs.RAY_WORDS * 4
    period = serial
    kernel = pkg.last_kernel()
    worst = max(rows_bal, key=lambda r: r["ms"])
    cpu = None if args.no_cpu_baseline else gmm_cpu_baseline(m, args.method, W, H, K)
    out = {
        "metric": f"Mrays/s + fps at {n}^3 x {K}-component GMM volume, {W}x{H}; % HBM roofline "
                  f"({R}-rank slab chain rehearsed on one GPU: pipeline-period ESTIMATE, "
                  "not a measured N-GPU rate)",
        "value": None,
        "estimated_Mrays_s": round(W * H / (period * 1e-3) / 1e6, 3),
        "period_estimate_ms": round(period, 4),
        "period_estimate": (f"max over ranks of (alive lists received + march + sent + frame "
                            f"into the reduce), transfers at {args.link_gbs} GB/s per xGMI link "
                            "(assumed, not measured: one GPU here), nothing overlapped"),
        "period_overlapped_ms": round(overlap, 4),
        "period_march_only_ms": round(march_period, 4),
        "unit": "Mrays/s",
        "n_gpus": 1,
        "physical_gpus": 1,
        "rehearsal_shared_gpus": True,
        "rehearsal_ranks": R,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": None,
        "fps": None,
        "higher_is_better": True,
        "scaling": None,
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic seeded GMM volume (seed {SEED}, DESIGN.md s11.1), one slab in HBM at a time",
        "config": {
            "workload": f"{n}^3 x {K}-component GMM volume, {W}x{H}, camera {args.camera}, "
                        f"queryMethod {args.method}, {R} z-slabs",
            "volume": [n, n, n], "components": K, "image": [W, H], "camera": args.camera,
            "query_method": args.method, "density": 0.05,
            "parallelism": f"z-slabs x{R} ranks ({args.segments} segment(s) each) rehearsed on 1 "
                           "GPU (each segment's march timed on its real alive-list input; "
                           "hand-off and frame reduce not timed)",
            "segments_per_rank": args.segments,
            "march": "each segment's mean march time (HIP events, "
                     f"{args.steps} frames after {args.warmup} warm-up)",
            "rank_ms": [round(v, 4) for v in per_rank],
            "handoff": handoff,
            "ray_bytes": pkg.slabs.RAY_WORDS * 4,
            "slabs_equal": rows_eq,
            "slabs_balanced": rows_bal,
            "period_ms_per_pass": [round(v, 4) for v in passes],
            "kept_pass": passes.index(min(passes[1:])) if len(passes) > 1 else 0,
            "kept_cut_remeasured": args.rebalance > 1,
        },
        "roofline": {
            "bound": "hbm", "achieved": worst.get("GBps"), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": worst.get("frac"), "traffic": None,
            "traffic_source": "no PMC pass for this workload",
            "kernel": kernel, "kernel_ms": worst["ms"], "of": f"slowest slab ({worst['slab']})",
            "alg_bytes_per_launch": worst.get("alg_bytes"), "U_records": worst.get("U_records"),
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    return out


def gmm_two_segment_run(args, pkg, torch, dist, dev, stream, m, n, K, W, H, rank, world, ndev):
    """N > 1 GMM chain with two z segments per rank (--segments 2, DESIGN.md
    11.3): rank r holds front segment r in GMM slot 0 and back segment 2N-1-r in
    slot 1 (slabs.two_segment_bounds, segment_owner).  Ranks run a tick schedule
    (slabs.two_segment_ticks): at tick t, the front march of frame t - r (input
    from rank r - 1 over the forward group), then the back march of frame
    t - (2N-1-r) (input from rank r + 1 over the backward group; rank N-1 takes
    its own front output of the tick before), alive lists handed on by isend,
    each frame summed on rank 0 by an asynchronous reduce on a third group once
    the rank's back march of it is done.  Untimed balancing frames first
    (per-segment costs all-reduced, segments re-cut and regenerated), then the
    timed steady-state ticks: each completes one frame."""
    S = pkg.slabs
    R = world
    direction = S.march_direction(m, W, H)
    fwd, bwd, asm = (dist.new_group(list(range(world))) for _ in range(3))
    cdev = dev if args.dist_backend == "nccl" else "cpu"
    front_i, back_i = rank, 2 * R - 1 - rank
    RING = 2 * R + 2
    frames = [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(RING)]
    descs = [pkg.make_desc(f, W, H, m, query_method=args.method, volume_size=(1, 1, 1))
             for f in frames]
    lst = lambda: torch.zeros((W * H, S.RAY_WORDS), dtype=torch.int32, device=dev)
    f_in, b_in, b_out = lst(), lst(), lst()
    f_out = [lst(), lst()]  # rank N-1: its back march reads the previous tick's front output
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    own_front = [None, None]  # rank N-1: (buffer, count) of its front output by frame parity

    def generate(bounds):
        for slot, i in ((0, front_i), (1, back_i)):
            pkg.gmm_select(slot)
            pkg.free_gmm()
        torch.cuda.empty_cache()
        for slot, i in ((0, front_i), (1, back_i)):
            pkg.gmm_select(slot)
            zb, ns = S.resident_slices(*bounds[i], n)
            pkg.synthesize_gmm((n, n, n), K, SEED, z_base=zb, nslices=ns)
        torch.cuda.synchronize()

    state = {"works": [None] * RING, "sf": None, "sb": None}

    def run_ticks(t0, t1, nframes, seg_ev=None):
        for t in range(t0, t1):
            ff, fb = S.two_segment_ticks(rank, R, t)
            if 0 <= ff < nframes:
                b = ff % RING
                if state["works"][b] is not None:
                    state["works"][b].wait()
                    state["works"][b] = None
                frames[b].zero_()
                pkg.gmm_select(0)
                n_in = S.recv_alive(rank - 1, f_in, dist, group=fwd) if rank > 0 else 0
                out = f_out[ff % 2]
                if state["sf"] is not None:
                    state["sf"].wait()
                if seg_ev is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                pkg.render_gmm(descs[b], pkg.gmm_slab(*bounds[front_i], out, cnt,
                                                      d_rays_in=f_in if rank > 0 else None,
                                                      n_rays_in=n_in))
                if seg_ev is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record(stream)
                    seg_ev[0].append((e0, e1))
                n_out = int(cnt.item())
                if rank < R - 1:
                    state["sf"] = S.isend_alive(out, n_out, rank + 1, dist, group=fwd)
                else:
                    own_front[ff % 2] = (out, n_out)
            if 0 <= fb < nframes:
                b = fb % RING
                pkg.gmm_select(1)
                if rank == R - 1:
                    rin, n_in = own_front[fb % 2]
                else:
                    n_in = S.recv_alive(rank + 1, b_in, dist, group=bwd)
                    rin = b_in
                if state["sb"] is not None:
                    state["sb"].wait()
                if seg_ev is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                pkg.render_gmm(descs[b], pkg.gmm_slab(*bounds[back_i], b_out, cnt, d_rays_in=rin,
                                                      n_rays_in=n_in))
                if seg_ev is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record(stream)
                    seg_ev[1].append((e0, e1))
                n_out = int(cnt.item())
                if rank > 0:
                    state["sb"] = S.isend_alive(b_out, n_out, rank - 1, dist, group=bwd)
                elif n_out:
                    raise RuntimeError(f"{n_out} rays alive past the last segment")
                state["works"][b] = S.reduce_frame(frames[b], dist, group=asm, async_op=True)

    def drain():
        for w in state["works"]:
            if w is not None:
                w.wait()
        state["works"] = [None] * RING
        for k in ("sf", "sb"):
            if state[k] is not None:
                state[k].wait()
                state[k] = None
        torch.cuda.synchronize()

    # initial cut: uniform cost; then balancing frames (untimed): per-segment
    # march times all-reduced, segments re-cut by them and regenerated
    free_now, _ = torch.cuda.mem_get_info(dev)
    cap_t = torch.tensor([S.max_slices_for(n, n, K, free_now)], dtype=torch.int64, device=cdev)
    dist.all_reduce(cap_t, op=dist.ReduceOp.MIN)
    cap = int(cap_t.item())
    bounds = S.two_segment_bounds(n, R, direction, max_slices=cap)
    generate(bounds)
    passes = []
    best = None  # (period, cut) of the best measured pass: the steady state runs that cut
    for _ in range(max(args.rebalance, 1)):
        nf = 2
        ev = ([], [])
        run_ticks(0, nf + 2 * R - 1, nf, seg_ev=ev)
        drain()
        costs = torch.zeros(2 * R, dtype=torch.float64, device=cdev)
        costs[front_i] = float(np.mean([a.elapsed_time(b) for a, b in ev[0]])) if ev[0] else 0.0
        costs[back_i] = float(np.mean([a.elapsed_time(b) for a, b in ev[1]])) if ev[1] else 0.0
        dist.all_reduce(costs)
        c = costs.cpu().tolist()
        passes.append(max(c[i] + c[2 * R - 1 - i] for i in range(R)))
        if best is None or passes[-1] < best[0]:
            best = (passes[-1], list(bounds))
        bounds = S.two_segment_bounds(n, R, direction, bounds, c, cap)
        generate(bounds)
    if list(bounds) != best[1]:  # the last re-cut is unmeasured: run the best measured cut
        bounds = best[1]
        generate(bounds)
    # steady state: W warm-up frames' worth of ticks, then K timed ticks (each
    # completes one frame at rank 0), then the pipeline drains (untimed)
    F = args.warmup + args.steps + 2 * R
    t_start = args.warmup + 2 * R - 1
    run_ticks(0, t_start, F)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_ticks(t_start, t_start + args.steps, F)
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    run_ticks(t_start + args.steps, F + 2 * R - 1, F)
    drain()
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    if args.dump_frame and rank == 0:
        last = frames[(F - 1) % RING]
        np.save(args.dump_frame, last.cpu().numpy().view(np.uint32).reshape(H, W))
    out = None
    if rank == 0:
        phys = min(world, max(ndev, 1))
        out = {
            "metric": f"Mrays/s + fps at {n}^3 x {K}-component GMM volume, {W}x{H}; % HBM roofline",
            "value": round(W * H / (elapsed / args.steps) / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "physical_gpus": phys,
            "rehearsal_shared_gpus": world > phys,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1e3 / ms_per_step, 2),
            "higher_is_better": True,
            "scaling": None if world > phys else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic seeded GMM volume (seed {SEED}, DESIGN.md s11.1)",
            "config": {
                "workload": f"{n}^3 x {K}-component GMM volume, {W}x{H}, camera {args.camera}, "
                            f"queryMethod {args.method}",
                "volume": [n, n, n], "components": K, "image": [W, H], "camera": args.camera,
                "query_method": args.method, "density": 0.05,
                "parallelism": (f"z-slab chain x{world}, two segments per rank + " +
                                ("RCCL send/recv of alive rays + reduce"
                                 if args.dist_backend == "nccl" else "gloo host staging")),
                "segments": [list(b) for b in bounds],
                "balance_pass_max_rank_ms": [round(v, 4) for v in passes],
            },
            "roofline": None,
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return out


def main_gmm(args):
    """GMM volumes.  N = 1: the whole volume resident, one
    launch per frame.  N > 1: rank r holds z-slab r (in the view's march order)
    and the frame is a chain: receive the previous slab's alive rays, march,
    send the survivors on (RCCL point-to-point over xGMI), then the ranks'
    frames are summed on rank 0 by an asynchronous reduce on a separate group.
    Ranks run ahead frame by frame: the chain is a pipeline whose period is the
    slowest rank's (receive + march + send), not the sum over ranks."""
    import torch
    import torch.distributed as dist
    import __graft_entry__ as graft

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, (world, args.gpus)  # launch_plan refused anything else
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks need {world} GPUs, {ndev} visible")
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    pkg = graft.load_package()
    n, K, W, H = GMM_CONFIGS[args.config]
    if args.method not in (1, 2):
        raise SystemExit("GMM volumes support --method 1 (mean) and 2 (variance)")
    m = camera_matrix(pkg, args.camera)
    rec_bytes = 8 * K if args.method == 1 else 12 * K
    free, _ = torch.cuda.mem_get_info(dev)
    stream = torch.cuda.Stream(device=dev)
    pkg.set_stream(stream)
    if world == 1 and args.slab_rehearsal:
        with torch.cuda.stream(stream):  # the counter resets and the launches on one stream
            return gmm_slab_rehearsal(args, pkg, torch, dev, stream, m, n, K, W, H, rec_bytes)
    if world > 1 and args.segments == 2:
        with torch.cuda.stream(stream):
            return gmm_two_segment_run(args, pkg, torch, dist, dev, stream, m, n, K, W, H, rank,
                                       world, ndev)
    if world == 1:
        need = n ** 3 * 12 * K
        if need > free * 0.95:
            raise SystemExit(f"{args.config}: {need / 1e9:.0f} GB of GMM records exceed this GPU's "
                             f"{free / 1e9:.0f} GB; run it on >= {int(need / (free * 0.9)) + 1} "
                             "GPUs (z-slabs) or simulate the ranks with tools/gmm_slab_sim.py")
        pkg.synthesize_gmm((n, n, n), K, SEED)
        z_lo, z_hi = 0, n
    else:
        direction = pkg.slabs.march_direction(m, W, H)
        z_lo, z_hi = pkg.slabs.slab_bounds(n, world, direction)[rank]
        zb, ns = pkg.slabs.resident_slices(z_lo, z_hi, n)
        pkg.synthesize_gmm((n, n, n), K, SEED, z_base=zb, nslices=ns)
    # Frames: a ring of 2N buffers.  Each frame's assembly (a SUM reduce on its
    # own process group, hence its own RCCL stream) is issued asynchronously
    # right after the frame's march, so no rank waits for the whole chain: rank 0
    # can march frame f+1 while the last rank still marches frame f, and a ring
    # buffer is reused only after its reduce has consumed it.
    R = 2 * world if world > 1 else 1
    frames = [torch.zeros(W * H, dtype=torch.int32, device=dev) for _ in range(R)]
    descs = [pkg.make_desc(f, W, H, m, query_method=args.method, volume_size=(1, 1, 1))
             for f in frames]
    desc = descs[0]
    asm_group = None
    if world > 1:
        rays_in = torch.zeros((W * H, pkg.slabs.RAY_WORDS), dtype=torch.int32, device=dev)
        rays_out = torch.zeros((W * H, pkg.slabs.RAY_WORDS), dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        asm_group = dist.new_group(list(range(world)))
    torch.cuda.synchronize()
    ev, alive = [], []
    balanced = False
    works = [None] * R
    nframe = [0]

    def step(timed):
        b = nframe[0] % R
        nframe[0] += 1
        frame = frames[b]
        with torch.cuda.stream(stream):
            if works[b] is not None:
                works[b].wait()  # this buffer's previous frame has been reduced
            frame.zero_()  # C:208
            n_in = 0
            if world > 1:
                if rank > 0:
                    n_in = pkg.slabs.recv_alive(rank - 1, rays_in, dist)
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            if world == 1:
                pkg.render_gmm(descs[b])
            else:
                pkg.render_gmm(descs[b], pkg.gmm_slab(z_lo, z_hi, rays_out, cnt,
                                                      d_rays_in=rays_in if rank > 0 else None,
                                                      n_rays_in=n_in))
            if timed:
                e1.record(stream)
                ev.append((e0, e1))
            if world > 1:
                n_out = int(cnt.item())
                if timed:
                    alive.append(n_out)
                if rank < world - 1:
                    pkg.slabs.send_alive(rays_out, n_out, rank + 1, dist)
                works[b] = pkg.slabs.reduce_frame(frame, dist, group=asm_group, async_op=True)

    def drain():
        for w in works:
            if w is not None:
                w.wait()
        torch.cuda.synchronize()

    if world > 1 and not args.no_balance:
        # Cost-balanced slabs (untimed, once per view): early ray termination
        # front-loads the work, so one frame on equal slabs measures every rank's
        # march, and all ranks re-cut the slabs by those costs (largest slab cost
        # minimised, each slab within the smallest rank's free HBM), then
        # generate their new slab (slabs.bounds_by_cost).  --rebalance passes: the
        # cut assumes a uniform cost inside each measured slab, so a second pass
        # on the first cut's costs tightens it (the one-GPU rehearsal of config 5:
        # period 6.44 ms equal, 4.51 after one pass; profiles/r05).
        direction = pkg.slabs.march_direction(m, W, H)
        bounds = pkg.slabs.slab_bounds(n, world, direction)
        cdev = dev if args.dist_backend == "nccl" else "cpu"
        best = None  # (max rank ms, cut) of the best measured pass: the timed frames run it

        def regenerate(cut):
            pkg.free_gmm()
            zb, ns = pkg.slabs.resident_slices(*cut[rank], n)
            pkg.synthesize_gmm((n, n, n), K, SEED, z_base=zb, nslices=ns)
            torch.cuda.synchronize()
            return cut[rank]

        for _ in range(max(args.rebalance, 1)):
            step(True)
            drain()
            ms = ev[-1][0].elapsed_time(ev[-1][1])
            ev.clear()
            alive.clear()
            pkg.free_gmm()
            free_now, _ = torch.cuda.mem_get_info(dev)
            costs = torch.zeros(world, dtype=torch.float64, device=cdev)
            costs[rank] = ms
            dist.all_reduce(costs)
            c = costs.cpu().tolist()
            if best is None or max(c) < best[0]:
                best = (max(c), list(bounds))
            cap = torch.tensor([pkg.slabs.max_slices_for(n, n, K, free_now)], dtype=torch.int64,
                               device=cdev)
            dist.all_reduce(cap, op=dist.ReduceOp.MIN)
            bounds = pkg.slabs.bounds_by_cost(n, world, direction, bounds, c, int(cap.item()))
            z_lo, z_hi = regenerate(bounds)
        if list(bounds) != best[1]:
            # the last re-cut was never measured (re-cuts that assume a uniform
            # cost inside each slab can oscillate): time the best measured cut
            bounds = best[1]
            z_lo, z_hi = regenerate(bounds)
        balanced = True
    # U before the warm-up (as in main(): the counting pass warms clocks and translation)
    u = pkg.gmm_count_footprint(desc) if world == 1 else None
    for _ in range(args.warmup):
        step(False)
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    drain()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if args.dump_frame and rank == 0:
        last = frames[(nframe[0] - 1) % R]
        np.save(args.dump_frame, last.cpu().numpy().view(np.uint32).reshape(H, W))
    kernel = pkg.last_kernel()
    pmc, traffic_src = traffic_entry(args, kernel, world)
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    alg_bytes = u * rec_bytes + W * H * 4 if u is not None else None
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if alg_bytes else None
    ms_per_step = elapsed / args.steps * 1e3
    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = gmm_cpu_baseline(m, args.method, W, H, K)
        out = {
            "metric": f"Mrays/s + fps at {n}^3 x {K}-component GMM volume, {W}x{H}; % HBM roofline",
            "value": round(W * H / (elapsed / args.steps) / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "physical_gpus": min(world, max(ndev, 1)),
            "rehearsal_shared_gpus": world > max(ndev, 1),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1e3 / ms_per_step, 2),
            "higher_is_better": True,
            "scaling": None if world > max(ndev, 1) else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic seeded GMM volume (seed {SEED}, DESIGN.md s11.1)",
            "config": {
                "workload": f"{n}^3 x {K}-component GMM volume, {W}x{H}, camera {args.camera}, "
                            f"queryMethod {args.method}",
                "volume": [n, n, n], "components": K, "image": [W, H], "camera": args.camera,
                "query_method": args.method, "density": 0.05,
                "parallelism": ("whole volume x1" if world == 1 else
                                f"z-slabs x{world} + " + ("RCCL send/recv of alive rays + reduce"
                                                          if args.dist_backend == "nccl"
                                                          else "gloo host staging")),
                "slab": [z_lo, z_hi],
                "slab_cut": (None if world == 1 else f"measured cost ({max(args.rebalance, 1)} untimed frame(s))"
                             if balanced else "equal"),
                "alive_rays_out_rank0": int(np.mean(alive)) if alive else None,
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernel,
                "kernel_ms": round(kern_ms, 4),
                "alg_bytes_per_launch": int(alg_bytes) if alg_bytes else None,
                "U_records": int(u) if u is not None else None,
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


def main():
    args = parse()
    what, detail = launch_plan(args.gpus, sys.argv[1:], os.environ)
    if what == "error":
        print(f"bench.py: {detail}", file=sys.stderr)
        sys.exit(2)
    if what == "spawn":
        print(f"bench.py: starting {args.gpus} ranks: {' '.join(detail)}", file=sys.stderr,
              flush=True)
        sys.exit(relay_ranks(detail))
    args.gpus = int(os.environ.get("WORLD_SIZE", "1"))  # launch_plan checked any explicit --gpus
    if args.config in GMM_CONFIGS:
        if args.baked:
            raise SystemExit("--baked applies to the histogram / codec volumes (DESIGN.md s12)")
        return main_gmm(args)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as graft

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, (world, args.gpus)  # launch_plan refused anything else
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks need {world} GPUs, {ndev} visible")
    dev = torch.device("cuda", local_rank % max(ndev, 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    pkg = graft.load_package()
    n, nb, W, H = CONFIGS[args.config]
    m = camera_matrix(pkg, args.camera)

    stream = torch.cuda.Stream(device=dev)
    pkg.set_stream(stream)
    if args.method in (4, 5, 6):
        pkg.synthesize_codec((n, n, n), nb, CODEC_TEMPLATES, CODEC_SLOTS, SEED)
    else:
        pkg.synthesize((n, n, n), nb, SEED)
    bake_ms = None
    if args.baked:  # once per volume, outside the timed frames (C:1200-1203)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        pkg.bake_stats()
        bake_ms = (time.perf_counter() - tb) * 1e3

    lists = pkg.tiles.tile_lists(W, H, world, m)
    if world > 1 and not args.no_balance:
        lists = balanced_lists(pkg, lists, world, rank, W, H, m, args.method, dev, stream,
                               args.dist_backend)
    n_slots = lists.shape[1]
    frame = torch.zeros(W * H, dtype=torch.int32, device=dev)
    # N > 1: a ring of RING packed buffers (and gather targets on rank 0): frame f
    # renders into buffer f % RING; the render stream waits for the gathers and
    # assemblies once per RING frames (below), so each buffer's gather had up to
    # RING - 1 frames to finish.  Rank 0's frame loop with an 8-rank split, on one
    # GPU: 0.2199 ms per frame waiting every frame (ring 4), 0.2179 every 4th,
    # 0.2150 every 8th (ring 8), against 0.1984 without gather and assembly
    # (tools/host_cost.py, profiles/r04/host_cost_N8_r4h.log).
    RING = 8 if world > 1 else 1
    # N > 1: consecutive frames alternate over two render streams, so a frame's
    # launch can start while the previous one drains its last waves (the frames
    # are independent: their own ring buffers; the gathers wait on their frame's
    # stream).  Rank lists are short launches whose ramp and tail are a larger
    # share: one rank's frame period at N = 8, C0 0.196 -> 0.186 ms, C1 0.449 ->
    # 0.412, side view 0.242 -> 0.219 (tools/overlap_sim.py,
    # profiles/r04/overlap_*_r4u.log).  N = 1 keeps one stream: its per-frame
    # HIP events time each launch alone for the roofline.
    NSTREAMS = args.render_streams if args.render_streams else (2 if world > 1 else 1)
    if world == 1:
        NSTREAMS = 1
    with torch.cuda.stream(stream):
        if world > 1:
            packed = [torch.zeros(n_slots * 256, dtype=torch.int32, device=dev) for _ in range(RING)]
            recv = ([torch.empty((world, n_slots * 256), dtype=torch.int32, device=dev)
                     for _ in range(RING)] if rank == 0 else [None] * RING)
            my_list = torch.from_numpy(lists[rank].view(np.int32).copy()).to(dev)
            all_lists = torch.from_numpy(lists.view(np.int32).copy()).to(dev)
            descs = [pkg.make_desc(packed[b], W, H, m, query_method=args.method,
                                   d_tile_list=my_list, n_tiles=n_slots) for b in range(RING)]
        else:
            descs = [pkg.make_desc(frame, W, H, m, query_method=args.method)]
    desc = descs[0]
    torch.cuda.synchronize()
    assemble = torch.cuda.Stream(device=dev) if world > 1 else None
    render_streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(NSTREAMS - 1)]
    works, assembled = [None] * RING, [None] * RING

    # algorithmic bytes of one launch on this rank: the volume bytes
    # under the footprints (U*S_rec; codec: codebook + used error pairs) + pixels*4.
    # Counted before the warm-up: the counting pass marches the same footprints once,
    # so the frames that follow start with the clocks and the address translation
    # of a running frame loop (profiles/r02/loop_timing.log)
    pixels = W * H if world == 1 else int(np.sum(lists[rank] != pkg.tiles.PAD)) * 256
    u = pkg.count_footprint(desc) if args.method in (1, 2, 3) else None
    # baked frames read one f32 statistic per footprint voxel instead of the record
    rec_bytes = 4 if args.baked else nb * 4
    vol_bytes = (u * rec_bytes if u is not None
                 else pkg.footprint_bytes(desc) if args.method in (4, 5, 6) and not args.baked
                 else None)
    alg_bytes = (vol_bytes + pixels * 4) if vol_bytes is not None else None
    torch.cuda.synchronize()

    # the measured read ceiling of this GPU beside the 8 TB/s peak:
    # the resident record volume streamed by a coalesced read kernel (vr_stream_read),
    # ~50 ms of saturating reads before the warm-up frames, so those start on the
    # clocks of a loaded GPU (the frame time settles over the first ~50 ms of work,
    # DESIGN.md section 6)
    # (a codec volume, methods 4/5/6, has no record volume to stream: none)
    ceiling = None
    if world == 1 and args.method not in (4, 5, 6):
        rb, rms, rmean = pkg.stream_read(8)
        ceiling = {"kernel": "k_stream_read", "bytes": rb, "ms": round(rms, 4),
                   "mean_ms": round(rmean, 4), "GBps": round(rb / (rms * 1e-3) / 1e9, 1),
                   "frac_of_peak": round(rb / (rms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "what": "the resident record volume (pitches included) read once per "
                           "pass, 16 B per lane, fastest of 8 timed passes"}
    torch.cuda.synchronize()

    ev = []
    nframe = [0]

    def step(timed):
        b = nframe[0] % RING
        rs = render_streams[nframe[0] % NSTREAMS]
        nframe[0] += 1
        if NSTREAMS > 1:
            pkg.set_stream(rs)  # the library launches this frame on its stream
        if world > 1 and (nframe[0] - 1) % RING == 0 and nframe[0] > 1:
            # once per RING frames, on the newest gather and assembly (their
            # streams run in order, so this covers the older ones): the next
            # RING frames reuse buffers whose gathers and assemblies (frames
            # f - RING .. f - 1) are then done.  One wait per frame cost the
            # loop more (tools/host_cost.py).  Every render stream
            # waits: the next RING frames use all of them.
            w = (nframe[0] - 2) % RING
            for s_ in render_streams:
                with torch.cuda.stream(s_):
                    if works[w] is not None:
                        works[w].wait()
                    if assembled[w] is not None:
                        s_.wait_event(assembled[w])
        with torch.cuda.stream(rs):
            if world == 1:
                frame.zero_()  # C:208 (tile slots need none: misses are written as 0)
            # per-frame timing events only at N = 1: between the render, the gather
            # and the assembly streams of N > 1 they cost the frame loop ~0.1 ms per
            # frame (tools/host_cost.py); N > 1 times its renders after the loop
            timed = timed and world == 1
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(rs)
            pkg.render(descs[b])
            if timed:
                e1.record(rs)
                ev.append((e0, e1))
            if world > 1:
                works[b] = pkg.tiles.gather_packed_into(packed[b], recv[b], world, rank)
        if world > 1 and rank == 0:
            with torch.cuda.stream(assemble):
                works[b].wait()
                pkg.set_stream(assemble)
                pkg.unscatter_tiles(recv[b], all_lists, world, n_slots, frame, W, H)
                pkg.set_stream(rs)
                done = torch.cuda.Event()
                done.record(assemble)
                assembled[b] = done

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    # layout copies the view needed (micro-bricks / axis rows, include/vr.h): made
    # synchronously inside the first warm-up frame, whose extra cost this reports
    layout = pkg.layout_info()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    t_enq = time.perf_counter()  # host time to issue the K steps (host-bound if ~ t1 - t0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    pkg.set_stream(stream)  # (N > 1: the loop left the library on the last frame's stream)
    if world > 1:
        # this rank's render alone (untimed, after the loop): HIP events around 5
        # renders of its list; the line reports the max over ranks
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                pkg.render(descs[0])
                e1.record(stream)
                ev.append((e0, e1))
        torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    per_rank = None
    if world > 1:
        # every rank's (alg bytes, U, render ms, pixels), summed into a world x 4
        # table: the whole-node roofline (aggregate_roofline)
        per_rank = torch.zeros((world, 4), dtype=torch.float64,
                               device=dev if args.dist_backend == "nccl" else "cpu")
        per_rank[rank] = torch.tensor([float(alg_bytes or 0), float(u if u is not None else -1),
                                       kern_ms, float(pixels)], dtype=torch.float64)
        dist.all_reduce(per_rank)
        per_rank = per_rank.cpu().numpy()
    if args.dump_frame and rank == 0:
        np.save(args.dump_frame, frame.cpu().numpy().view(np.uint32).reshape(H, W))
    kernel = pkg.last_kernel()

    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9 if alg_bytes else None

    # HBM bytes per launch from the committed PMC passes of this same workload
    # (tools/pmc_traffic.py; FETCH_SIZE x 2 + WRITE_SIZE), only if they were
    # measured on this very libvr.so build (sha256 of the file) and kernel
    pmc, traffic_src = traffic_entry(args, kernel, world,
                                     lists_sha16(lists) if world > 1 else None, rank)
    rank_traffic = pmc.get("per_rank_hbm_bytes") if pmc and world > 1 else None
    traffic = (rank_traffic[rank] if rank_traffic else None) if world > 1 else (
        pmc.get("hbm_bytes_per_launch") if pmc else None)
    # the bounds that apply when the frame is not HBM-bound (the smaller configs)
    bounds = (compute_bounds(pkg, torch, stream, W, H, m, args.method, kern_ms, pmc)
              if world == 1 and not args.no_issue_bounds else None)

    # parity of the timed frame's view (untimed; full frames at N = 1 are checked
    # against the oracle frame of the CPU baseline below, N > 1 assembled frames
    # against rank 0's own whole-frame render)
    check = None
    if rank == 0:
        with torch.cuda.stream(stream):
            g8 = torch.zeros(W * H, dtype=torch.int32, device=dev)
            gf = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
            gn = torch.full((W * H,), -2, dtype=torch.int32, device=dev)
            pkg.render(pkg.make_desc(g8, W, H, m, query_method=args.method, d_output_f=gf,
                                     d_steps=gn))
        torch.cuda.synchronize()
        check = (g8.cpu().numpy().view(np.uint32).reshape(H, W),
                 gf.cpu().numpy().reshape(H, W, 4), gn.cpu().numpy().reshape(H, W),
                 pkg.last_kernel())

    gather_bytes = None
    if check is not None and world == 1 and args.method in (1, 2, 3):
        gather_bytes = int(check[2][check[2] > 0].astype(np.int64).sum()) * 8 * rec_bytes
    ms_per_step = elapsed / args.steps * 1e3
    value = W * H / (elapsed / args.steps) / 1e6
    phys = min(world, max(ndev, 1))
    rehearsal = world > phys
    aggregate = (aggregate_roofline(per_rank, ms_per_step, rank_traffic=rank_traffic)
                 if per_rank is not None and np.all(per_rank[:, 0] > 0) else None)
    out = None
    if rank == 0:
        cpu, parity = None, None
        if not args.no_cpu_baseline:
            # N > 1 too: the same oracle frame the N = 1 line checks, compared
            # with the frame rank 0 assembled from the ranks' tiles
            cpu, (ref, stride) = cpu_baseline(pkg, args.config, m, args.method,
                                              args.cpu_row_stride)
            parity = frame_parity(*check, ref=ref, row_stride=stride)
            parity["timed_kernel"] = kernel
            if world > 1:
                parity = assembled_parity(frame.cpu().numpy().view(np.uint32).reshape(H, W),
                                          ref, stride, world, parity)
        elif world > 1:
            got = frame.cpu().numpy().view(np.uint32).reshape(H, W)
            parity = {"against": "rank 0's whole-frame render of the same view (no oracle: "
                                 "--no-cpu-baseline)",
                      "pixels": W * H, "rgba8_mismatch": int(np.sum(got != check[0])),
                      "kernel": check[3]}
        out = {
            "metric": f"Mrays/s + fps at {n}^3 x {nb}-bin volume, {W}x{H}; % HBM roofline",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            # devices the ranks actually ran on: a gloo rehearsal of N ranks on
            # fewer GPUs is not an N-GPU measurement (scaling null)
            "physical_gpus": phys,
            "rehearsal_shared_gpus": rehearsal,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(1e3 / ms_per_step, 2),
            "host_issue_ms_per_step": round((t_enq - t0) / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": None if rehearsal else "strong",
            "vs_baseline": None,
            "dtype": "f32 (f64 decode terms)",
            "data": f"synthetic seeded distribution volume (seed {SEED}, DESIGN.md s5)",
            "config": {
                "workload": f"{n}^3 x {nb}-bin distribution volume, {W}x{H}, camera "
                            f"{args.camera}, queryMethod {args.method}",
                "volume": [n, n, n], "bins": nb, "image": [W, H], "camera": args.camera,
                "query_method": args.method, "density": 0.05,
                "statistics": ("baked once by basicDataProcessing (f32 statistics planes)"
                               if args.baked else "decoded from the records at every step"),
                "bake_ms": round(bake_ms, 3) if bake_ms is not None else None,
                "layout_copies": layout,
                "render_streams": NSTREAMS,
                "tile_deal": (None if world == 1 else "estimate" if args.no_balance
                              else "measured cost (one untimed frame)"),
                "lists_sha16": lists_sha16(lists) if world > 1 else None,
                "parallelism": f"image tiles x{world}" + (
                (" + RCCL gather" if args.dist_backend == "nccl" else " + gloo host gather")
                if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernel,
                "kernel_ms": round(kern_ms, 4),
                "alg_bytes_per_launch": int(alg_bytes) if alg_bytes else None,
                "U_records": int(u) if u is not None else None,
                "compute": bounds,
                "read_ceiling": ceiling,
                "frac_of_read_ceiling": (round(achieved / ceiling["GBps"], 4)
                                         if achieved and ceiling else None),
                "traffic_GBps": (round(traffic / (kern_ms * 1e-3) / 1e9, 1)
                                 if traffic else None),
                # informational: every sample's 8 corner records
                # as if none were shared, samples * 8 * S_rec
                "gather_bytes_per_launch": gather_bytes,
            },
            "parity": parity,
            "cpu_baseline": cpu,
        }
        if world > 1:
            # the node's line: achieved / peak / frac are the whole node's (sum of
            # the ranks' algorithmic bytes over ms_per_step against N x 8 TB/s);
            # rank 0's own launch (a smaller share: it also assembles) moves to "rank0"
            roof = out["roofline"]
            roof["rank0"] = {k: roof.pop(k) for k in ("achieved", "frac", "kernel_ms",
                                                      "alg_bytes_per_launch", "U_records")}
            roof["aggregate"] = aggregate
            roof["rank0"]["traffic"] = roof.pop("traffic")
            roof["rank0"]["traffic_GBps"] = roof.pop("traffic_GBps")
            roof["traffic"] = aggregate.get("traffic") if aggregate else None
            roof["traffic_GBps"] = aggregate.get("traffic_GBps") if aggregate else None
            roof["achieved"] = aggregate["achieved"] if aggregate else None
            roof["peak"] = aggregate["peak"] if aggregate else HBM_PEAK_GBS * world
            roof["frac"] = aggregate["frac"] if aggregate else None
            roof["render_ms_max_over_ranks"] = (aggregate["render_ms_max_over_ranks"]
                                                if aggregate else None)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
