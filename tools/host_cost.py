"""Per-frame host cost of bench.py's N > 1 frame loop, on one GPU (tooling).

bench.py's step() at N > 1 issues, per frame: the wait on the gather that last
read the packed buffer (a ring of RING buffers), the wait on rank 0's last
assembly, the render of this rank's tile list (ctypes -> vr_render), the
asynchronous RCCL gather, and on rank 0 the unscatter on the assembly stream
(two vr_set_stream calls, an event).  Round 3's loop also recorded two timing
events per frame and had a ring of 2; both are kept as variants here.  This replays rank 0's loop for an N-rank
split with a one-rank NCCL group (the gather of an N-rank group cannot be
issued on one GPU; a one-rank gather's host path is the same torch/RCCL call,
one peer instead of N) and reports

  * dry: the host time per frame with every render stubbed (tuning knob
    VR_DRY: the library fills the launch parameters, chooses the kernel and
    returns without launching) -- what the issuing thread costs a frame;
  * live: the frame period of the same loop with the real renders of rank 0's
    list and the unscatter of N buffers -- max(GPU, host) per frame when the
    host keeps ahead;
  * the components (render call, gather call, unscatter call) in isolation.

  python tools/host_cost.py [--config 1024x8] [--camera C0] [--world 8] [--frames 300]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="1024x8")
    ap.add_argument("--camera", default="C0")
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--port", default="29533")
    ap.add_argument("--env", default="", help="tuning knobs NAME=VALUE[,...] for the live loop")
    ap.add_argument("--streams-only", action="store_true",
                    help="only the ring-8 loop on one vs two alternating render streams")
    ap.add_argument("--priority", type=int, default=0,
                    help="torch stream priority of the render stream (-1 = high)")
    ap.add_argument("--all-ranks", action="store_true",
                    help="replay EVERY rank's frame loop as bench.py runs it (ring 8, a wait "
                         "every 8 frames, two render streams, host included): each rank's "
                         "frame period, the max over ranks and full frame / max.  Rank 0 also "
                         "copies N - 1 staged peer buffers into its gather target per frame "
                         "(device copies standing in for the xGMI receive: a lower bound of "
                         "its traffic) before the unscatter")
    ap.add_argument("--rank0-share", type=float, default=-1.0,
                    help="rank 0's work share in the cost dealing (bench.py: tiles.rank0_share; "
                         "-1 = that default, 1 = equal shares)")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", args.port)
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    import bench
    pkg = g.load_package()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n, nb, W, H = bench.CONFIGS[args.config]
    pkg.synthesize((n, n, n), nb, bench.SEED)
    for kv in filter(None, args.env.split(",")):
        k, v = kv.split("=")
        pkg.set_tuning(k, v)
    m = bench.camera_matrix(pkg, args.camera)
    N = args.world
    # the cost-dealt lists bench.py renders at N > 1 (per-tile costs of one full frame)
    full = torch.zeros(W * H, dtype=torch.int32, device=dev)
    steps = torch.full((W * H,), -1, dtype=torch.int32, device=dev)
    pkg.render(pkg.make_desc(full, W, H, m, query_method=args.method, d_steps=steps))
    share = np.ones(N)
    share[0] = pkg.tiles.rank0_share(N) if args.rank0_share < 0 else args.rank0_share
    lists = pkg.tiles.tile_lists_by_cost(W, H, N, pkg.tiles.tile_costs_from_frame(
        steps.cpu().numpy(), W, H), share=share)
    print(f"rank 0 work share {share[0]:.4f}", flush=True)
    slots = lists.shape[1]
    stream = torch.cuda.Stream(device=dev, priority=args.priority)
    assemble = torch.cuda.Stream(device=dev)
    pkg.set_stream(stream)
    frame = torch.zeros(W * H, dtype=torch.int32, device=dev)
    with torch.cuda.stream(stream):
        packed = [torch.zeros(slots * 256, dtype=torch.int32, device=dev) for _ in range(8)]
        recv1 = [torch.empty((1, slots * 256), dtype=torch.int32, device=dev) for _ in range(8)]
        recvN = torch.zeros((N, slots * 256), dtype=torch.int32, device=dev)
        my_list = torch.from_numpy(lists[0].view(np.int32).copy()).to(dev)
        all_lists = torch.from_numpy(lists.view(np.int32).copy()).to(dev)
        descs = [pkg.make_desc(packed[b], W, H, m, query_method=args.method,
                               d_tile_list=my_list, n_tiles=slots) for b in range(8)]
    torch.cuda.synchronize()
    works, assembled, ev = [None] * 8, [None] * 8, []
    nframe = [0]

    render_streams = [stream] + [torch.cuda.Stream(device=dev, priority=args.priority)
                                 for _ in range(3)]

    def step(events=False, gather=True, unscatter=True, ring=4, mode="nccl", on_render=False,
             every=1, streams=1):
        # bench.py step(), N > 1, rank 0.  mode: "nccl" the gather on the one-rank
        # group, "copy" a device copy on the assembly stream instead; on_render: the
        # unscatter of the previous frame on the render stream after this render;
        # streams: consecutive frames alternate over that many render streams
        f = nframe[0]
        b = f % ring
        nframe[0] += 1
        rs = render_streams[f % streams]
        pkg.set_stream(rs)
        # every: wait once per `every` frames, on the newest gather / assembly
        # (the NCCL and assembly streams are in order, so that covers the
        # older ones; needs ring >= every), on every render stream
        w = b if every == 1 else ((f - 1) % ring if f % every == 0 else None)
        for s in (render_streams[:streams] if every > 1 else [rs]):
            with torch.cuda.stream(s):
                if w is not None and works[w] is not None:
                    works[w].wait()
                if w is not None and assembled[w] is not None:
                    s.wait_event(assembled[w])
        with torch.cuda.stream(rs):
            if events:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(rs)
            pkg.render(descs[b])
            if events:
                e1.record(rs)
                ev.append((e0, e1))
            works[b] = (dist.gather(packed[b], gather_list=list(recv1[b].unbind(0)), dst=0,
                                    async_op=True) if gather and mode == "nccl" else None)
            if on_render and unscatter:
                pkg.unscatter_tiles(recvN, all_lists, N, slots, frame, W, H)
        if gather and mode == "copy":
            ev_r = torch.cuda.Event()
            ev_r.record(rs)
            with torch.cuda.stream(assemble):
                assemble.wait_event(ev_r)
                recv1[b][0].copy_(packed[b])
        if unscatter and not on_render:
            with torch.cuda.stream(assemble):
                if works[b] is not None:
                    works[b].wait()
                pkg.set_stream(assemble)
                pkg.unscatter_tiles(recvN, all_lists, N, slots, frame, W, H)
                pkg.set_stream(rs)
                done = torch.cuda.Event()
                done.record(assemble)
                assembled[b] = done
        else:
            assembled[b] = None

    def loop(k, **kw):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step(**kw)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        return t_issue / k * 1e3, (time.perf_counter() - t0) / k * 1e3

    def each(fn, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        dt = (time.perf_counter() - t0) / k * 1e3
        torch.cuda.synchronize()
        return dt

    if args.all_ranks:
        return all_ranks(args, pkg, torch, dist, dev, lists, m, W, H, N, slots, frame)
    print(f"{args.config} {args.camera} m{args.method}, rank 0 of {N}: {slots} slots "
          f"({slots * 256} rays), one-rank NCCL group, GPU_MAX_HW_QUEUES="
          f"{os.environ.get('GPU_MAX_HW_QUEUES', '(unset)')}, render stream priority "
          f"{args.priority}", flush=True)
    # dry: renders stubbed
    pkg.set_tuning("VR_DRY", "1")
    loop(50)
    issue, period = loop(args.frames)
    with torch.cuda.stream(stream):
        t_render = each(lambda: pkg.render(descs[0]), args.frames)
        t_gather = each(lambda: dist.gather(packed[0], gather_list=list(recv1[0].unbind(0)),
                                            dst=0, async_op=True), args.frames)
    t_unsc = each(lambda: pkg.unscatter_tiles(recvN, all_lists, N, slots, frame, W, H), args.frames)
    print(f"  dry  (renders stubbed): host issue {issue:.4f} ms/frame, period {period:.4f} ms/frame",
          flush=True)
    print(f"  host calls alone: vr_render {t_render:.4f} ms (no launch), dist.gather {t_gather:.4f} ms, "
          f"unscatter {t_unsc:.4f} ms", flush=True)
    pkg.set_tuning("VR_DRY", "0")
    variants = ({}, {"every": 4}, {"every": 8, "ring": 8}, {"mode": "copy"}, {"unscatter": False},
                {"gather": False}, {"gather": False, "unscatter": False},
                {"events": True, "gather": False, "unscatter": False})
    if args.streams_only:
        variants = ()
    variants += ({"every": 8, "ring": 8}, {"every": 8, "ring": 8, "streams": 2},
                 {"every": 8, "ring": 8, "streams": 3}, {"every": 8, "ring": 8, "streams": 4},
                 {"every": 8, "ring": 8, "gather": False, "unscatter": False},
                 {"every": 8, "ring": 8, "streams": 2, "gather": False, "unscatter": False})
    # the steady full frame (one GPU, one stream, zeroed output as bench.py N = 1)
    # in the same process, for loop speed-ups full frame / frame period
    fdesc = pkg.make_desc(frame, W, H, m, query_method=args.method)

    def full_frame():
        with torch.cuda.stream(stream):
            frame.zero_()
            pkg.render(fdesc)
    pkg.set_stream(stream)
    for _ in range(40):
        full_frame()
    t_full = each(full_frame, 100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        full_frame()
    torch.cuda.synchronize()
    t_full = (time.perf_counter() - t0) * 10.0
    print(f"  full frame (N = 1 loop, {pkg.last_kernel()}): period {t_full:.4f} ms", flush=True)
    for kw in variants:
        works[:] = [None] * 8
        assembled[:] = [None] * 8
        ev.clear()
        loop(50, **kw)
        ev.clear()
        issue, period = loop(args.frames, **kw)
        what = ",".join(f"{k}={v}" for k, v in kw.items()) or "bench step (ring 4, no events)"
        if ev:
            kern = float(np.mean([a.elapsed_time(b) for a, b in ev]))
            gap = float(np.median([ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]))
            print(f"  live [{what}] ({pkg.last_kernel()}): host issue {issue:.4f} ms/frame, frame period "
                  f"{period:.4f} ms, render (HIP events) {kern:.4f} ms, median gap between renders "
                  f"{gap:.4f} ms", flush=True)
        else:
            print(f"  live [{what}]: host issue {issue:.4f} ms/frame, frame period {period:.4f} ms"
                  f"  (full frame / period = {t_full / period:.2f}x)", flush=True)
    dist.destroy_process_group()


def all_ranks(args, pkg, torch, dist, dev, lists, m, W, H, N, slots, frame):
    """Every rank's bench.py N > 1 frame loop in turn on this GPU (tools/host_cost.py
    --all-ranks): the max over ranks of the live frame period, host issue included."""
    RING, STREAMS = 8, 2
    rs_list = [torch.cuda.Stream(device=dev) for _ in range(STREAMS)]
    assemble = torch.cuda.Stream(device=dev)
    all_lists = torch.from_numpy(lists.view(np.int32).copy()).to(dev)
    recvN = [torch.zeros((N, slots * 256), dtype=torch.int32, device=dev) for _ in range(RING)]
    peers = torch.zeros((N, slots * 256), dtype=torch.int32, device=dev)  # staged peer buffers
    recv1 = [torch.empty((1, slots * 256), dtype=torch.int32, device=dev) for _ in range(RING)]
    fdesc = pkg.make_desc(frame, W, H, m, query_method=args.method)
    st = rs_list[0]
    pkg.set_stream(st)

    def full_period(k):
        with torch.cuda.stream(st):
            for _ in range(k):
                frame.zero_()
                pkg.render(fdesc)
        torch.cuda.synchronize()
    full_period(40)
    t0 = time.perf_counter()
    full_period(100)
    t_full = (time.perf_counter() - t0) * 10.0
    print(f"{args.config} {args.camera} m{args.method}: full frame (N = 1 loop, "
          f"{pkg.last_kernel()}) period {t_full:.4f} ms; N = {N}, {slots} slots per rank, "
          f"ring {RING}, {STREAMS} render streams, one-rank NCCL gather per frame", flush=True)
    per = []
    for r in range(N):
        with torch.cuda.stream(st):
            mine = torch.from_numpy(lists[r].view(np.int32).copy()).to(dev)
            packed = [torch.zeros(slots * 256, dtype=torch.int32, device=dev) for _ in range(RING)]
            descs = [pkg.make_desc(packed[b], W, H, m, query_method=args.method, d_tile_list=mine,
                                   n_tiles=slots) for b in range(RING)]
        torch.cuda.synchronize()
        works, assembled = [None] * RING, [None] * RING
        nframe = [0]

        def step():  # bench.py step() at N > 1 for rank r
            f = nframe[0]
            b, rs = f % RING, rs_list[f % STREAMS]
            nframe[0] += 1
            pkg.set_stream(rs)
            if f % RING == 0 and f > 0:
                w = (f - 1) % RING
                for s_ in rs_list:
                    with torch.cuda.stream(s_):
                        if works[w] is not None:
                            works[w].wait()
                        if assembled[w] is not None:
                            s_.wait_event(assembled[w])
            with torch.cuda.stream(rs):
                pkg.render(descs[b])
                works[b] = dist.gather(packed[b], gather_list=list(recv1[b].unbind(0)), dst=0,
                                       async_op=True)
            if r == 0:
                with torch.cuda.stream(assemble):
                    works[b].wait()
                    for j in range(1, N):  # the N - 1 peers' buffers arriving
                        recvN[b][j].copy_(peers[j])
                    pkg.set_stream(assemble)
                    pkg.unscatter_tiles(recvN[b], all_lists, N, slots, frame, W, H)
                    pkg.set_stream(rs)
                    done = torch.cuda.Event()
                    done.record(assemble)
                    assembled[b] = done

        for _ in range(50):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.frames):
            step()
        issue = (time.perf_counter() - t0) / args.frames * 1e3
        torch.cuda.synchronize()
        period = (time.perf_counter() - t0) / args.frames * 1e3
        per.append(period)
        print(f"  rank {r}: host issue {issue:.4f} ms/frame, frame period {period:.4f} ms "
              f"({pkg.last_kernel()})", flush=True)
    worst = max(per)
    print(f"  N = {N}: max over ranks {worst:.4f} ms (rank {per.index(worst)}) -> "
          f"full frame / max = {t_full / worst:.2f}x", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
