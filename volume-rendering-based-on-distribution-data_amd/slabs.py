"""Slab-chained GMM rendering: host logic of BASELINE config 5.

A 2048^3 x 16-component GMM volume is 1.65 TB: it cannot be replicated per
GPU (288 GB HBM), but split into z-slabs it is resident across 8 GPUs (one
slab of 256 slices + 1 halo slice, 207 GB, per rank).  Every ray crosses the
slabs in one order (its z step has the sign of the view's; vr_render_gmm
rejects views whose rays step both ways), so the march is a chain: slab 0
marches the camera rays and hands every ray that leaves it alive -- its exact
state: colour sums, t, position, samples taken -- to slab 1, and so on.  The
chain reproduces the whole-volume march bit for bit (same float operations in
the same order); a ray's pixel is written by the slab where it ends, and the
ranks' frames (zero elsewhere) add up to the frame.

This module has no device code: partitions, the march order and the
alive-list exchange over torch.distributed (RCCL send/recv on GPUs, gloo in
the CPU tests).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np

RAY_WORDS = 9  # alive-list entry: 36 bytes (float sum[4], t, pos[3]; u32 pixel | samples << 23)


def march_direction(inv_view, width: int, height: int) -> int:
    """+1 if every ray of the frame steps towards +z, -1 towards -z, 0 if both
    occur.  A ray's z step has the sign of u M8 + v M9 - 2 M10 (K:288-296), a
    linear form of (u, v), so the frame's four corner pixels decide."""
    M = np.asarray(inv_view, dtype=np.float32).reshape(12)
    pos = neg = 0
    for c in range(4):
        u = np.float32(np.float32((width - 1) / width) * 2 - 1) if c & 1 else np.float32(-1)
        v = np.float32(np.float32((height - 1) / height) * 2 - 1) if c & 2 else np.float32(-1)
        dz = np.float32(u * M[8] + v * M[9]) - np.float32(2) * M[10]
        pos += dz > 0
        neg += dz < 0
    if pos and neg:
        return 0
    return -1 if neg else 1


def slab_bounds(nz: int, n: int, direction: int) -> List[Tuple[int, int]]:
    """n z-ranges [z_lo, z_hi) covering [0, nz), listed in march order (the
    i-th is crossed i-th by every ray).  Equal splits (+-1 slice)."""
    if n < 1 or n > nz:
        raise ValueError(f"cannot split {nz} slices into {n} slabs")
    if direction == 0:
        raise ValueError("rays of this view cross z-slabs in both directions")
    edges = [(i * nz) // n for i in range(n + 1)]
    b = [(edges[i], edges[i + 1]) for i in range(n)]
    return b if direction > 0 else b[::-1]


def bounds_by_cost(nz: int, n: int, direction: int, bounds, costs,
                   max_slices: Optional[int] = None) -> List[Tuple[int, int]]:
    """Re-cut n slabs so every rank gets about the same march time.

    bounds/costs: a previous partition (march order) and its measured cost per
    slab (kernel ms).  Early ray termination front-loads the work (the first
    slabs a view's rays cross do most of the sampling), so equal slabs leave the
    back ranks idle.  The cost density is taken as uniform inside each measured
    slab; the cuts minimise the largest slab cost (bisection on it, greedy
    fill) with no slab holding more than max_slices slices (the HBM cap: a
    slab's records + halo must fit one GPU).  Returns n (z_lo, z_hi) ranges in
    march order covering [0, nz)."""
    if direction == 0:
        raise ValueError("rays of this view cross z-slabs in both directions")
    if n < 1 or n > nz:
        raise ValueError(f"{n} slabs cannot partition {nz} slices (1 <= n <= nz)")
    # per-slice cost in march order (slice index 0 = first crossed)
    dens = np.zeros(nz, dtype=np.float64)
    for (lo, hi), c in zip(bounds, costs):
        for z in range(lo, hi):
            k = z if direction > 0 else nz - 1 - z
            dens[k] = max(float(c), 1e-9) / (hi - lo)
    cap = nz if max_slices is None else int(max_slices)
    if cap * n < nz:
        raise ValueError(f"{n} slabs of at most {cap} slices cannot cover {nz} slices")
    pre = np.concatenate([[0.0], np.cumsum(dens)])

    def greedy(T):
        """fewest cuts with every slab's cost <= T and <= cap slices (None: > n slabs)"""
        cuts, start = [0], 0
        while start < nz:
            # furthest end with cost(start, end) <= T and end - start <= cap
            end = int(np.searchsorted(pre, pre[start] + T * (1 + 1e-12), side="right")) - 1
            end = min(max(end, start + 1), start + cap, nz)
            cuts.append(end)
            start = end
            if len(cuts) - 1 > n:
                return None
        return cuts

    lo, hi = float(dens.max()), float(pre[-1])
    for _ in range(100):  # bisection on the largest slab cost
        mid = (lo + hi) / 2
        if greedy(mid) is None:
            lo = mid
        else:
            hi = mid
    cuts = greedy(hi)
    while len(cuts) - 1 < n:  # fewer slabs needed: halve the thickest
        i = max(range(len(cuts) - 1), key=lambda j: cuts[j + 1] - cuts[j])
        cuts.insert(i + 1, (cuts[i] + cuts[i + 1]) // 2)
    march = [(cuts[i], cuts[i + 1]) for i in range(n)]  # in march-order slice indices
    # n <= nz and every halving splits a slab of >= 2 slices, so no slab is empty
    assert len(cuts) == n + 1 and all(b > a for a, b in march), march
    if direction > 0:
        return march
    return [(nz - b, nz - a) for a, b in march]


def _march_density(nz: int, direction: int, bounds, costs) -> np.ndarray:
    """per-slice cost in march order (index 0 = first crossed), uniform inside
    each measured segment (bounds in z, any order, covering [0, nz))"""
    dens = np.zeros(nz, dtype=np.float64)
    for (lo, hi), c in zip(bounds, costs):
        for z in range(lo, hi):
            k = z if direction > 0 else nz - 1 - z
            dens[k] = max(float(c), 1e-9) / (hi - lo)
    return dens


def _equal_cost_cuts(pre: np.ndarray, a: int, b: int, n: int) -> List[int]:
    """n + 1 cut points a = c0 < c1 < ... < cn = b (march-order slices) with
    about equal cost between them (pre: prefix sums of the density), every part
    at least one slice"""
    cuts = [a]
    for i in range(1, n):
        target = pre[a] + (pre[b] - pre[a]) * i / n
        c = int(np.searchsorted(pre, target, side="left"))
        c = min(max(c, cuts[-1] + 1), b - (n - i))
        cuts.append(c)
    cuts.append(b)
    return cuts


def segment_owner(n_segments: int, world: int) -> List[int]:
    """rank holding each segment of a two-segment chain (march order): the front
    segments 0 .. N-1 on ranks 0 .. N-1, the back ones N .. 2N-1 snaking back on
    N-1 .. 0, so rank r holds segments r and 2N-1-r"""
    assert n_segments == 2 * world
    return list(range(world)) + list(range(world - 1, -1, -1))


def two_segment_bounds(nz: int, world: int, direction: int, bounds=None, costs=None,
                       max_slices: Optional[int] = None) -> List[Tuple[int, int]]:
    """2N z-ranges [z_lo, z_hi) in march order for a chain in which every rank
    holds two segments (segment_owner): a thin front one and a thick back one.

    Early ray termination front-loads the work: with one slab per rank the back
    ranks idle while their slabs (at the HBM cap) still cannot take work off the
    front ones (config 5: 4.2 ms period for 19 ms of work on 8 ranks).  Here the
    volume is cut at a split S (march order) into a back region [S, nz), cut
    into N equal-thickness segments (it holds little work: the slices that
    fill the HBM), and a front region [0, S) cut so that rank r's front segment
    r carries C / N minus the cost of its back segment N-1-r (C: the frame's
    cost), i.e. every rank carries about C / N.  S is chosen for the smallest
    slowest rank, then the thinnest rank (its two segments + their halo slices,
    which must fit max_slices + 1 resident slices).  bounds/costs: a measured
    partition (any number of segments, z coordinates) and its costs; None =
    uniform cost."""
    if direction == 0:
        raise ValueError("rays of this view cross z-slabs in both directions")
    if world < 1 or 2 * world > nz:
        raise ValueError(f"{2 * world} segments cannot partition {nz} slices")
    if bounds is None:
        dens = np.ones(nz, dtype=np.float64)
    else:
        dens = _march_density(nz, direction, bounds, costs)
    pre = np.concatenate([[0.0], np.cumsum(dens)])
    total = pre[-1]
    cands = []
    for S in range(world, nz - world + 1):
        back = [S + ((nz - S) * j) // world for j in range(world + 1)]
        if any(back[j + 1] <= back[j] for j in range(world)):
            continue
        front = [0]
        for r in range(world - 1):
            j = world - 1 - r  # rank r's back segment
            want = max(total / world - (pre[back[j + 1]] - pre[back[j]]), 0.0)
            c = int(np.searchsorted(pre, pre[front[-1]] + want, side="left"))
            front.append(min(max(c, front[-1] + 1), S - (world - 1 - r)))
        front.append(S)
        if any(front[r + 1] <= front[r] for r in range(world)):
            continue
        per = [(pre[front[r + 1]] - pre[front[r]]) +
               (pre[back[world - r]] - pre[back[world - 1 - r]]) for r in range(world)]
        thick = max((front[r + 1] - front[r]) + (back[world - r] - back[world - 1 - r]) + 2
                    for r in range(world))
        if max_slices is None or thick <= max_slices + 1:
            cands.append((max(per), thick, front, back))
    if not cands:
        raise ValueError(f"no two-segment cut of {nz} slices fits {max_slices} slices per rank")
    # the cheapest slowest rank (within 2 %: slice discretisation), then the thinnest
    floor = min(c[0] for c in cands)
    _, _, front, back = min((c for c in cands if c[0] <= floor * 1.02), key=lambda c: (c[1], c[0]))
    cuts = front + back[1:]
    march = [(cuts[i], cuts[i + 1]) for i in range(2 * world)]
    if direction > 0:
        return march
    return [(nz - b, nz - a) for a, b in march]


def period_with_handoff(march_ms, rays_out, owners, world: int, frame_bytes: int,
                        link_gbs: float, ray_bytes: int = RAY_WORDS * 4):
    """Pipeline period of a slab chain from its segments' measured marches and
    the bytes its ranks exchange, at an assumed point-to-point link rate.

    march_ms[i], rays_out[i]: segment i's march time and the rays it hands on
    (march order); owners[i]: its rank.  The hand-off i -> i+1 (rays_out[i] x
    ray_bytes + the 8-byte count) crosses one xGMI link unless both segments sit
    on one rank; every rank also sends its frame (frame_bytes) into the reduce
    to rank 0.  Per rank:
      serial  = sum over its segments of (receive + march + send) + reduce:
                nothing overlaps (the chain's recv -> march -> send order);
      overlap = max(sum of marches, sum of receives, sum of sends + reduce):
                transfers on their own streams, full-duplex links.
    Returns (max serial, max overlap, per-rank rows)."""
    n = len(march_ms)
    recv, send = [0.0] * n, [0.0] * n
    for i in range(n - 1):
        if owners[i] != owners[i + 1]:
            ms = (rays_out[i] * ray_bytes + 8) / (link_gbs * 1e9) * 1e3
            send[i] += ms
            recv[i + 1] += ms
    red = frame_bytes / (link_gbs * 1e9) * 1e3
    rows = []
    for r in range(world):
        seg = [i for i in range(n) if owners[i] == r]
        m, rv, sd = (sum(v[i] for i in seg) for v in (march_ms, recv, send))
        rows.append({"rank": r, "march_ms": round(m, 4), "recv_ms": round(rv, 4),
                     "send_ms": round(sd, 4), "reduce_ms": round(red, 4),
                     "serial_ms": round(rv + m + sd + red, 4),
                     "overlap_ms": round(max(m, rv, sd + red), 4)})
    return (max(r["serial_ms"] for r in rows), max(r["overlap_ms"] for r in rows), rows)


def max_slices_for(nx: int, ny: int, ncomp: int, hbm_bytes: float, reserve: float = 0.1) -> int:
    """Largest slab (slices, excluding its halo slice) whose GMM records fit in
    hbm_bytes with a `reserve` fraction left for frame and alive-list buffers."""
    per_slice = nx * ny * 12 * ncomp
    return int(hbm_bytes * (1 - reserve) // per_slice) - 1


def resident_slices(z_lo: int, z_hi: int, nz: int) -> Tuple[int, int]:
    """(z_base, nslices) a slab must hold: footprints starting in [z_lo, z_hi)
    read slices z0 and min(z0 + 1, nz - 1), i.e. one halo slice past z_hi."""
    return z_lo, min(z_hi + 1, nz) - z_lo


def _staged(dist, group=None) -> bool:
    """gloo carries only host tensors: device buffers are staged through host
    memory (multi-rank rehearsal on one GPU; never for measurement)"""
    return dist.get_backend(group) == "gloo"


def send_alive(rays, count: int, dst: int, dist, group=None) -> None:
    """Send an alive list (first `count` rows of an (n, RAY_WORDS) int32 tensor) to rank
    dst: the count first, then the rows (RCCL point-to-point over xGMI on GPUs)."""
    import torch
    dev = "cpu" if _staged(dist, group) else rays.device
    c = torch.tensor([count], dtype=torch.int64, device=dev)
    dist.send(c, dst, group=group)
    if count:
        dist.send(rays[:count].contiguous().to(dev), dst, group=group)


class _Sends:
    """pending isends of an alive list and the tensors they read"""

    def __init__(self, works, keep):
        self.works, self.keep = works, keep

    def wait(self):
        for w in self.works:
            w.wait()
        self.works, self.keep = [], []


def isend_alive(rays, count: int, dst: int, dist, group=None) -> _Sends:
    """send_alive without blocking: the count and the rows go out as isends;
    wait() on the result before `rays` is written again (with NCCL it makes the
    calling stream wait for the transfer)"""
    import torch
    dev = "cpu" if _staged(dist, group) else rays.device
    c = torch.tensor([count], dtype=torch.int64, device=dev)
    keep, works = [c], [dist.isend(c, dst, group=group)]
    if count:
        t = rays[:count].contiguous().to(dev)
        keep.append(t)
        works.append(dist.isend(t, dst, group=group))
    return _Sends(works, keep)


def recv_alive(src: int, out, dist, group=None) -> int:
    """Receive an alive list from rank src into out ((cap, RAY_WORDS) int32 tensor);
    returns its length."""
    import torch
    dev = "cpu" if _staged(dist, group) else out.device
    c = torch.zeros(1, dtype=torch.int64, device=dev)
    dist.recv(c, src, group=group)
    n = int(c.item())
    if n > out.shape[0]:
        raise RuntimeError(f"alive list of {n} rays exceeds the buffer ({out.shape[0]})")
    if n:
        if dev == "cpu" and out.is_cuda:
            buf = torch.empty((n, out.shape[1]), dtype=out.dtype)
            dist.recv(buf, src, group=group)
            out[:n].copy_(buf)
        else:
            buf = out[:n]
            dist.recv(buf, src, group=group)
    return n


class _Done:
    def wait(self):
        return True


def two_segment_ticks(rank: int, world: int, tick: int):
    """(front frame, back frame) rank `rank` marches at `tick` of a two-segment
    chain (segment_owner): front segment `rank` of frame tick - rank, back
    segment 2N-1-rank of frame tick - (2N-1-rank).  A front segment's input was
    handed on by rank - 1 one tick earlier, a back segment's by rank + 1 one
    tick earlier (rank N-1's back input is its own front output of the tick
    before), so every wait points to an earlier tick: no rank waits on a later
    one, and in the steady state every tick completes one frame."""
    return tick - rank, tick - (2 * world - 1 - rank)


class _StagedReduce:
    """an asynchronous gloo reduce of a host copy; wait() puts the sum back into
    rank 0's device frame"""

    def __init__(self, work, host, frame, root):
        self.work, self.host, self.frame, self.root = work, host, frame, root

    def wait(self):
        if self.work is not None:
            self.work.wait()
            if self.root:
                self.frame.copy_(self.host)
            self.work = None
        return True


def reduce_frame(frame, dist, group=None, async_op=False):
    """Sum the ranks' frames on rank 0: each pixel was written by the one slab
    where its ray ended (or by none: a miss), every other rank holds 0 there.
    async_op: returns a handle whose wait() completes the reduce (RCCL: makes
    the calling stream wait for it; gloo, staged through host memory: waits and
    copies the sum into rank 0's frame) -- a rank may not block in it while
    the ranks it waits for still need this rank (the two-segment schedule's
    ranks reduce a frame at different ticks).  Without async_op it completes
    before returning."""
    if _staged(dist, group) and frame.is_cuda:
        h = frame.cpu()
        w = dist.reduce(h, 0, op=dist.ReduceOp.SUM, group=group, async_op=True)
        r = _StagedReduce(w, h, frame, dist.get_rank() == 0)
        if not async_op:
            r.wait()
        return r
    w = dist.reduce(frame, 0, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
    return w if async_op else _Done()


def chain_frame(rank: int, world: int, render_slab, rays_in, n_in: Optional[int], dist):
    """One frame of the slab chain on this rank: receive the previous slab's
    alive list (rank > 0), march this slab (render_slab(rays_in, n_in) ->
    (rays_out, n_out)), pass the alive list on (rank < world - 1).  Returns the
    number of rays this slab handed on."""
    if rank > 0:
        n_in = recv_alive(rank - 1, rays_in, dist)
    rays_out, n_out = render_slab(rays_in if rank > 0 else None, n_in if rank > 0 else 0)
    if rank < world - 1:
        send_alive(rays_out, n_out, rank + 1, dist)
    return n_out
