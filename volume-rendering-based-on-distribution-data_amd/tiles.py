"""Image-tile partition of one frame across GPUs, and the frame gather.

Each GPU holds a full replica of the distribution volume (<= 32 GiB, well
inside 288 GB of HBM) and ray-casts only its own tiles.  Rays are independent
(K:282-716 read only the image size, the view matrix and the read-only
volume), so the one exchange per frame is gathering the finished tiles to
rank 0 (an RCCL gather over xGMI when the process group is NCCL/RCCL).

Tiles are the 64x4-pixel tiles of the march kernel (one 256-thread
workgroup).  They are grouped in 1x4-tile blocks (64x16 px) which are dealt
to the ranks along a diagonal lattice (below), so every rank gets about the
same number of blocks spread over the whole image: only ~45 % of the pixels
hit the volume at the reference camera, so contiguous bands would be badly
unbalanced.

Inside a rank the list order matters too: workgroup s of the launch renders
list entry s and runs on XCD s % 8, each XCD with its own L2.  Block (i, j)
goes to bin (i + m j) mod 8*world (m = 3, or the next odd number coprime
with 8*world) -- rank = bin mod world, XCD = bin div
world -- a diagonal lattice that spreads every (rank, XCD) pair evenly over
the frame; the list interleaves the rank's 8 XCD sublists (entry 8*k + g =
k-th tile of XCD g) and the tiles of a block, which share footprint records,
stay in one L2.
"""
from __future__ import annotations

import numpy as np

TILE_W, TILE_H = 64, 4
PAD = 0xFFFFFFFF
BLOCK_X, BLOCK_Y = 1, 4  # tiles per block
XCDS = 8   # MI355X accelerator complex dies (workgroup b runs on XCD b % 8)


def tiles_x(width: int) -> int:
    return (width + TILE_W - 1) // TILE_W


def tiles_y(height: int) -> int:
    return (height + TILE_H - 1) // TILE_H


def _lattice_step(world_size: int) -> int:
    """row shift of the dealing lattice: odd, > 1, coprime with 8 * world_size"""
    import math
    m = 3
    while math.gcd(m, XCDS * world_size) != 1:
        m += 2
    return m


def _bin(bx: int, by: int, world_size: int) -> int:
    return (bx + _lattice_step(world_size) * by) % (XCDS * world_size)


def owner_of(width: int, height: int, world_size: int) -> np.ndarray:
    """rank owning each tile, shape (tiles_y, tiles_x)."""
    tx, ty = tiles_x(width), tiles_y(height)
    nbx, nby = (tx + BLOCK_X - 1) // BLOCK_X, (ty + BLOCK_Y - 1) // BLOCK_Y
    by, bx = np.mgrid[0:nby, 0:nbx]
    m = _lattice_step(world_size)
    block_rank = ((bx + m * by) % (XCDS * world_size)) % world_size
    return np.repeat(np.repeat(block_rank, BLOCK_Y, 0), BLOCK_X, 1)[:ty, :tx].astype(np.int64)


def est_steps(inv_view, width: int, height: int, px, py) -> np.ndarray:
    """samples a pixel's ray takes before leaving the volume (slab test, K:136-156;
    early termination ignored) -- the cost estimate of the longest-first order"""
    M = np.asarray(inv_view, dtype=np.float64).reshape(3, 4)
    u = np.asarray(px, np.float64) / width * 2 - 1
    v = np.asarray(py, np.float64) / height * 2 - 1
    inv = 1 / np.sqrt(u * u + v * v + 4)
    a = np.stack([u * inv, v * inv, -2 * inv])
    d = M[:, :3] @ a.reshape(3, -1)
    o = M[:, 3:4]
    with np.errstate(divide="ignore", invalid="ignore"):
        t1, t2 = (-1 - o) / d, (1 - o) / d
    tn = np.maximum(np.nanmax(np.minimum(t1, t2), axis=0), 0)
    tf = np.nanmin(np.maximum(t1, t2), axis=0)
    return np.where(tf > tn, (tf - tn) / 0.01, 0.0).reshape(np.shape(u))


def tile_lists(width: int, height: int, world_size: int, inv_view=None) -> np.ndarray:
    """(world_size, n_slots) uint32 tile ids, XCD-interleaved per rank (module
    docstring), PAD-padded to the longest list so every rank gathers the same
    number of bytes.  With the view matrix, each XCD's blocks are ordered
    longest-ray first (as the library orders full frames): a tile's march is a
    chain of dependent gathers, so the longest tiles must start first."""
    tx, ty = tiles_x(width), tiles_y(height)
    nbx, nby = (tx + BLOCK_X - 1) // BLOCK_X, (ty + BLOCK_Y - 1) // BLOCK_Y
    cost = np.zeros((nby, nbx))
    if inv_view is not None:
        gy, gx = np.mgrid[0:ty, 0:tx]
        c = np.zeros((ty, tx))
        for k in range(3):
            c = np.maximum(c, est_steps(inv_view, width, height,
                                        gx * TILE_W + k * (TILE_W - 1) // 2,
                                        gy * TILE_H + TILE_H // 2))
        pad = np.zeros((nby * BLOCK_Y, nbx * BLOCK_X))
        pad[:ty, :tx] = c
        cost = pad.reshape(nby, BLOCK_Y, nbx, BLOCK_X).max(axis=(1, 3))
    subs_blocks = [[[] for _ in range(XCDS)] for _ in range(world_size)]
    for by in range(nby):
        for bx in range(nbx):
            b = _bin(bx, by, world_size)
            subs_blocks[b % world_size][b // world_size].append((bx, by))
    ids = []
    for subs in subs_blocks:
        lists = []
        for blocks in subs:
            blocks = sorted(blocks, key=lambda q: -cost[q[1], q[0]])  # stable
            lst = []
            for bx, by in blocks:
                for y in range(by * BLOCK_Y, min(ty, by * BLOCK_Y + BLOCK_Y)):
                    for x in range(bx * BLOCK_X, min(tx, bx * BLOCK_X + BLOCK_X)):
                        lst.append(y * tx + x)
            lists.append(lst)
        longest = max((len(l) for l in lists), default=0)
        ids.append(np.array([l[i] for i in range(longest) for l in lists if i < len(l)],
                            dtype=np.uint32))
    n_slots = max((len(i) for i in ids), default=0)
    out = np.full((world_size, n_slots), PAD, dtype=np.uint32)
    for r, i in enumerate(ids):
        out[r, :len(i)] = i
    return out


def tile_costs_from_steps(steps, tile_list, n_tiles_total: int) -> np.ndarray:
    """Per-tile march cost from a render's per-pixel sample counts (d_steps).

    steps: (n_slots*256,) int32 packed like the tile buffer (-1 = miss / no
    ray), tile_list: the (n_slots,) uint32 list it was rendered with.  A tile's
    cost is what its four waves spend: per 64-pixel row (one wave), the row's
    longest ray's samples + 2 (the wave loops while any lane is live; +2 for
    ray setup and the store) -- the measure the library's own adaptive
    full-frame order records (record_tile_cost, vr_march.h).  Returns a
    (n_tiles_total,) int64 vector, zero for tiles not in the list, so ranks can
    sum their vectors into the whole frame's."""
    tl = np.asarray(tile_list, dtype=np.uint32)
    s = np.asarray(steps, dtype=np.int64).reshape(len(tl), TILE_H, TILE_W)
    row = s.max(axis=2) + 2                       # (n_slots, 4)
    cost = np.zeros(n_tiles_total, dtype=np.int64)
    ok = tl != PAD
    cost[tl[ok].astype(np.int64)] = row[ok].sum(axis=1)
    return cost


def tile_costs_from_frame(steps, width: int, height: int) -> np.ndarray:
    """tile_costs_from_steps for a full-frame render's (height, width) step map"""
    tx, ty = tiles_x(width), tiles_y(height)
    s = np.full((ty * TILE_H, tx * TILE_W), -1, dtype=np.int64)
    s[:height, :width] = np.asarray(steps, dtype=np.int64).reshape(height, width)
    packed = s.reshape(ty, TILE_H, tx, TILE_W).transpose(0, 2, 1, 3).reshape(-1)
    return tile_costs_from_steps(packed, np.arange(tx * ty, dtype=np.uint32), tx * ty)


def rank0_share(world_size: int) -> float:
    """Rank 0's share of the render work relative to the other ranks'.  Rank 0
    also receives the N - 1 peers' tile buffers and assembles the frame (the
    unscatter, on its own stream beside the next render): replaying every rank's
    bench.py frame loop on one GPU (tools/host_cost.py --all-ranks, 1024^3 x 8)
    put rank 0 ~0.02 ms per frame behind the others at every N (N = 8 C0: 0.210
    vs 0.185-0.192 ms; C1 0.460 vs 0.430-0.444), a fixed cost that is a larger
    fraction of a rank's frame as N grows."""
    return 1.0 if world_size <= 1 else max(0.5, 1.0 - 0.0125 * world_size)


def tile_lists_by_cost(width: int, height: int, world_size: int, cost,
                       block=(BLOCK_X, BLOCK_Y), share=None) -> np.ndarray:
    """Like tile_lists, but dealt by measured per-tile costs (tile_costs_from_steps
    summed over the ranks of a previous frame of the same view).

    Blocks (1x4 tiles, as in tile_lists) are taken most expensive first and each
    goes to the least loaded (rank, XCD) bin that still has room; every bin
    ends with the same number of blocks (+-1), so ranks get equal pixel counts
    (equal-size gathers) and work is balanced over all 8*world XCDs, not only
    over ranks.  A bin's blocks stay in dealing order, i.e. longest first.
    Each rank's 8 XCD sublists are PAD-padded to one length before they are
    interleaved, so list entry 8*k + g is always the k-th tile of XCD g.
    share: per-rank work weights (None = equal): a bin's load is compared as
    load / share of its rank, so a rank with share < 1 ends with the same block
    count but cheaper blocks (rank0_share: rank 0 also assembles the frame)."""
    tx, ty = tiles_x(width), tiles_y(height)
    BX, BY = int(block[0]), int(block[1])  # tiles per block (tooling sweeps other shapes)
    cost = np.asarray(cost, dtype=np.int64).reshape(ty, tx)
    nbx, nby = (tx + BX - 1) // BX, (ty + BY - 1) // BY
    pad = np.zeros((nby * BY, nbx * BX), dtype=np.int64)
    pad[:ty, :tx] = cost
    bcost = pad.reshape(nby, BY, nbx, BX).sum(axis=(1, 3)).reshape(-1)
    nbins = XCDS * world_size
    # every bin ends with lo or lo + 1 blocks, exactly `extra` of them with lo + 1
    lo, extra = divmod(len(bcost), nbins)
    order = np.argsort(-bcost, kind="stable")
    load = np.zeros(nbins, dtype=np.int64)
    count = np.zeros(nbins, dtype=np.int64)
    members = [[] for _ in range(nbins)]
    w = np.ones(world_size) if share is None else np.asarray(share, dtype=np.float64)
    if w.shape != (world_size,) or not np.all(w > 0):
        raise ValueError(f"share must hold {world_size} positive weights")
    wbin = w[np.arange(nbins) % world_size]  # bin g * world_size + r belongs to rank r
    n_plus = 0
    for b in order:
        room = (count < lo) | ((count == lo) & (n_plus < extra))
        best = int(np.argmin(np.where(room, load / wbin, np.inf)))
        n_plus += int(count[best] == lo)
        load[best] += bcost[b]
        count[best] += 1
        members[best].append(int(b))
    ids = []
    for r in range(world_size):
        lists = []
        for g in range(XCDS):
            lst = []
            for b in members[g * world_size + r]:
                by, bx = divmod(b, nbx)
                for y in range(by * BY, min(ty, by * BY + BY)):
                    for x in range(bx * BX, min(tx, bx * BX + BX)):
                        lst.append(y * tx + x)
            lists.append(lst)
        longest = max(len(l) for l in lists)
        inter = np.full((longest, XCDS), PAD, dtype=np.uint32)
        for g, l in enumerate(lists):
            inter[:len(l), g] = l
        ids.append(inter.reshape(-1))
    n_slots = max(len(i) for i in ids)
    out = np.full((world_size, n_slots), PAD, dtype=np.uint32)
    for r, i in enumerate(ids):
        out[r, :len(i)] = i
    return out


def gather_packed(packed, world_size: int, rank: int, group=None):
    """Gather every rank's packed tile buffer to rank 0.

    packed: this rank's (n_slots*256,) tensor.  Returns the (world_size,
    n_slots*256) tensor on rank 0 and None elsewhere.  One collective per
    frame; with the NCCL (= RCCL on ROCm) backend it runs over xGMI.
    """
    import torch
    import torch.distributed as dist

    if world_size == 1:
        return packed.view(1, -1)
    if packed.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device gather: stage through host memory (tests only)
        host = gather_packed(packed.cpu(), world_size, rank, group)
        return None if host is None else host.to(packed.device)
    recv = None
    if rank == 0:
        recv = torch.empty((world_size,) + tuple(packed.shape), dtype=packed.dtype,
                           device=packed.device)
        dist.gather(packed, gather_list=list(recv.unbind(0)), dst=0, group=group)
    else:
        dist.gather(packed, gather_list=None, dst=0, group=group)
    return recv


class _Done:
    """handle of a gather that has already completed on the current stream"""

    def wait(self):
        return None


def gather_packed_into(packed, recv, world_size: int, rank: int, group=None):
    """Asynchronous gather of every rank's packed tile buffer into ``recv``
    ((world_size, n_slots*256) on rank 0, None elsewhere), for frame pipelining.

    Issue it under the stream that rendered ``packed``.  With NCCL (= RCCL over
    xGMI) the collective runs on the process group's own stream after the
    render; the returned handle's ``wait()`` makes the calling stream wait for
    it (before ``packed`` is rendered into again, or before rank 0 reads
    ``recv``).  With gloo (tests) the gather is staged through host memory
    synchronously and the handle is already complete.
    """
    import torch.distributed as dist

    if world_size == 1:
        recv[0].copy_(packed)
        return _Done()
    if packed.is_cuda and dist.get_backend(group) == "gloo":
        host = gather_packed(packed.cpu(), world_size, rank, group)
        if rank == 0:
            recv.copy_(host)
        return _Done()
    if rank == 0:
        return dist.gather(packed, gather_list=list(recv.unbind(0)), dst=0, group=group,
                           async_op=True)
    return dist.gather(packed, gather_list=None, dst=0, group=group, async_op=True)
