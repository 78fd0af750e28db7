"""Image-tile partition of one frame across GPUs, and the frame gather.

Each GPU holds a full replica of the distribution volume (<= 32 GiB, well
inside 288 GB of HBM) and ray-casts only its own tiles.  Rays are independent
(K:282-716 read only the image size, the view matrix and the read-only
volume), so the one exchange per frame is gathering the finished tiles to
rank 0 (an RCCL gather over xGMI when the process group is NCCL/RCCL).

Tiles are the 16x16-pixel tiles of the march kernel.  They are grouped in
2x2-tile blocks (32x32 px); the blocks are enumerated along a serpentine
(boustrophedon) path over the image and dealt round-robin, so every rank gets
the same number of blocks (+-1) spread over the whole image: only ~45 % of the
pixels hit the volume at the reference camera, so contiguous bands would be
badly unbalanced.

Inside a rank the list order matters too: workgroup s of the launch renders
list entry s and runs on XCD s % 8, each XCD with its own L2.  The rank's
blocks are therefore dealt round-robin to the 8 XCDs along its serpentine
order and the list interleaves them (entry 8*i + g = i-th tile of XCD g), so
every XCD gets an equal, frame-wide share of the work while the 4 tiles of a
block -- which share footprint records -- stay in one L2.
"""
from __future__ import annotations

import numpy as np

TILE = 16
PAD = 0xFFFFFFFF
BLOCK = 2  # tiles per block edge
XCDS = 8   # MI355X accelerator complex dies (workgroup b runs on XCD b % 8)


def tiles_x(width: int) -> int:
    return (width + TILE - 1) // TILE


def tiles_y(height: int) -> int:
    return (height + TILE - 1) // TILE


def owner_of(width: int, height: int, world_size: int) -> np.ndarray:
    """rank owning each tile, shape (tiles_y, tiles_x)."""
    tx, ty = tiles_x(width), tiles_y(height)
    nbx, nby = (tx + BLOCK - 1) // BLOCK, (ty + BLOCK - 1) // BLOCK
    by, bx = np.mgrid[0:nby, 0:nbx]
    snake = np.where(by % 2 == 0, bx, nbx - 1 - bx)
    block_rank = (by * nbx + snake) % world_size
    return np.repeat(np.repeat(block_rank, BLOCK, 0), BLOCK, 1)[:ty, :tx].astype(np.int64)


def tile_lists(width: int, height: int, world_size: int) -> np.ndarray:
    """(world_size, n_slots) uint32 tile ids, XCD-interleaved per rank (module
    docstring), PAD-padded to the longest list so every rank gathers the same
    number of bytes."""
    tx, ty = tiles_x(width), tiles_y(height)
    nbx, nby = (tx + BLOCK - 1) // BLOCK, (ty + BLOCK - 1) // BLOCK
    per_rank = [[[] for _ in range(XCDS)] for _ in range(world_size)]
    j = 0
    for by in range(nby):
        for k in range(nbx):
            bx = k if by % 2 == 0 else nbx - 1 - k
            r, q = j % world_size, j // world_size   # q-th block of rank r
            j += 1
            lst = per_rank[r][q % XCDS]
            for y in range(by * BLOCK, min(ty, by * BLOCK + BLOCK)):
                for x in range(bx * BLOCK, min(tx, bx * BLOCK + BLOCK)):
                    lst.append(y * tx + x)
    ids = []
    for subs in per_rank:
        longest = max((len(l) for l in subs), default=0)
        ids.append(np.array([l[i] for i in range(longest) for l in subs if i < len(l)],
                            dtype=np.uint32))
    n_slots = max((len(i) for i in ids), default=0)
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
