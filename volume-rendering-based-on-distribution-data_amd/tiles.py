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
"""
from __future__ import annotations

import numpy as np

TILE = 16
PAD = 0xFFFFFFFF
BLOCK = 2  # tiles per block edge


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
    """(world_size, n_slots) uint32 tile ids (row-major order per rank), PAD-padded
    to the longest list so every rank gathers the same number of bytes."""
    own = owner_of(width, height, world_size).reshape(-1)
    ids = [np.nonzero(own == r)[0].astype(np.uint32) for r in range(world_size)]
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
    recv = None
    if rank == 0:
        recv = torch.empty((world_size,) + tuple(packed.shape), dtype=packed.dtype,
                           device=packed.device)
        dist.gather(packed, gather_list=list(recv.unbind(0)), dst=0, group=group)
    else:
        dist.gather(packed, gather_list=None, dst=0, group=group)
    return recv
