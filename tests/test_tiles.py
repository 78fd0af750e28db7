"""Multi-GPU image split, on CPU: tile partition properties, and the rank-0 gather
of packed tile buffers over a world_size-2 gloo process group."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("W,H", [(1920, 1080), (512, 512), (256, 256), (33, 17), (16, 16)])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_partition_covers_each_tile_once(pkg, W, H, world):
    T = pkg.tiles
    lists = T.tile_lists(W, H, world)
    assert lists.shape[0] == world
    real = lists[lists != T.PAD]
    ntiles = T.tiles_x(W) * T.tiles_y(H)
    assert sorted(real.tolist()) == list(range(ntiles))
    counts = (lists != T.PAD).sum(1)
    # +-1 block (+ ragged edge)
    assert counts.max() - counts.min() <= T.BLOCK_X * T.BLOCK_Y + T.tiles_x(W) * T.BLOCK_Y // 2


def test_partition_spreads_the_hit_region(pkg):
    """every rank gets ~1/8 of the tiles that intersect the box (C0 camera)"""
    T = pkg.tiles
    own = T.owner_of(1920, 1080, 8)
    ty, tx = np.mgrid[0:own.shape[0], 0:own.shape[1]]
    cx = (tx * T.TILE_W + T.TILE_W / 2) / 1920 * 2 - 1
    cy = (ty * T.TILE_H + T.TILE_H / 2) / 1080 * 2 - 1
    hit = (np.abs(cx) < 0.5) & (np.abs(cy) < 0.5)  # ~ the box's screen footprint
    per_rank = np.bincount(own[hit], minlength=8)
    assert per_rank.max() / per_rank.mean() < 1.1


def _unscatter_np(gathered, lists, W, H, T):
    frame = np.zeros(H * W, np.uint32)
    tx = T.tiles_x(W)
    for r in range(lists.shape[0]):
        for s, tile in enumerate(lists[r]):
            if tile == T.PAD:
                continue
            for i in range(256):
                px = (tile % tx) * T.TILE_W + i % T.TILE_W
                py = (tile // tx) * T.TILE_H + i // T.TILE_W
                if px < W and py < H:
                    frame[py * W + px] = gathered[r, s * 256 + i]
    return frame


def _worker(rank, world, port, W, H, q):
    import torch
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import __graft_entry__ as g
    T = g.load_package().tiles
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    frame = rng.integers(0, 2**32, size=H * W, dtype=np.uint64).astype(np.uint32)
    lists = T.tile_lists(W, H, world)
    tx = T.tiles_x(W)
    packed = np.zeros(lists.shape[1] * 256, np.uint32)
    for s, tile in enumerate(lists[rank]):  # this rank's "render": copy its tiles
        if tile == T.PAD:
            continue
        for i in range(256):
            px = (tile % tx) * T.TILE_W + i % T.TILE_W
            py = (tile // tx) * T.TILE_H + i // T.TILE_W
            if px < W and py < H:
                packed[s * 256 + i] = frame[py * W + px]
    t = torch.from_numpy(packed.view(np.int32).copy())
    got = T.gather_packed(t, world, rank)
    # the asynchronous form the pipelined bench uses, into a preallocated target
    recv = torch.full((world, t.numel()), -7, dtype=torch.int32) if rank == 0 else None
    T.gather_packed_into(t, recv, world, rank).wait()
    if rank == 0:
        g_np = got.numpy().view(np.uint32)
        ok = np.array_equal(_unscatter_np(g_np, lists, W, H, T), frame)
        ok = ok and np.array_equal(recv.numpy().view(np.uint32), g_np)
        q.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("W,H", [(100, 52), (64, 64)])
def test_gloo_gather_world2(pkg, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world", [1, 2, 8])
def test_lists_match_owner_and_balance_xcds(pkg, world):
    """list entry s runs on XCD s % 8: every (rank, XCD) pair gets an equal share of
    the tiles that hit the box at the C0 camera, and lists agree with owner_of"""
    T = pkg.tiles
    W, H = 1920, 1080
    lists = T.tile_lists(W, H, world)
    own = T.owner_of(W, H, world).reshape(-1)
    tx = T.tiles_x(W)
    share = np.zeros((world, T.XCDS))
    for r in range(world):
        for s, tile in enumerate(lists[r]):
            if tile == T.PAD:
                continue
            assert own[tile] == r
            cx = (tile % tx * T.TILE_W + T.TILE_W / 2) / W * 2 - 1
            cy = (tile // tx * T.TILE_H + T.TILE_H / 2) / H * 2 - 1
            share[r, s % T.XCDS] += (abs(cx) < 0.6) and (abs(cy) < 0.6)
    assert share.max() / share.mean() < 1.2, share


@pytest.mark.parametrize("world", [1, 2, 8])
def test_lists_longest_first(pkg, world):
    """with the view matrix every XCD sublist runs its blocks longest-ray first and
    the lists still cover every tile exactly once"""
    T = pkg.tiles
    W, H = 1920, 1080
    m = pkg.camera.display_inv_view((30.0, 45.0))
    lists = T.tile_lists(W, H, world, m)
    real = lists[lists != T.PAD]
    assert sorted(real.tolist()) == list(range(T.tiles_x(W) * T.tiles_y(H)))
    tx = T.tiles_x(W)
    for r in range(world):
        for g in range(T.XCDS):
            sub = [t for t in lists[r][g::T.XCDS] if t != T.PAD]
            c = [max(T.est_steps(m, W, H, (t % tx) * T.TILE_W + k * (T.TILE_W - 1) // 2,
                                 (t // tx) * T.TILE_H + T.TILE_H // 2) for k in range(3))
                 for t in sub]
            blocks = [max(c[i:i + T.BLOCK_X * T.BLOCK_Y]) for i in range(0, len(c), T.BLOCK_X * T.BLOCK_Y)]
            assert all(a >= b - 1e-6 for a, b in zip(blocks, blocks[1:]))
