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


def _synthetic_cost(pkg, W, H, seed=0):
    """per-tile costs shaped like a real view: the C0 slab-test lengths x noise"""
    T = pkg.tiles
    tx, ty = T.tiles_x(W), T.tiles_y(H)
    gy, gx = np.mgrid[0:ty, 0:tx]
    c = T.est_steps(pkg.camera.single_test_inv_view(), W, H, gx * T.TILE_W + T.TILE_W // 2,
                    gy * T.TILE_H + T.TILE_H // 2)
    rng = np.random.default_rng(seed)
    return (4 * c * rng.uniform(0.3, 1.0, c.shape) + 4).astype(np.int64).reshape(-1)


def _bin_loads(T, lists, cost):
    """(world, 8) summed cost per (rank, XCD): entry 8k+g of a list runs on XCD g"""
    out = np.zeros((lists.shape[0], T.XCDS), dtype=np.int64)
    for r, l in enumerate(lists):
        for g in range(T.XCDS):
            t = l[g::T.XCDS]
            out[r, g] = cost[t[t != T.PAD].astype(np.int64)].sum()
    return out


@pytest.mark.parametrize("W,H", [(1920, 1080), (512, 512), (33, 17), (16, 16)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cost_lists_cover_each_tile_once(pkg, W, H, world):
    T = pkg.tiles
    cost = _synthetic_cost(pkg, W, H)
    lists = T.tile_lists_by_cost(W, H, world, cost)
    real = lists[lists != T.PAD]
    assert sorted(real.tolist()) == list(range(T.tiles_x(W) * T.tiles_y(H)))
    assert lists.shape[0] == world and lists.shape[1] % T.XCDS == 0
    # equal block counts per (rank, XCD) bin, +-1 block
    nblk = np.array([[len(set((t // T.tiles_x(W)) // T.BLOCK_Y * 100000 + t % T.tiles_x(W)
                               for t in l[g::T.XCDS][l[g::T.XCDS] != T.PAD].tolist()))
                      for g in range(T.XCDS)] for l in lists])
    assert nblk.max() - nblk.min() <= 1


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cost_lists_balance_ranks_and_xcds(pkg, world):
    """measured-cost dealing balances every (rank, XCD) bin far better than the
    estimate lattice, longest blocks first inside each bin"""
    T = pkg.tiles
    W, H = 1920, 1080
    cost = _synthetic_cost(pkg, W, H, seed=world)
    by_cost = _bin_loads(T, T.tile_lists_by_cost(W, H, world, cost), cost)
    by_est = _bin_loads(T, T.tile_lists(W, H, world, pkg.camera.single_test_inv_view()), cost)
    assert by_cost.max() / by_cost.mean() < 1.01
    assert by_cost.max() <= by_est.max()
    lists = T.tile_lists_by_cost(W, H, world, cost)
    for l in lists:
        for g in range(T.XCDS):
            t = l[g::T.XCDS]
            t = t[t != T.PAD].astype(np.int64)
            blk = cost[t].reshape(-1, T.BLOCK_Y).sum(1) if len(t) % T.BLOCK_Y == 0 else None
            if blk is not None:
                assert np.all(np.diff(blk) <= 0)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cost_lists_rank0_share(pkg, world):
    """a work share below 1 for rank 0 (it also assembles the frame) gives its bins
    proportionally less cost at the same block counts (equal-size gathers), every
    tile still dealt once; the other ranks stay balanced"""
    T = pkg.tiles
    W, H = 1920, 1080
    cost = _synthetic_cost(pkg, W, H, seed=world)
    sh = T.rank0_share(world)
    assert 0.5 <= sh < 1.0 and T.rank0_share(1) == 1.0
    share = np.ones(world)
    share[0] = sh
    lists = T.tile_lists_by_cost(W, H, world, cost, share=share)
    real = lists[lists != T.PAD]
    assert sorted(real.tolist()) == list(range(T.tiles_x(W) * T.tiles_y(H)))
    eq = T.tile_lists_by_cost(W, H, world, cost)
    # one slot count for every rank (the gather stays equal-size), within a block
    # row of the equal deal's (short edge blocks may gather in rank 0's sublists)
    assert lists.shape[0] == world and abs(lists.shape[1] - eq.shape[1]) <= T.XCDS * T.BLOCK_Y
    loads = _bin_loads(T, lists, cost).sum(axis=1)
    assert abs(loads[0] / loads[1:].mean() - sh) < 0.02
    assert loads[1:].max() / loads[1:].min() < 1.01
    with pytest.raises(ValueError):
        T.tile_lists_by_cost(W, H, world, cost, share=np.zeros(world))


def test_tile_costs_from_steps(pkg):
    """per wave (64-pixel row): longest ray + 2; misses (-1) cost 1; PAD slots skipped;
    the full-frame form agrees with the packed form"""
    T = pkg.tiles
    W, H = 128, 8
    rng = np.random.default_rng(3)
    frame = rng.integers(-1, 300, size=(H, W)).astype(np.int32)
    frame[0:4, 64:128] = -1
    c = T.tile_costs_from_frame(frame, W, H)
    tx = T.tiles_x(W)
    for t in range(tx * T.tiles_y(H)):
        y0, x0 = (t // tx) * T.TILE_H, (t % tx) * T.TILE_W
        rows = frame[y0:y0 + T.TILE_H, x0:x0 + T.TILE_W]
        assert c[t] == int((rows.max(axis=1) + 2).sum())
    assert c[1] == 4
    lst = np.array([3, T.PAD, 0], dtype=np.uint32)
    packed = np.full((3, T.TILE_H, T.TILE_W), 7, dtype=np.int32)
    for s, t in enumerate(lst):
        if t != T.PAD:
            y0, x0 = (t // tx) * T.TILE_H, (t % tx) * T.TILE_W
            packed[s] = frame[y0:y0 + T.TILE_H, x0:x0 + T.TILE_W]
    cp = T.tile_costs_from_steps(packed.reshape(-1), lst, tx * T.tiles_y(H))
    assert cp[3] == c[3] and cp[0] == c[0] and cp[1] == 0 and cp[2] == 0
