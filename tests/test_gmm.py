"""GMM volumes (BASELINE config 5) -- CPU side.

The oracle's GMM restatement is pinned by known answers (single-component
mixtures, exact bin-free moments), an independent numpy restatement of the
canonical decode order, the synthetic generator's stated properties, and the
slab-chain identity (a chain of slab renders equals the whole-volume render
bit for bit).  The reference has no GMM record, so there is nothing of the
reference to pin against beyond the march semantics it shares with methods 1/2
(ray, footprint, transfer, composite): "parity unpinned" for the record decode
itself, which is this build's definition.
"""
import os
import socket

import numpy as np
import pytest


def np_fma32(a, b, c):
    # float32 fma emulated in double: a*b is exact in double; the double sum
    # rounds once more than a true fma, which can differ only at rare exact
    # float midpoints (probability ~2^-29 per operation)
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def np_gmm_stat(wm, sg, method):
    """independent restatement of the canonical lane order (vr_gmm.hip header):
    L = K/4 lanes, lane s partial over components 4s .. 4s+3, pairwise tree"""
    K = sg.shape[-1]
    L = K // 4
    w = wm.reshape(K, 2)[:, 0].astype(np.float32)
    mu = wm.reshape(K, 2)[:, 1].astype(np.float32)
    s = sg.astype(np.float32)
    pm, pq = [], []
    for lane in range(L):
        k0 = 4 * lane
        a = np.float32(w[k0] * mu[k0])
        for j in range(1, 4):
            a = np_fma32(w[k0 + j], mu[k0 + j], a)
        pm.append(a)
        q = np.float32(w[k0] * np_fma32(s[k0], s[k0], np.float32(mu[k0] * mu[k0])))
        for j in range(1, 4):
            k = k0 + j
            q = np_fma32(w[k], np_fma32(s[k], s[k], np.float32(mu[k] * mu[k])), q)
        pq.append(q)

    def tree(p):
        f = np.float32
        while len(p) > 1:  # pairwise: (p0 + p1), (p2 + p3), ... then again
            p = [f(p[i] + p[i + 1]) for i in range(0, len(p), 2)]
        return p[0]
    m = tree(pm)
    if method == 1:
        return float(m)
    return float(np.float32(np.float32(tree(pq) - np.float32(m * m)) * np.float32(16.0)))


@pytest.mark.parametrize("K", [8, 16, 32])
def test_gmm_stat_known_answers(orc, K):
    wm = np.zeros((K, 2), np.float32)
    sg = np.zeros(K, np.float32)
    # one component carries all the weight: mean = mu, variance = sigma^2
    wm[3] = (1.0, 0.375)
    sg[3] = 0.125
    sg[5] = 0.5  # weightless components contribute nothing
    wm[5, 1] = 0.9
    assert orc.gmm_stat(wm, sg, 1) == 0.375
    assert orc.gmm_stat(wm, sg, 2) == pytest.approx(16 * 0.125 ** 2, abs=1e-6)
    # two equal halves at 0.25 / 0.75, sigma 0: mean 0.5, variance 0.0625
    wm[:] = 0
    sg[:] = 0
    wm[0] = (0.5, 0.25)
    wm[K - 1] = (0.5, 0.75)
    assert orc.gmm_stat(wm, sg, 1) == 0.5
    assert orc.gmm_stat(wm, sg, 2) == pytest.approx(16 * 0.0625, abs=1e-6)


@pytest.mark.parametrize("K", [8, 16, 32])
def test_gmm_stat_matches_numpy_restatement(orc, K):
    rng = np.random.default_rng(K)
    for _ in range(200):
        r = rng.random(K).astype(np.float32) + np.float32(0.05)
        wm = np.stack([r / np.float32(r.sum()), rng.random(K).astype(np.float32)], -1)
        sg = (rng.random(K) * 0.05 + 0.005).astype(np.float32)
        for m in (1, 2):
            assert orc.gmm_stat(wm, sg, m) == np_gmm_stat(wm, sg, m)


def test_synth_gmm_properties(orc):
    wm, sg = orc.synth_gmm(20, 18, 16, 16)
    w, mu = wm[..., 0], wm[..., 1]
    assert np.all(np.abs(w.sum(-1, dtype=np.float64) - 1) < 1e-5)
    assert w.min() > 0 and mu.min() >= 0 and mu.max() <= 1
    assert sg.min() >= 0.005 and sg.max() <= 0.055
    # the mixture follows the section-5 blob field: means are not flat
    mean = (w * mu).sum(-1)
    assert mean.max() - mean.min() > 0.3
    # slices generated on their own equal the same slices of the whole volume
    part = orc.synth_gmm(20, 18, 16, 16, z_base=5, nslices=7)
    assert np.array_equal(part[0], wm[5:12]) and np.array_equal(part[1], sg[5:12])


@pytest.mark.parametrize("view", ["C0", (30.0, 45.0), (180.0, 0.0)])
@pytest.mark.parametrize("method", [1, 2])
def test_procedural_rows_equal_resident_render(orc, pkg, view, method):
    """the procedural source (records computed from the voxel index, used where
    no host holds the volume: config 5 at size, test_gpu_gmm.py) renders rows
    identical to the render of the generated volume, in any row order"""
    dims, K, W, H = (30, 26, 22), 16, 96, 64
    wm, sg = orc.synth_gmm(*dims, K, seed=7)
    m = pkg.camera.single_test_inv_view() if view == "C0" else pkg.camera.display_inv_view(view)
    p = orc.make_params(W, H, m, query_method=method, density=0.2)
    ref = orc.render_gmm(wm, sg, dims, p)
    rows = np.array([63, 0, 17, 32, 5, 17], np.int32)
    out, out_n, samples = orc.render_gmm_rows_proc(dims, K, p, rows, seed=7)
    want_n = np.where(ref["out_n"][rows] == -2, -1, ref["out_n"][rows])
    assert np.array_equal(out, ref["out"][rows]) and np.array_equal(out_n, want_n)
    assert samples == int(want_n[want_n > 0].sum()) > 0
    with pytest.raises(ValueError):
        orc.render_gmm_rows_proc(dims, K, p, np.array([H], np.int32))


def test_gmm_render_known_answers(orc, pkg):
    """constant mixtures: every sample has the same statistic, so the composite is
    the closed form of a constant-alpha ray (the methods-1/2 march semantics)"""
    nx = ny = nz = 8
    K = 8
    wm = np.zeros((nz, ny, nx, K, 2), np.float32)
    sg = np.zeros((nz, ny, nx, K), np.float32)
    wm[..., 0, :] = (1.0, 0.5)   # mean 0.5 -> TF entry 4 (green, alpha 1)
    W, H = 32, 32
    m = pkg.camera.single_test_inv_view()
    p = orc.make_params(W, H, m, query_method=1)
    r = orc.render_gmm(wm, sg, (nx, ny, nz), p)
    steps = r["out_n"]
    # centre ray: tnear = 3, tfar = 5 -> 200 samples without early exit; with
    # alpha = 0.05 per sample the ray stops at sample 59 (sum.w = 0.9515)
    assert steps[16, 16] == 59
    assert r["out_f"][16, 16, 3] == pytest.approx(1 - 0.95 ** 59, abs=1e-5)
    assert r["out_n"][0, 0] == -1  # corner pixel misses the box


def _chain(orc, wm, sg, dims, p, bounds):
    """render slab by slab (each slab from only its resident slices)"""
    nx, ny, nz = dims
    out = np.zeros((p.height, p.width), np.uint32)
    out_f = np.zeros((p.height, p.width, 4), np.float32)
    out_n = np.full((p.height, p.width), -2, np.int32)
    rays = None
    for (z_lo, z_hi) in bounds:
        zb = z_lo
        ns = min(z_hi + 1, nz) - z_lo
        r = orc.render_gmm(wm[zb:zb + ns], sg[zb:zb + ns], dims, p, z_base=zb,
                           slab=(z_lo, z_hi), rays_in=rays)
        w = r["out_n"] != -2
        out[w], out_f[w], out_n[w] = r["out"][w], r["out_f"][w], r["out_n"][w]
        rays = r["rays_out"]
    assert rays is not None and rays.shape[0] == 0  # the last slab ends every ray
    return out, out_f, out_n


@pytest.mark.parametrize("view", ["C0", (30.0, 45.0), (180.0, 0.0), (200.0, 20.0)])
@pytest.mark.parametrize("method", [1, 2])
def test_slab_chain_equals_whole_volume(orc, pkg, view, method):
    dims = (22, 18, 20)
    wm, sg = orc.synth_gmm(*dims, 16)
    m = pkg.camera.single_test_inv_view() if view == "C0" else pkg.camera.display_inv_view(view)
    W, H = 64, 48
    p = orc.make_params(W, H, m, query_method=method, density=0.3)
    full = orc.render_gmm(wm, sg, dims, p)
    direction = pkg.slabs.march_direction(m, W, H)
    assert direction != 0
    for n in (1, 2, 3, 7, dims[2]):  # down to one slice per slab
        bounds = pkg.slabs.slab_bounds(dims[2], n, direction)
        out, out_f, out_n = _chain(orc, wm, sg, dims, p, bounds)
        assert np.array_equal(out, full["out"]), f"{n} slabs: RGBA8 differs"
        assert np.array_equal(out_f, full["out_f"]), f"{n} slabs: float RGBA differs"
        assert np.array_equal(out_n, full["out_n"]), f"{n} slabs: samples differ"


def test_slab_partition_helpers(pkg):
    s = pkg.slabs
    assert s.slab_bounds(2048, 8, -1)[0] == (1792, 2048)
    b = s.slab_bounds(100, 7, 1)
    assert b[0][0] == 0 and b[-1][1] == 100
    assert all(b[i][1] == b[i + 1][0] for i in range(6))
    assert s.resident_slices(1792, 2048, 2048) == (1792, 256)
    assert s.resident_slices(0, 256, 2048) == (0, 257)
    with pytest.raises(ValueError):
        s.slab_bounds(10, 2, 0)
    # the config-5 slab with its halo: 2048 x 2048 x 257 voxels x 192 B per voxel
    assert 2048 * 2048 * 257 * 192 < 288e9 * 0.75


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _chain_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = g.load_oracle()
        pkg = g.load_package()
        dims = (18, 16, 21)
        m = pkg.camera.display_inv_view((30.0, 45.0))
        W, H = 48, 40
        p = orc.make_params(W, H, m, query_method=1, density=0.3)
        bounds = pkg.slabs.slab_bounds(dims[2], world, pkg.slabs.march_direction(m, W, H))
        z_lo, z_hi = bounds[rank]
        zb, ns = pkg.slabs.resident_slices(z_lo, z_hi, dims[2])
        wm, sg = orc.synth_gmm(*dims, 8, z_base=zb, nslices=ns)  # this rank's slab only
        frame = np.zeros((H, W), np.uint32)
        rays_in = torch.zeros((W * H, pkg.slabs.RAY_WORDS), dtype=torch.int32)

        def render_slab(rin, n_in):
            r = orc.render_gmm(wm, sg, dims, p, z_base=zb, slab=(z_lo, z_hi),
                               rays_in=None if rin is None else rin[:n_in].numpy().view(np.uint32))
            frame[:] = r["out"]
            ro = r["rays_out"]
            return torch.from_numpy(ro.view(np.int32).copy()), ro.shape[0]

        pkg.slabs.chain_frame(rank, world, render_slab, rays_in, 0, dist)
        t = torch.from_numpy(frame.view(np.int32).copy())
        dist.reduce(t, 0, op=dist.ReduceOp.SUM)  # every pixel is written by one rank
        if rank == 0:
            q.put(t.numpy().view(np.uint32).copy())
    finally:
        dist.destroy_process_group()


def test_gloo_slab_chain_matches_whole_volume(orc, pkg):
    """two ranks (gloo): rank 0 marches its slab, sends the alive list, rank 1 marches
    the rest; the summed frames equal the single-process whole-volume render"""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(120)
        assert pr.exitcode == 0
    got = q.get()
    dims = (18, 16, 21)
    wm, sg = orc.synth_gmm(*dims, 8)
    m = pkg.camera.display_inv_view((30.0, 45.0))
    full = orc.render_gmm(wm, sg, dims, orc.make_params(48, 40, m, query_method=1, density=0.3))
    assert np.array_equal(got, full["out"])


def test_bounds_by_cost(pkg):
    S = pkg.slabs
    # front-loaded costs (the measured config-5 chain): the largest slab cost drops
    b = S.slab_bounds(2048, 8, -1)
    c = [6.12, 6.56, 3.90, 1.25, 0.48, 0.08, 0.006, 0.004]
    cap = S.max_slices_for(2048, 2048, 16, 288e9)
    nb = S.bounds_by_cost(2048, 8, -1, b, c, cap)
    assert len(nb) == 8 and nb[0][1] == 2048 and nb[-1][0] == 0
    assert all(nb[i][0] == nb[i + 1][1] for i in range(7))       # contiguous, march order
    assert all(0 < hi - lo <= cap for lo, hi in nb)

    def cost(lo, hi):  # the uniform-density model the cut assumes
        return sum(cc * (min(hi, h) - max(lo, l)) / (h - l)
                   for (l, h), cc in zip(b, c) if min(hi, h) > max(lo, l))
    assert max(cost(lo, hi) for lo, hi in nb) < 0.65 * max(c)
    # uniform costs keep (nearly) equal slabs; ascending march order too
    nb = S.bounds_by_cost(100, 4, 1, S.slab_bounds(100, 4, 1), [1, 1, 1, 1])
    assert [hi - lo for lo, hi in nb] == [25, 25, 25, 25]
    with pytest.raises(ValueError):
        S.bounds_by_cost(100, 2, 1, [(0, 50), (50, 100)], [1, 1], max_slices=40)


def test_stream_bounds(pkg):
    """streamed slabs: fixed thickness, the last thinner, march order, full cover"""
    sb = pkg.stream.stream_bounds
    assert sb(10, 4, 1) == [(0, 4), (4, 8), (8, 10)]
    assert sb(10, 4, -1) == [(8, 10), (4, 8), (0, 4)]
    assert sb(3, 8, 1) == [(0, 3)]
    for nz in (1, 7, 64):
        for S in (1, 3, 64):
            b = sb(nz, S, 1)
            assert b[0][0] == 0 and b[-1][1] == nz
            assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    with pytest.raises(ValueError):
        sb(10, 0, 1)
    with pytest.raises(ValueError):
        sb(10, 4, 0)


def test_two_segment_bounds(pkg):
    """two z segments per rank: the 2N segments cover the volume in march order,
    rank r holds segments r and 2N-1-r, a front-loaded cost profile gives every
    rank about C / N (one slab per rank could not: the back slabs hit the HBM
    cap), and the thickest rank fits the cap"""
    S = pkg.slabs
    n, R = 2048, 8
    b = S.slab_bounds(n, R, -1)
    c = [5.98, 6.44, 3.74, 1.19, 0.47, 0.07, 0.0, 0.0]  # the measured equal-slab chain
    cap = S.max_slices_for(n, n, 16, 288e9)
    seg = S.two_segment_bounds(n, R, -1, b, c, cap)
    assert len(seg) == 2 * R and seg[0][1] == n and seg[-1][0] == 0
    assert all(seg[i][0] == seg[i + 1][1] for i in range(2 * R - 1))  # contiguous, march order
    own = S.segment_owner(2 * R, R)
    assert own == list(range(R)) + list(range(R - 1, -1, -1))
    dens = S._march_density(n, -1, b, c)
    pre = np.concatenate([[0.0], np.cumsum(dens)])
    per, thick = [0.0] * R, [0] * R
    for (lo, hi), r in zip(seg, own):
        per[r] += pre[n - lo] - pre[n - hi]
        thick[r] += hi - lo + 1
    assert max(per) < 1.05 * sum(c) / R
    assert max(thick) <= cap + 1
    one = S.bounds_by_cost(n, R, -1, b, c, cap)  # one slab per rank: bound by the cap
    one_max = max(pre[n - lo] - pre[n - hi] for lo, hi in one)
    assert max(per) < 0.6 * one_max
    # uniform cost: equal work per rank; ascending march order too
    seg = S.two_segment_bounds(64, 4, 1)
    assert seg[0][0] == 0 and seg[-1][1] == 64
    work = [0] * 4
    for (lo, hi), r in zip(seg, S.segment_owner(8, 4)):
        work[r] += hi - lo
    assert max(work) - min(work) <= 2
    with pytest.raises(ValueError):
        S.two_segment_bounds(n, R, -1, b, c, max_slices=200)


def test_two_segment_ticks_wait_only_on_earlier_ticks(pkg):
    """the tick schedule: every frame's 2N segments are marched in march order,
    each at a later tick than the segment it takes its alive list from, and in
    the steady state every rank marches one front and one back segment a tick"""
    S = pkg.slabs
    for R in (1, 2, 3, 8):
        when = {}
        for t in range(6 * R + 4):
            for r in range(R):
                ff, fb = S.two_segment_ticks(r, R, t)
                when[(ff, r)] = t
                when[(fb, 2 * R - 1 - r)] = t
        for f in range(3):
            ticks = [when[(f, i)] for i in range(2 * R)]  # segment i of frame f
            assert all(ticks[i + 1] == ticks[i] + 1 for i in range(2 * R - 1)), (R, ticks)


def _two_segment_worker(rank, world, port, q):
    """bench.py's --segments 2 schedule on the CPU: rank r marches front segment r
    and back segment 2N-1-r of the oracle's GMM volume at the ticks of
    slabs.two_segment_ticks, alive lists handed on by isend / recv over two gloo
    groups (forward, backward), frames summed by a reduce on a third"""
    import torch
    import torch.distributed as dist
    import __graft_entry__ as g
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = g.load_oracle()
        S = g.load_package().slabs
        pkg = g.load_package()
        dims = (18, 16, 21)
        m = pkg.camera.display_inv_view((30.0, 45.0))
        W, H, R, F = 48, 40, world, 3
        p = orc.make_params(W, H, m, query_method=1, density=0.3)
        fwd, bwd, asm = (dist.new_group(list(range(world))) for _ in range(3))
        bounds = S.two_segment_bounds(dims[2], R, S.march_direction(m, W, H))
        vols = {}
        for i in (rank, 2 * R - 1 - rank):
            zb, ns = S.resident_slices(*bounds[i], dims[2])
            vols[i] = (zb,) + orc.synth_gmm(*dims, 8, z_base=zb, nslices=ns)
        frames = {f: torch.zeros((H, W), dtype=torch.int32) for f in range(F)}
        buf_in = torch.zeros((W * H, S.RAY_WORDS), dtype=torch.int32)
        own, pend, works = {}, [], {}

        def march(i, f, rin):
            zb, wm, sg = vols[i]
            r = orc.render_gmm(wm, sg, dims, p, z_base=zb, slab=bounds[i], rays_in=rin)
            frames[f] += torch.from_numpy(r["out"].view(np.int32))  # rays ending here
            return torch.from_numpy(r["rays_out"].view(np.int32).copy())

        for t in range(F + 2 * R - 1):
            if t == 2 * R - 1:
                dist.barrier()  # as bench.py's timed window: ranks mid-pipeline
            ff, fb = S.two_segment_ticks(rank, R, t)
            if 0 <= ff < F:
                rin = None
                if rank > 0:
                    n = S.recv_alive(rank - 1, buf_in, dist, group=fwd)
                    rin = buf_in[:n].numpy().view(np.uint32).copy()
                out = march(rank, ff, rin)
                if rank < R - 1:
                    pend.append(S.isend_alive(out, out.shape[0], rank + 1, dist, group=fwd))
                else:
                    own[ff] = out
            if 0 <= fb < F:
                if rank == R - 1:
                    rin = own.pop(fb).numpy().view(np.uint32)
                else:
                    n = S.recv_alive(rank + 1, buf_in, dist, group=bwd)
                    rin = buf_in[:n].numpy().view(np.uint32).copy()
                out = march(2 * R - 1 - rank, fb, rin)
                if rank > 0:
                    pend.append(S.isend_alive(out, out.shape[0], rank - 1, dist, group=bwd))
                else:
                    assert out.shape[0] == 0
                # the rank's last touch of frame fb: its share summed on rank 0,
                # asynchronously (ranks reach a frame's reduce at different ticks)
                works[fb] = S.reduce_frame(frames[fb], dist, group=asm, async_op=True)
        for w in pend:
            w.wait()
        for w in works.values():
            w.wait()
        if rank == 0:
            q.put([frames[f].numpy().view(np.uint32).copy() for f in range(F)])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_two_segment_chain_matches_whole_volume(orc, pkg, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_two_segment_worker, args=(r, world, port, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    for pr in procs:
        pr.join(180)
        assert pr.exitcode == 0
    got = q.get()
    dims = (18, 16, 21)
    wm, sg = orc.synth_gmm(*dims, 8)
    m = pkg.camera.display_inv_view((30.0, 45.0))
    full = orc.render_gmm(wm, sg, dims, orc.make_params(48, 40, m, query_method=1, density=0.3))
    assert np.count_nonzero(full["out"]) > 0
    for f in got:
        assert np.array_equal(f, full["out"])


def test_period_with_handoff(pkg):
    """config 5's period estimate: a hand-off between two ranks costs both the
    sender and the receiver, one between two segments of one rank costs nothing,
    every rank sends its frame into the reduce"""
    S = pkg.slabs
    link = 100.0  # GB/s: 1e8 bytes = 1 ms
    march = [2.0, 1.0, 0.5, 0.25]
    rb = S.RAY_WORDS * 4  # bytes per alive-list entry (36)
    rays = [100_000_000 // rb, 40_000_000 // rb, 0, 0]  # ~1 ms and ~0.4 ms hops
    owners = [0, 1, 1, 0]  # two-segment snake of 2 ranks: 1 -> 1 is local
    serial, overlap, rows = S.period_with_handoff(march, rays, owners, 2, 10_000_000, link)
    hop0 = (rays[0] * rb + 8) / 1e8
    assert abs(rows[0]["send_ms"] - hop0) < 1e-4 and abs(rows[1]["recv_ms"] - hop0) < 1e-4
    assert rows[1]["send_ms"] == 0.0  # segment 1 -> 2 stays on rank 1
    hop2 = 8 / 1e8  # segment 2 -> 3: the count only
    assert abs(rows[0]["recv_ms"] - hop2) < 1e-4
    assert rows[0]["reduce_ms"] == 0.1
    assert abs(rows[0]["serial_ms"] - (2.25 + hop0 + hop2 + 0.1)) < 1e-3
    assert S.RAY_WORDS == 9
    assert abs(rows[1]["overlap_ms"] - 1.5) < 1e-3
    assert serial == max(r["serial_ms"] for r in rows) and overlap <= serial
