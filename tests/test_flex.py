"""Flexible blocks (queryMethod 8/9/0): the dataProcessing pre-pass and its render,
on the CPU oracle (test infrastructure; the GPU parity is in test_gpu_parity.py).

The reference ships no span files and no output for these methods (SURVEY.md
8(c)), so the restatement is pinned by known answers derived from the source
(K:892-1126, 1142-1544, 654-680) and by a second, independently written numpy
restatement (tests/ref_numpy.py) that must agree bit for bit.
"""
import numpy as np
import pytest

import ref_numpy as R


def test_dyadic_split_matches_reference_loop(orc):
    """K:1248-1282: [1, x] as dyadic spans, lowest set bit first"""
    assert orc.flex_split(6) == [(5, 6), (1, 4)]
    assert orc.flex_split(64) == [(1, 64)]
    assert orc.flex_split(63) == [(63, 63), (61, 62), (57, 60), (49, 56), (33, 48), (1, 32)]
    for x in range(1, 127):
        sp = orc.flex_split(x)
        assert sp[-1][0] == 1 and sp[0][1] == x and len(sp) == bin(x).count("1")
        assert all(a[0] == b[1] + 1 for a, b in zip(sp, sp[1:]))


@pytest.mark.parametrize("dim,block,nb", [(12, 5, 16), (16, 6, 8), (20, 3, 64), (9, 9, 4)])
def test_prepass_matches_numpy_restatement(orc, dim, block, nb):
    t = orc.synth_flex(dim, block, nb, ntemplates=7, seed=dim * 100 + block)
    a = orc.flex_process(t)
    b = R.flex_process(t)
    assert a.shape == (orc.flex_blocks_per_axis(dim, block),) * 3 + (4,)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _constant_tables(orc, dim, block, q):
    """every span's histogram is q: fractal entries decode the template q as is,
    simple entries list q's non-zero bins"""
    nb = q.size
    fr, si = [], []
    for lo, hi in orc.flex_needed_spans(dim, block):
        size = np.prod(np.asarray(hi) - np.asarray(lo) + 1)
        (fr if size >= 8 else si).append((lo, hi))
    nz = np.nonzero(q)[0]
    t = {"dim": dim, "block": block, "nbins": nb,
         "fractal_low": np.array([[*lo, 0] for lo, _ in fr], np.int32).reshape(-1, 4),
         "fractal_high": np.array([[*hi, 0] for _, hi in fr], np.int32).reshape(-1, 4),
         "fractal_code": np.zeros((len(fr), 4), np.int32),
         "fractal_err": np.zeros((len(fr), nb, 2), np.float32),
         "simple_low": np.array([[*(np.asarray(lo) - 1), 0] for lo, _ in si], np.int32).reshape(-1, 4),
         "simple_high": np.array([[*(np.asarray(hi) - 1), 0] for _, hi in si], np.int32).reshape(-1, 4),
         "simple_count": np.full(len(si), nz.size, np.int32),
         "simple_hist": np.zeros((len(si), nb, 2), np.float32),
         "templates": q[None, :].astype(np.float32)}
    t["simple_hist"][:, :nz.size, 0] = nz
    t["simple_hist"][:, :nz.size, 1] = q[nz]
    return t


def test_constant_distribution_known_answer(orc):
    """all spans hold the same distribution q: every corner sum is x*y*z*q, so the
    block histogram is a multiple of q (whatever the sign pattern, when positive)
    and the statistics are q's: mean sum q_i c_i, variance sum q_i (c_i - mean)^2,
    entropy -sum q_i log2 q_i / log2 B, with c_i = (i + 1/2) 255/B (K:1084-1115)"""
    nb = 16
    q = np.zeros(nb, np.float32)
    q[[2, 3, 7, 11]] = [0.125, 0.375, 0.25, 0.25]
    t = _constant_tables(orc, 12, 4, q)
    n, corner = orc.flex_corner(t, 5, 9, 12)  # a block corner: 2 x 2 x 2 sub-spans
    assert n == 2 * 2 * 2
    np.testing.assert_allclose(corner, 5 * 9 * 12 * q, rtol=1e-6)
    blocks = orc.flex_process(t)
    c = (np.arange(nb) + 0.5) * 255.0 / nb
    mean = float(np.sum(q * c))
    var = float(np.sum(q * (c - mean) ** 2))
    ent = float(-np.sum(q[q > 0] * np.log2(q[q > 0])) / np.log2(nb))
    # blocks whose +c0+c3+c4+c7-c1-c2-c5-c6 volume is positive normalise to q
    for bz, by, bx in np.ndindex(blocks.shape[:3]):
        lo = np.array([1 + bx * 4, 1 + by * 4, 1 + bz * 4])
        hi = np.minimum(lo + 3, 12)
        v = [np.prod([hi[a] if k >> a & 1 else lo[a] for a in range(3)]) for k in range(8)]
        s = v[0] + v[3] + v[4] + v[7] - v[1] - v[2] - v[5] - v[6]
        b = blocks[bz, by, bx]
        if s > 0:
            np.testing.assert_allclose(b[:3], [mean, var, ent], rtol=2e-5)
        else:
            assert b[0] == 0 and b[1] == 0 and b[2] == 0  # clamped to 0, not normalised


def test_decode_flip_shift_errors_known_answer(orc):
    """one fractal span ([1,2]^3, 8 voxels): one-hot template at bin 3, flipped and
    shifted by 5 -> bin (B-1-3+5) mod B; an error adds to a bin (clamped at 0), an
    error on bin B (out of range) is skipped, then the sum renormalises
    (K:225-250, 1400-1431)"""
    nb = 8
    tpl = np.zeros((1, nb), np.float32)
    tpl[0, 3] = 1.0
    t = _constant_tables(orc, 2, 2, np.full(nb, 1.0 / nb, np.float32))
    t["templates"] = tpl
    i = int(np.nonzero((t["fractal_low"][:, :3] == 1).all(1) & (t["fractal_high"][:, :3] == 2).all(1))[0][0])
    t["fractal_code"][i] = (0, 5, 1, 3)
    t["fractal_err"][i, :3] = [(1, 0.5), (nb, 9.0), (4, -2.0)]  # (1 += .5), skipped, (4 -> 0)
    n, h = orc.flex_corner(t, 2, 2, 2)
    assert n == 1
    expect = np.zeros(nb, np.float32)
    expect[(nb - 1 - 3 + 5) % nb] = 1.0
    expect[1] += 0.5
    expect = expect / expect.sum() * 8
    np.testing.assert_allclose(h, expect, rtol=1e-7)


def test_duplicate_spans_resolve_like_the_reference_scan(orc):
    """K:1352-1372: `break` leaves only the x loop, so the last 64-entry row holding
    the span wins, and the first entry of that row"""
    nb = 8
    q = np.full(nb, 1.0 / nb, np.float32)
    t = _constant_tables(orc, 2, 2, q)
    i = int(np.nonzero((t["fractal_low"][:, :3] == 1).all(1) & (t["fractal_high"][:, :3] == 2).all(1))[0][0])
    nf = 200
    for k in ("fractal_low", "fractal_high", "fractal_code"):
        t[k] = np.repeat(t[k][i:i + 1], nf, 0)
    t["fractal_err"] = np.zeros((nf, nb, 2), np.float32)
    t["templates"] = np.eye(nb, dtype=np.float32)
    # entry e decodes to one-hot bin e % nb; rows: 0-63, 64-127, 128-191, 192-199
    t["fractal_code"][:, 0] = np.arange(nf) % nb
    t["fractal_code"][:, 1:] = 0
    for keep, want in ((slice(None), 192), (slice(0, 130), 128), (slice(0, 64), 0)):
        u = dict(t)
        for k in ("fractal_low", "fractal_high", "fractal_code", "fractal_err"):
            u[k] = t[k][keep]
        _, h = orc.flex_corner(u, 2, 2, 2)
        assert int(np.argmax(h)) == want % nb and h.max() == 8.0


def test_missing_span_is_an_error(orc):
    t = orc.synth_flex(10, 4, 8, dup=False, extra=0)
    t["simple_low"] = t["simple_low"][1:]
    t["simple_high"] = t["simple_high"][1:]
    t["simple_count"] = t["simple_count"][1:]
    t["simple_hist"] = t["simple_hist"][1:]
    with pytest.raises(ValueError):
        orc.flex_process(t)


@pytest.mark.parametrize("method", [8, 9, 0])
def test_flex_render_matches_numpy(orc, pkg, method):
    t = orc.synth_flex(16, 5, 16, ntemplates=5, seed=7)
    blocks = orc.flex_process(t)
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))):
        ts = {9: 1 / 255, 0: 1 / 4000, 8: 1.0}[method]
        p = orc.make_params(40, 32, cam, density=0.3, transfer_scale=ts, query_method=method)
        out, f, n, _ = orc.render_flex(blocks, p)
        rf, rn = R.render(blocks, 40, 32, cam, method, density=0.3, tscale=ts)
        assert np.array_equal(n, rn)
        assert np.array_equal(f[n >= 0].view(np.uint32), rf[n >= 0].view(np.uint32))


def test_flex_render_constant_blocks(orc, pkg):
    """every block holds the same entropy v: the centre ray of the runSingleTest
    camera (x = y = 0, d = (0, 0, -1)) samples v wherever both z texels are blocks
    and blends towards the zero texels past the last block near the front face
    (unnormalised linear fetch, K:654-680, 500^3 texture zero-filled, K:1691-1714);
    per step, composited front to back (K:683-705), restated here in float32"""
    f32 = np.float32
    n, v = 4, f32(0.5)
    blocks = np.zeros((n, n, n, 4), np.float32)
    blocks[..., 2] = v
    p = orc.make_params(2, 2, pkg.camera.single_test_inv_view(), density=0.05, query_method=8)
    out, f, steps, _ = orc.render_flex(blocks, p)
    pz, t, tfar = f32(1), f32(3), f32(5)
    s = np.zeros(4, np.float32)
    k = 0
    for k in range(1, 501):
        xb = (pz * f32(0.5) + f32(0.5)) * f32(n) - f32(0.5)
        i = int(np.floor(xb))
        a = f32(np.rint((xb - f32(np.floor(xb))) * f32(256)) / f32(256))
        t0 = v if 0 <= min(max(i, 0), 499) < n else f32(0)
        t1 = v if min(max(i + 1, 0), 499) < n else f32(0)
        smp = (f32(1) - a) * t0 + a * t1
        col = orc.transfer(float(smp)).astype(np.float32)
        col[3] = col[3] * f32(0.05)
        col[:3] = col[:3] * col[3]
        s = (s + col * (f32(1) - s[3])).astype(np.float32)
        if s[3] > f32(0.95):
            break
        t = f32(t + f32(0.01))
        if t > tfar:
            break
        pz = f32(pz + f32(-0.01))
    assert steps[1, 1] == k
    np.testing.assert_array_equal(f[1, 1], np.clip(s, 0, 1))
