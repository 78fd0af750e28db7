"""Independent numpy restatement of d_render (methods 1/2/3/7, 4/5/6 from decoded
codec records, 8/9/0 from flexible-block statistics) and of the flexible-block
pre-pass, for small cases.

Test infrastructure: a second, separately written reading of the reference
(volumeRender_kernel.cu = K) used to cross-check the C oracle bit for bit.
numpy float32 arithmetic is IEEE single precision without contraction, which is
the canonical arithmetic of DESIGN.md section 3; float64 is used exactly where
the reference source promotes to double.
"""
import numpy as np

f32 = np.float32
TF = np.array([[0, 0, 0, 0], [1, 0, 0, 1], [1, .5, 0, 1], [1, 1, 0, 1], [0, 1, 0, 1],
               [0, 1, 1, 1], [0, 0, 1, 1], [1, 0, 1, 1], [0, 0, 0, 0]], dtype=np.float32)
LN2 = np.float64(0.6931471805599453)


def _clamp01(u):
    return np.fmin(np.fmax(u, f32(0)), f32(1))


def _lin(u, n):
    u = _clamp01(u)
    xb = u * f32(n) - f32(0.5)
    fl = np.floor(xb)
    a = np.rint((xb - fl) * f32(256)) * f32(1.0 / 256)
    i = fl.astype(np.int64)
    return np.clip(i, 0, n - 1), np.clip(i + 1, 0, n - 1), a.astype(np.float32)


def _lin_unnorm(u, n=500):
    """unnormalised linear fetch on the 500^3 flexBlockTex, clamp (K:1691-1714)"""
    xb = u - f32(0.5)
    fl = np.floor(xb)
    a = np.rint((xb - fl) * f32(256)) * f32(1.0 / 256)
    i = fl.astype(np.int64)
    return np.clip(i, 0, n - 1), np.clip(i + 1, 0, n - 1), a.astype(np.float32)


def _point(u, n):
    u = _clamp01(u)
    return np.minimum(np.floor(u * f32(n)).astype(np.int64), n - 1)


def _lerp(a, b, t):
    return (f32(1) - t) * a + t * b


def transfer(x):
    i0, i1, a = _lin(np.asarray(x, dtype=np.float32), 9)
    return _lerp(TF[i0], TF[i1], a[..., None])


def _bw(nb):
    return (f32(0.0217) - f32(0)) / f32(nb)


def raw_mean(p):
    """p: (..., B) float32 records -> float32 (K:742-747)"""
    nb = p.shape[-1]
    bw = _bw(nb)
    mean = np.zeros(p.shape[:-1], dtype=np.float32)
    for i in range(nb):
        c = np.float64(bw * f32(i)) + np.float64(bw) / 2.0
        mean = (mean.astype(np.float64) + p[..., i].astype(np.float64) * c).astype(np.float32)
    return mean


def stat(p, comp):
    nb = p.shape[-1]
    mean = raw_mean(p)
    if comp == 0:
        return (mean.astype(np.float64) / 0.0217).astype(np.float32)
    if comp == 1:
        var = np.zeros_like(mean)
        for i in range(nb):
            d = (f32(i) / f32(nb)) * f32(0.0217) - mean
            var = var + p[..., i] * d * d
        return (var.astype(np.float64) / 0.000021).astype(np.float32)
    ent = np.zeros_like(mean)
    enorm = np.float32(np.log(np.float64(f32(nb)))) / np.float32(np.log(np.float64(f32(2))))
    for i in range(nb):
        pr = p[..., i]
        with np.errstate(divide="ignore", invalid="ignore"):
            lg = np.log(pr.astype(np.float64)).astype(np.float32).astype(np.float64) / LN2
        t = np.where(pr <= 0, 0.0, lg)
        ent = (ent.astype(np.float64) + pr.astype(np.float64) * t).astype(np.float32)
    return (-ent) / enorm


def render(vol, W, H, m, method=1, density=0.05, brightness=1.0, toff=0.0, tscale=1.0,
           m7_dims=None, footprint=None):
    """Returns (rgba float32 (H,W,4) saturated, steps int (H,W), -1 = miss).
    footprint: optional set, receives the flat indices of every voxel read by a
    trilinear footprint of a sample taken (methods 1/2/3)."""
    with np.errstate(all="ignore"):
        return _render(vol, W, H, m, method, density, brightness, toff, tscale, m7_dims,
                       footprint)


def _render(vol, W, H, m, method, density, brightness, toff, tscale, m7_dims, footprint):
    vol = np.asarray(vol, dtype=np.float32)
    nz, ny, nx, nb = vol.shape
    M = np.asarray(m, dtype=np.float32).reshape(12)
    ys, xs = np.mgrid[0:H, 0:W]
    u = (xs.astype(np.float32) / f32(W)) * f32(2) - f32(1)
    v = (ys.astype(np.float32) / f32(H)) * f32(2) - f32(1)
    o = np.array([f32(0) * M[4 * r] + f32(0) * M[4 * r + 1] + f32(0) * M[4 * r + 2]
                  + f32(1) * M[4 * r + 3] for r in range(3)], dtype=np.float32)
    inv = f32(1) / np.sqrt(u * u + v * v + f32(-2) * f32(-2))
    d0 = [u * inv, v * inv, f32(-2) * inv]
    d = [d0[0] * M[4 * r] + d0[1] * M[4 * r + 1] + d0[2] * M[4 * r + 2] for r in range(3)]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        invR = [f32(1) / d[k] for k in range(3)]
        tb = [invR[k] * (f32(-1) - o[k]) for k in range(3)]
        tt = [invR[k] * (f32(1) - o[k]) for k in range(3)]
    tmn = [np.fmin(tt[k], tb[k]) for k in range(3)]
    tmx = [np.fmax(tt[k], tb[k]) for k in range(3)]
    tnear = np.fmax(np.fmax(tmn[0], tmn[1]), np.fmax(tmn[0], tmn[2]))
    tfar = np.fmin(np.fmin(tmx[0], tmx[1]), np.fmin(tmx[0], tmx[2]))
    hit = tfar > tnear
    tnear = np.where(tnear < 0, f32(0), tnear).astype(np.float32)
    pos = [o[k] + d[k] * tnear for k in range(3)]
    step = [d[k] * f32(0.01) for k in range(3)]
    t = tnear.copy()
    s = np.zeros((H, W, 4), dtype=np.float32)
    n = np.where(hit, 0, -1)
    active = hit.copy()
    dims = (nx, ny, nz)
    if method == 7:
        N = m7_dims or dims
        fpos, cpos, means = None, None, None

    def m7_refresh(mask, pos, fpos, cpos, means):
        q = [pos[k] * f32(0.5) + f32(0.5) for k in range(3)]
        nf = [np.floor(q[k] * f32(N[k])) / f32(N[k]) for k in range(3)]
        nc = [np.ceil(q[k] * f32(N[k])) / f32(N[k]) for k in range(3)]
        nm = np.zeros((H, W, 8), dtype=np.float32)
        for j in range(8):
            cx = nc[0] if j & 1 else nf[0]
            cy = nc[1] if j & 2 else nf[1]
            cz = nc[2] if j & 4 else nf[2]
            rec = vol[_point(cz, nz), _point(cy, ny), _point(cx, nx)]
            nm[..., j] = raw_mean(rec)
        if fpos is None:
            return nf, nc, nm
        for k in range(3):
            fpos[k] = np.where(mask, nf[k], fpos[k])
            cpos[k] = np.where(mask, nc[k], cpos[k])
        means = np.where(mask[..., None], nm, means)
        return fpos, cpos, means

    if method == 7:
        fpos, cpos, means = m7_refresh(hit, pos, None, None, None)
    for i in range(500):
        if not active.any():
            break
        if method == 7:
            q = [pos[k] * f32(0.5) + f32(0.5) for k in range(3)]
            out = np.zeros_like(active)
            for k in range(3):
                out |= (q[k] < fpos[k]) | (q[k] > cpos[k])
            if (out & active).any():
                fpos, cpos, means = m7_refresh(out & active, pos, fpos, cpos, means)
            with np.errstate(divide="ignore", invalid="ignore"):
                xd = (pos[0] * f32(0.5) + f32(0.5) - fpos[0]) / (cpos[0] - fpos[0])
                yd = (pos[1] * f32(0.5) + f32(0.5) - fpos[1]) / (cpos[1] - fpos[1])
                zd = (pos[2] * f32(0.5) + f32(0.5) - fpos[2]) / (cpos[2] - fpos[2])
            mn = means.astype(np.float64)

            def bl(a, b, w):
                with np.errstate(invalid="ignore"):
                    return (a.astype(np.float64) * (1.0 - w.astype(np.float64))
                            + (b * w).astype(np.float64)).astype(np.float32)
            m00 = bl(mn[..., 0].astype(np.float32), mn[..., 1].astype(np.float32), xd)
            m10 = bl(mn[..., 2].astype(np.float32), mn[..., 3].astype(np.float32), xd)
            m01 = bl(mn[..., 4].astype(np.float32), mn[..., 5].astype(np.float32), xd)
            m11 = bl(mn[..., 6].astype(np.float32), mn[..., 7].astype(np.float32), xd)
            m0 = bl(m00, m10, yd)
            m1 = bl(m01, m11, yd)
            sample = bl(m0, m1, zd) * f32(50)
        elif method in (8, 9, 0):  # K:654-680, vol = block statistics (n, n, n, 4)
            nbk = vol.shape[0]
            comp = {9: 0, 0: 1, 8: 2}[method]
            ax = [_lin_unnorm((pos[k] * f32(0.5) + f32(0.5)) * f32(nbk)) for k in range(3)]
            vals = []
            for j in range(8):
                xi = ax[0][1] if j & 1 else ax[0][0]
                yi = ax[1][1] if j & 2 else ax[1][0]
                zi = ax[2][1] if j & 4 else ax[2][0]
                ok = (xi < nbk) & (yi < nbk) & (zi < nbk)
                vals.append(np.where(ok, vol[np.minimum(zi, nbk - 1), np.minimum(yi, nbk - 1),
                                             np.minimum(xi, nbk - 1), comp], f32(0)))
            c00 = _lerp(vals[0], vals[1], ax[0][2])
            c10 = _lerp(vals[2], vals[3], ax[0][2])
            c01 = _lerp(vals[4], vals[5], ax[0][2])
            c11 = _lerp(vals[6], vals[7], ax[0][2])
            sample = _lerp(_lerp(c00, c10, ax[1][2]), _lerp(c01, c11, ax[1][2]), ax[2][2])
        else:
            comp = method - 1 if method <= 3 else method - 4
            sfun = stat if method <= 3 else codec_stat  # 4/5/6: vol = codec_decode(...)
            ax = [_lin(pos[k] * f32(0.5) + f32(0.5), dims[k]) for k in range(3)]
            vals = []
            for j in range(8):
                xi = ax[0][1] if j & 1 else ax[0][0]
                yi = ax[1][1] if j & 2 else ax[1][0]
                zi = ax[2][1] if j & 4 else ax[2][0]
                vals.append(sfun(vol[zi, yi, xi], comp))
                if footprint is not None:
                    flat = (zi * ny + yi) * nx + xi
                    footprint.update(np.unique(flat[active]).tolist())
            c00 = _lerp(vals[0], vals[1], ax[0][2])
            c10 = _lerp(vals[2], vals[3], ax[0][2])
            c01 = _lerp(vals[4], vals[5], ax[0][2])
            c11 = _lerp(vals[6], vals[7], ax[0][2])
            sample = _lerp(_lerp(c00, c10, ax[1][2]), _lerp(c01, c11, ax[1][2]), ax[2][2])
        col = transfer((sample - f32(toff)) * f32(tscale))
        cw = col[..., 3] * f32(density)
        col = np.stack([col[..., 0] * cw, col[..., 1] * cw, col[..., 2] * cw, cw], -1)
        om = f32(1) - s[..., 3]
        ns = s + col * om[..., None]
        s = np.where(active[..., None], ns, s)
        n = np.where(active, i + 1, n)
        done = s[..., 3] > f32(0.95)
        t = np.where(active & ~done, t + f32(0.01), t).astype(np.float32)
        done |= t > tfar
        active &= ~done
        pos = [np.where(active, pos[k] + step[k], pos[k]).astype(np.float32) for k in range(3)]
    out = s * f32(brightness)
    out = np.where(out > 0, np.where(out > 1, f32(1), out), f32(0))
    out = np.where(hit[..., None], out, f32(0))
    return out.astype(np.float32), n


def pack(rgba):
    r = np.asarray(rgba, dtype=np.float32)
    c = np.where(r > 0, np.where(r > 1, f32(1), r), f32(0))
    q = (c * f32(255)).astype(np.uint32)
    return (q[..., 3] << 24) | (q[..., 2] << 16) | (q[..., 1] << 8) | q[..., 0]


# ---- fractal/template codec, methods 4/5/6 (K:195-222, 775-871) ----

def codec_decode(codebook, templates, errors):
    """codebook int32 (..., 4), templates float32 (T, B), errors float32 (..., E, 2)
    -> decoded, error-corrected, normalised histograms float32 (..., B)"""
    nb = templates.shape[1]
    tid, shift, flip, ne = (codebook[..., k] for k in range(4))
    orig = templates[tid]                                     # (..., B)
    src = np.where(flip[..., None] != 0, orig[..., ::-1], orig)
    idx = (np.arange(nb) - shift[..., None]) % nb             # dec[m] = src[m - shift]
    dec = np.take_along_axis(src, idx, axis=-1).astype(np.float32)
    for j in range(errors.shape[-2]):
        use = j < ne
        b = errors[..., j, 0].astype(np.int64)
        ok = use & (b >= 0) & (b < nb)
        bb = np.where(ok, b, 0)
        cur = np.take_along_axis(dec, bb[..., None], axis=-1)[..., 0]
        new = cur + errors[..., j, 1]
        new = np.where(new < 0, f32(0), new)
        np.put_along_axis(dec, bb[..., None], np.where(ok, new, cur)[..., None], axis=-1)
    total = np.zeros(dec.shape[:-1], np.float32)
    for i in range(nb):
        total = total + dec[..., i]
    return np.where(total[..., None] > 0, dec / total[..., None], dec).astype(np.float32)


def codec_stat(dec, comp):
    """K:837-868: bin centre in both mean and variance"""
    nb = dec.shape[-1]
    if comp != 1:
        return stat(dec, comp)
    bw = _bw(nb)
    mean = raw_mean(dec)
    var = np.zeros_like(mean)
    for i in range(nb):
        c = np.float64(bw * f32(i)) + np.float64(bw) / 2.0
        d = c - mean.astype(np.float64)
        var = (var.astype(np.float64) + dec[..., i].astype(np.float64) * d * d).astype(np.float32)
    return (var.astype(np.float64) / 0.000021).astype(np.float32)


# ---- flexible-block pre-pass (dataProcessing, K:892-1126, 1142-1544) ----

def _split(x):
    out = []
    for i in range(7):
        if x & (1 << i):
            out.append((x & ~(1 << i)) + 1)
            out[-1] = (out[-1], x)
            x &= ~(1 << i)
        if x == 0:
            break
    return out


def _table(low, high):
    """span -> entry the reference's scan returns (last row with a match, first in it)"""
    best = {}
    for i in range(low.shape[0]):
        key = tuple(low[i, :3].tolist()) + tuple(high[i, :3].tolist())
        if key not in best or best[key] // 64 != i // 64:
            best[key] = i
    return best


def flex_process(t):
    """(n, n, n, 4) float32 block statistics, [z, y, x]"""
    D, bs, nb = t["dim"], t["block"], t["nbins"]
    ftab = _table(t["fractal_low"], t["fractal_high"])
    stab = _table(t["simple_low"], t["simple_high"])
    tp = np.asarray(t["templates"], np.float32)

    def span_hist(lo, hi):
        size = (hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1)
        if size >= 8:
            e = ftab[tuple(lo) + tuple(hi)]
            tid, shift, flip, ne = t["fractal_code"][e].tolist()
            src = tp[tid][::-1] if flip else tp[tid]
            dec = np.roll(src, shift).astype(np.float32)
            for b, v in t["fractal_err"][e][:ne].tolist():
                b = int(b)
                if 0 <= b < nb:
                    dec[b] = max(f32(dec[b] + f32(v)), f32(0)) if not np.isnan(dec[b] + f32(v)) else dec[b] + f32(v)
            tot = f32(0)
            for q in range(nb):
                tot = f32(tot + dec[q])
            return (dec / tot).astype(np.float32), size
        e = stab[tuple(x - 1 for x in lo) + tuple(x - 1 for x in hi)]
        h = np.zeros(nb, np.float32)
        for b, v in t["simple_hist"][e][:t["simple_count"][e]].tolist():
            if 0 <= int(b) < nb:
                h[int(b)] = f32(v)
        return h, size

    def corner(x, y, z):
        acc = np.zeros(nb, np.float32)
        for xs in _split(x):
            for ys in _split(y):
                for zs in _split(z):
                    h, w = span_hist((xs[0], ys[0], zs[0]), (xs[1], ys[1], zs[1]))
                    acc = (acc + h * f32(w)).astype(np.float32)
        return acc

    n = (D + bs - 1) // bs
    out = np.zeros((n, n, n, 4), np.float32)
    bw = f32(255) / f32(nb)
    enorm = f32(np.log(np.float64(f32(nb)))) / f32(np.log(2.0))
    for bz in range(n):
        for by in range(n):
            for bx in range(n):
                lo = [1 + bx * bs, 1 + by * bs, 1 + bz * bs]
                hi = [D if b == n - 1 else (b + 1) * bs for b in (bx, by, bz)]
                c = [corner(hi[0] if k & 1 else lo[0], hi[1] if k & 2 else lo[1],
                            hi[2] if k & 4 else lo[2]) for k in range(8)]
                h = c[0] + c[3] + c[4] + c[7] - c[1] - c[2] - c[5] - c[6]
                h = np.where(h < 0, f32(0), h).astype(np.float32)
                tot = f32(0)
                for q in range(nb):
                    tot = f32(tot + h[q])
                if not tot <= 0:
                    h = np.clip(h / tot, f32(0), f32(1)).astype(np.float32)
                mean = f32(0)
                for i in range(nb):
                    mean = f32(np.float64(mean) + np.float64(h[i]) *
                               (np.float64(bw * f32(i)) + np.float64(bw) / 2.0))
                var = f32(0)
                for i in range(nb):
                    dd = (np.float64(bw * f32(i)) + np.float64(bw) / 2.0) - np.float64(mean)
                    var = f32(np.float64(var) + np.float64(h[i]) * dd * dd)
                ent = f32(0)
                for i in range(nb):
                    p = h[i]
                    tt = 0.0 if p <= 0 else np.float64(f32(np.log(np.float64(p)))) / LN2
                    ent = f32(np.float64(ent) + np.float64(p) * tt)
                out[bz, by, bx] = (mean, var, f32(-ent) / enorm, 0)
    return out
