"""ctypes wrapper of the CPU oracle (oracle/vr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, by __graft_entry__.smoke() as the
checker, and by bench.py's cpu_baseline leg.  The product never imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


class RenderParams(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("inv_view", ctypes.c_float * 12),
        ("density", ctypes.c_float),
        ("brightness", ctypes.c_float),
        ("transfer_offset", ctypes.c_float),
        ("transfer_scale", ctypes.c_float),
        ("query_method", ctypes.c_int),
        ("m7_dims", ctypes.c_int * 3),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        fp = ctypes.POINTER(ctypes.c_float)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.orc_record_stats.argtypes = [fp, ctypes.c_int, fp]
        L.orc_corner_mean.argtypes = [fp, ctypes.c_int]
        L.orc_corner_mean.restype = ctypes.c_float
        L.orc_transfer.argtypes = [ctypes.c_float, fp]
        L.orc_pack.argtypes = [fp]
        L.orc_pack.restype = ctypes.c_uint32
        L.orc_render.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.POINTER(RenderParams), u32p, fp, i32p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_render.restype = ctypes.c_int64
        L.orc_count_footprint.argtypes = [fp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(RenderParams), ctypes.c_int]
        L.orc_count_footprint.restype = ctypes.c_int64
        L.orc_render_codec.argtypes = [ctypes.POINTER(Codec), ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, ctypes.POINTER(RenderParams),
                                       u32p, fp, i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_render_codec.restype = ctypes.c_int64
        L.orc_codec_decode.argtypes = [ctypes.POINTER(Codec), ctypes.c_int, ctypes.c_size_t, fp]
        L.orc_codec_stats.argtypes = [ctypes.POINTER(Codec), ctypes.c_int, ctypes.c_size_t, fp]
        L.orc_synth_codec.argtypes = [ctypes.c_int] * 6 + [ctypes.c_uint64, ctypes.c_void_p,
                                                           ctypes.c_void_p, ctypes.c_void_p]
        L.orc_splitmix64.argtypes = [ctypes.c_uint64]
        L.orc_splitmix64.restype = ctypes.c_uint64
        L.orc_max_threads.argtypes = []
        L.orc_max_threads.restype = ctypes.c_int
        L.orc_set_reading.argtypes = [ctypes.c_int] * 3
        L.orc_set_reading.restype = None
        L.orc_synth_fill.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint64, fp, ctypes.c_int]
        L.orc_flex_corner.argtypes = [ctypes.POINTER(Flex), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, fp]
        L.orc_flex_process.argtypes = [ctypes.POINTER(Flex), fp]
        L.orc_render_flex.argtypes = [fp, ctypes.c_int, ctypes.POINTER(RenderParams), u32p, fp,
                                      i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_render_flex.restype = ctypes.c_int64
        L.orc_gmm_stat.argtypes = [fp, fp, ctypes.c_int, ctypes.c_int]
        L.orc_gmm_stat.restype = ctypes.c_float
        L.orc_synth_gmm.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint64, ctypes.c_int,
                                                         ctypes.c_int, fp, fp, ctypes.c_int]
        L.orc_render_gmm.argtypes = [ctypes.POINTER(Gmm), ctypes.POINTER(RenderParams),
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.c_void_p, u32p, u32p, fp, i32p,
                                     ctypes.c_void_p]
        L.orc_render_gmm.restype = ctypes.c_int64
        L.orc_render_gmm_rows.argtypes = [ctypes.POINTER(Gmm), ctypes.POINTER(RenderParams),
                                          ctypes.c_int, ctypes.c_int, u32p, ctypes.c_int]
        L.orc_render_gmm_rows.restype = ctypes.c_int64
        L.orc_gmm_proc_new.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint64]
        L.orc_gmm_proc_new.restype = ctypes.c_void_p
        L.orc_gmm_proc_free.argtypes = [ctypes.c_void_p]
        L.orc_render_gmm_rows_proc.argtypes = [ctypes.c_void_p, ctypes.POINTER(RenderParams),
                                               i32p, ctypes.c_int, u32p, i32p, ctypes.c_int]
        L.orc_render_gmm_rows_proc.restype = ctypes.c_int64
        _lib = L
    return _lib


class Codec(ctypes.Structure):
    _fields_ = [("codebook", ctypes.POINTER(ctypes.c_int32)),
                ("templates", ctypes.POINTER(ctypes.c_float)),
                ("ntemplates", ctypes.c_int),
                ("errors", ctypes.POINTER(ctypes.c_float)),
                ("err_slots", ctypes.c_int)]


def _codec(codebook, templates, errors):
    """ctypes view of (codebook int32[..., 4], templates float32[T, B], errors float32[..., E, 2]);
    the arrays must stay alive while the struct is used"""
    c = Codec()
    c.codebook = codebook.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    c.templates = _fp(templates)
    c.ntemplates = templates.shape[0]
    c.errors = _fp(errors)
    c.err_slots = errors.shape[-2]
    return c


def codec_decode(codebook, templates, errors, vidx):
    codebook, templates, errors = _codec_arrays(codebook, templates, errors)
    out = np.zeros(templates.shape[1], np.float32)
    lib().orc_codec_decode(ctypes.byref(_codec(codebook, templates, errors)), templates.shape[1],
                           int(vidx), _fp(out))
    return out


def codec_stats(codebook, templates, errors, vidx):
    codebook, templates, errors = _codec_arrays(codebook, templates, errors)
    out = np.zeros(3, np.float32)
    lib().orc_codec_stats(ctypes.byref(_codec(codebook, templates, errors)), templates.shape[1],
                          int(vidx), _fp(out))
    return out


def _codec_arrays(codebook, templates, errors):
    return (np.ascontiguousarray(codebook, dtype=np.int32),
            np.ascontiguousarray(templates, dtype=np.float32),
            np.ascontiguousarray(errors, dtype=np.float32))


def render_codec(codebook, templates, errors, params, row_start=0, row_stride=1, nthreads=0):
    """methods 4/5/6 from a codec volume: codebook int32 (nz, ny, nx, 4), templates
    float32 (T, B), errors float32 (nz, ny, nx, E, 2).  Returns like render()."""
    codebook, templates, errors = _codec_arrays(codebook, templates, errors)
    nz, ny, nx, _ = codebook.shape
    H, W = params.height, params.width
    out = np.zeros((H, W), dtype=np.uint32)
    out_f = np.zeros((H, W, 4), dtype=np.float32)
    out_n = np.full((H, W), -2, dtype=np.int32)
    total = lib().orc_render_codec(
        ctypes.byref(_codec(codebook, templates, errors)), nx, ny, nz, templates.shape[1],
        ctypes.byref(params), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _fp(out_f),
        out_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row_start, row_stride, nthreads)
    return out, out_f, out_n, total


def synth_codec_field(nx, ny, nz, nbins, ntemplates=64, slots=4, seed=20261015):
    """the library's synthetic codec volume (vr_synthesize_codec):
    returns (codebook int32 (nz,ny,nx,4), templates float32 (T,B), errors float32
    (nz,ny,nx,slots,2))"""
    cb = np.zeros((nz, ny, nx, 4), np.int32)
    tp = np.zeros((ntemplates, nbins), np.float32)
    er = np.zeros((nz, ny, nx, max(slots, 1), 2), np.float32)[..., :slots, :].copy()
    lib().orc_synth_codec(nx, ny, nz, nbins, ntemplates, slots, seed, cb.ctypes.data,
                          tp.ctypes.data, er.ctypes.data)
    return cb, tp, er


def synth_codec(nx, ny, nz, nbins, ntemplates=24, slots=None, seed=20261015):
    """random codec volume for the parity tests (numpy PCG64, seeded): templates are
    normalised discretised Gaussians; per voxel a random template, shift, flip and
    0-4 sparse errors -- every decode branch is exercised, unlike the smooth
    synth_codec_field."""
    slots = nbins if slots is None else slots
    rng = np.random.default_rng(seed)
    mu = rng.uniform(0.1, 0.9, ntemplates)
    sig = rng.uniform(0.05, 0.3, ntemplates)
    c = (np.arange(nbins) + 0.5) / nbins
    t = np.exp(-((c[None, :] - mu[:, None]) ** 2) / (2 * sig[:, None] ** 2))
    templates = (t / t.sum(1, keepdims=True)).astype(np.float32)
    n = nx * ny * nz
    codebook = np.zeros((n, 4), np.int32)
    codebook[:, 0] = rng.integers(0, ntemplates, n)
    codebook[:, 1] = rng.integers(0, nbins, n)
    codebook[:, 2] = rng.integers(0, 2, n)
    codebook[:, 3] = rng.integers(0, min(4, slots) + 1, n)
    errors = np.zeros((n, slots, 2), np.float32)
    errors[:, :, 0] = rng.integers(0, nbins, (n, slots))
    errors[:, :, 1] = rng.uniform(-0.08, 0.08, (n, slots)).astype(np.float32)
    return (codebook.reshape(nz, ny, nx, 4), templates, errors.reshape(nz, ny, nx, slots, 2))


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def set_reading(w_trunc=0, rsqrt_ulps=0, log_ulps=0) -> None:
    """Parity-margin study only (tools/parity_margin.py): render with another
    reading of what the reference leaves open -- texture weights truncated
    (K:601/619/683), rsqrtf moved by ulps (K:295), per-bin logf moved by ulps
    (K:766).  set_reading() restores the canonical reading."""
    lib().orc_set_reading(int(w_trunc), int(rsqrt_ulps), int(log_ulps))


def max_threads() -> int:
    """omp_get_max_threads() of the oracle library in this process"""
    return int(lib().orc_max_threads())


def make_params(width, height, inv_view, density=0.05, brightness=1.0, transfer_offset=0.0,
                transfer_scale=1.0, query_method=1, m7_dims=(0, 0, 0)) -> RenderParams:
    p = RenderParams()
    p.width, p.height = int(width), int(height)
    for i, v in enumerate(np.asarray(inv_view, dtype=np.float32).reshape(12)):
        p.inv_view[i] = float(v)
    p.density, p.brightness = density, brightness
    p.transfer_offset, p.transfer_scale = transfer_offset, transfer_scale
    p.query_method = int(query_method)
    for i in range(3):
        p.m7_dims[i] = int(m7_dims[i])
    return p


def synth_volume(nx, ny, nz, nbins, seed=20261015, nthreads=0) -> np.ndarray:
    vol = np.empty((nz, ny, nx, nbins), dtype=np.float32)
    lib().orc_synth_fill(nx, ny, nz, nbins, seed, _fp(vol), nthreads)
    return vol


def render(vol: np.ndarray, params: RenderParams, row_start=0, row_stride=1, nthreads=0,
           want_float=True, want_steps=True):
    """Returns (rgba8 uint32[H,W], rgba_f float32[H,W,4] or None, steps int32[H,W] or None, total)."""
    vol = np.ascontiguousarray(vol, dtype=np.float32)
    nz, ny, nx, nb = vol.shape
    H, W = params.height, params.width
    out = np.zeros((H, W), dtype=np.uint32)
    out_f = np.zeros((H, W, 4), dtype=np.float32) if want_float else None
    out_n = np.full((H, W), -2, dtype=np.int32) if want_steps else None
    total = lib().orc_render(
        _fp(vol), nx, ny, nz, nb, ctypes.byref(params),
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
        _fp(out_f) if out_f is not None else None,
        out_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if out_n is not None else None,
        row_start, row_stride, nthreads)
    return out, out_f, out_n, total


def count_footprint(vol: np.ndarray, params: RenderParams, nthreads=0) -> int:
    vol = np.ascontiguousarray(vol, dtype=np.float32)
    nz, ny, nx, nb = vol.shape
    return int(lib().orc_count_footprint(_fp(vol), nx, ny, nz, nb, ctypes.byref(params), nthreads))


def record_stats(rec) -> np.ndarray:
    rec = np.ascontiguousarray(rec, dtype=np.float32)
    out = np.zeros(3, dtype=np.float32)
    lib().orc_record_stats(_fp(rec), rec.size, _fp(out))
    return out


def corner_mean(rec) -> float:
    rec = np.ascontiguousarray(rec, dtype=np.float32)
    return float(np.float32(lib().orc_corner_mean(_fp(rec), rec.size)))


def transfer(x: float) -> np.ndarray:
    out = np.zeros(4, dtype=np.float32)
    lib().orc_transfer(ctypes.c_float(x), _fp(out))
    return out


def pack(rgba) -> int:
    a = np.ascontiguousarray(rgba, dtype=np.float32)
    return int(lib().orc_pack(_fp(a)))


# ---- flexible blocks (methods 8/9/0): integral-histogram span tables ----

class Flex(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int), ("block", ctypes.c_int), ("nbins", ctypes.c_int),
                ("n_fractal", ctypes.c_int),
                ("fractal_low", ctypes.c_void_p), ("fractal_high", ctypes.c_void_p),
                ("fractal_code", ctypes.c_void_p), ("fractal_err", ctypes.c_void_p),
                ("n_simple", ctypes.c_int),
                ("simple_low", ctypes.c_void_p), ("simple_high", ctypes.c_void_p),
                ("simple_count", ctypes.c_void_p), ("simple_hist", ctypes.c_void_p),
                ("templates", ctypes.c_void_p), ("ntemplates", ctypes.c_int)]


FLEX_KEYS = ("fractal_low", "fractal_high", "fractal_code", "fractal_err", "simple_low",
             "simple_high", "simple_count", "simple_hist", "templates")


def flex_arrays(t: dict) -> dict:
    """contiguous typed copies of a span-table dict (keys FLEX_KEYS + dim/block/nbins)"""
    out = dict(t)
    for k in FLEX_KEYS:
        dt = np.float32 if k in ("fractal_err", "simple_hist", "templates") else np.int32
        out[k] = np.ascontiguousarray(t[k], dtype=dt)
    return out


def _flex(t: dict) -> Flex:
    f = Flex()
    f.dim, f.block, f.nbins = int(t["dim"]), int(t["block"]), int(t["nbins"])
    f.n_fractal = t["fractal_low"].shape[0]
    f.n_simple = t["simple_low"].shape[0]
    f.ntemplates = t["templates"].shape[0]
    for k in FLEX_KEYS:
        setattr(f, k, t[k].ctypes.data)
    return f


def flex_blocks_per_axis(dim, block):
    return (dim + block - 1) // block


def flex_corner(t: dict, x, y, z):
    t = flex_arrays(t)
    out = np.zeros(t["nbins"], np.float32)
    n = lib().orc_flex_corner(ctypes.byref(_flex(t)), int(x), int(y), int(z), _fp(out))
    return n, out


def flex_process(t: dict):
    """dataProcessing: (nblk, nblk, nblk, 4) float32 block statistics (mean, variance,
    entropy, 0) indexed [z, y, x]; raises if a sub-span has no table entry"""
    t = flex_arrays(t)
    nblk = flex_blocks_per_axis(t["dim"], t["block"])
    out = np.zeros((nblk, nblk, nblk, 4), np.float32)
    rc = lib().orc_flex_process(ctypes.byref(_flex(t)), _fp(out))
    if rc < 0:
        raise ValueError(f"flex pre-pass failed ({rc})")
    return out


def render_flex(blocks, params, row_start=0, row_stride=1, nthreads=0):
    """methods 8/9/0 from block statistics (nblk^3, 4).  Returns like render()."""
    blocks = np.ascontiguousarray(blocks, dtype=np.float32)
    H, W = params.height, params.width
    out = np.zeros((H, W), dtype=np.uint32)
    out_f = np.zeros((H, W, 4), dtype=np.float32)
    out_n = np.full((H, W), -2, dtype=np.int32)
    total = lib().orc_render_flex(
        _fp(blocks), blocks.shape[0], ctypes.byref(params),
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _fp(out_f),
        out_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), row_start, row_stride, nthreads)
    return out, out_f, out_n, total


def flex_split(x):
    """[1, x] as the dyadic spans of K:1248-1282, lowest set bit first"""
    out = []
    for i in range(7):
        if x & (1 << i):
            hi = x
            x &= ~(1 << i)
            out.append((x + 1, hi))
        if x == 0:
            break
    return out


def flex_needed_spans(dim, block):
    """every (low, high) 1-based span some block corner's decomposition looks up"""
    nblk = flex_blocks_per_axis(dim, block)
    coords = sorted({1 + i * block for i in range(nblk)} |
                    {min((i + 1) * block, dim) for i in range(nblk)})
    iv = sorted({s for c in coords for s in flex_split(c)})
    return [((a[0], b[0], c[0]), (a[1], b[1], c[1])) for a in iv for b in iv for c in iv]


def synth_flex(dim, block, nbins=64, ntemplates=40, seed=20261015, extra=50, dup=True):
    """random span tables (numpy PCG64) covering every span the pre-pass needs:
    spans of >= 8 voxels fractal-coded (random template, flip, shift, 0-4 errors, some
    with bin id == nbins), smaller ones as sparse simple histograms (0-based, some bin
    ids out of range); plus `extra` unreferenced entries and, with dup, duplicated
    spans placed so the reference's scan order decides which entry wins."""
    rng = np.random.default_rng(seed)
    c = (np.arange(nbins) + 0.5) / nbins
    mu, sig = rng.uniform(0.1, 0.9, ntemplates), rng.uniform(0.05, 0.3, ntemplates)
    tp = np.exp(-((c[None, :] - mu[:, None]) ** 2) / (2 * sig[:, None] ** 2))
    templates = (tp / tp.sum(1, keepdims=True)).astype(np.float32)
    frac, simp = [], []
    for lo, hi in flex_needed_spans(dim, block):
        size = (hi[0] - lo[0] + 1) * (hi[1] - lo[1] + 1) * (hi[2] - lo[2] + 1)
        (frac if size >= 8 else simp).append((lo, hi))
    for _ in range(extra):  # unreferenced decoys
        a = rng.integers(1, dim + 1, 3)
        b = np.minimum(a + rng.integers(0, 4, 3), dim)
        frac.append((tuple(a), tuple(b)))
        simp.append((tuple(a), tuple(b)))
    if dup:  # the same span again, later: the later 64-entry row wins (K:1352-1372)
        for lst in (frac, simp):
            k = len(lst)
            for j in rng.choice(k, size=min(k, 12), replace=False):
                lst.append(lst[j])
    rng.shuffle(frac)
    rng.shuffle(simp)
    nf, ns = len(frac), len(simp)
    fl = np.zeros((nf, 4), np.int32)
    fh = np.zeros((nf, 4), np.int32)
    for i, (lo, hi) in enumerate(frac):
        fl[i, :3], fh[i, :3] = lo, hi
    code = np.zeros((nf, 4), np.int32)
    code[:, 0] = rng.integers(0, ntemplates, nf)
    code[:, 1] = rng.integers(0, nbins, nf)
    code[:, 2] = rng.integers(0, 2, nf)
    code[:, 3] = rng.integers(0, 5, nf)
    ferr = np.zeros((nf, nbins, 2), np.float32)
    ferr[:, :, 0] = rng.integers(0, nbins + 1, (nf, nbins))  # nbins: out of range, skipped
    ferr[:, :, 1] = rng.uniform(-0.05, 0.05, (nf, nbins))
    sl = np.zeros((ns, 4), np.int32)
    sh = np.zeros((ns, 4), np.int32)
    for i, (lo, hi) in enumerate(simp):
        sl[i, :3] = np.asarray(lo) - 1
        sh[i, :3] = np.asarray(hi) - 1
    cnt = rng.integers(1, min(nbins, 6) + 1, ns).astype(np.int32)
    shist = np.zeros((ns, nbins, 2), np.float32)
    for i in range(ns):
        bins = rng.choice(nbins, size=cnt[i], replace=False)
        w = rng.uniform(0.1, 1.0, cnt[i])
        shist[i, :cnt[i], 0] = bins
        shist[i, :cnt[i], 1] = w / w.sum()
        if rng.uniform() < 0.05:
            shist[i, cnt[i] - 1, 0] = nbins  # out of range, skipped
    return {"dim": dim, "block": block, "nbins": nbins, "fractal_low": fl, "fractal_high": fh,
            "fractal_code": code, "fractal_err": ferr, "simple_low": sl, "simple_high": sh,
            "simple_count": cnt, "simple_hist": shist, "templates": templates}


# ---- GMM volumes (config 5) ----

class Gmm(ctypes.Structure):
    _fields_ = [("wm", ctypes.POINTER(ctypes.c_float)), ("sg", ctypes.POINTER(ctypes.c_float)),
                ("nx", ctypes.c_int), ("ny", ctypes.c_int), ("nz", ctypes.c_int),
                ("K", ctypes.c_int), ("z_base", ctypes.c_int), ("nzs", ctypes.c_int)]


GMM_RAY_WORDS = 9  # 36-byte alive-list entry as uint32 words (vr_gmm.hip GmmRay)


def synth_gmm(nx, ny, nz, K=16, seed=20261015, z_base=0, nslices=None, nthreads=0):
    """slices [z_base, z_base + nslices) of the synthetic GMM volume:
    (wm (nzs, ny, nx, K, 2), sigma (nzs, ny, nx, K)) float32"""
    if nslices is None:
        nslices = nz - z_base
    wm = np.zeros((nslices, ny, nx, K, 2), np.float32)
    sg = np.zeros((nslices, ny, nx, K), np.float32)
    lib().orc_synth_gmm(nx, ny, nz, K, seed, z_base, nslices, _fp(wm), _fp(sg), nthreads)
    return wm, sg


def gmm_stat(wm_rec, sg_rec, method):
    a = np.ascontiguousarray(wm_rec, dtype=np.float32).reshape(-1)
    b = np.ascontiguousarray(sg_rec, dtype=np.float32).reshape(-1)
    return float(lib().orc_gmm_stat(_fp(a), _fp(b), b.size, int(method)))


def render_gmm(wm, sg, dims, params, z_base=0, slab=None, rays_in=None, want_mark=False):
    """GMM render (whole volume when slab is None, else slab = (z_lo, z_hi)).
    rays_in: (n, 9) uint32 alive-list entries or None (camera rays).
    Returns dict: out (H, W) uint32, out_f (H, W, 4), out_n (H, W) int32 (-2 where
    not written), rays_out (m, 9) uint32 or None, samples, U (with want_mark)."""
    wm = np.ascontiguousarray(wm, dtype=np.float32)
    sg = np.ascontiguousarray(sg, dtype=np.float32)
    nx, ny, nz = (int(v) for v in dims)
    g = Gmm(_fp(wm), _fp(sg), nx, ny, nz, int(sg.shape[-1]), int(z_base), int(sg.shape[0]))
    W, H = params.width, params.height
    out = np.zeros((H, W), np.uint32)
    out_f = np.zeros((H, W, 4), np.float32)
    out_n = np.full((H, W), -2, np.int32)
    n_in = 0 if rays_in is None else int(rays_in.shape[0])
    cap = n_in if rays_in is not None else W * H
    rays_out = np.zeros((max(cap, 1), GMM_RAY_WORDS), np.uint32) if slab is not None else None
    n_out = ctypes.c_uint32(0)
    mark = None
    if want_mark:
        mark = np.zeros((nx * ny * nz + 63) // 64, np.uint64)
    z_lo, z_hi = (0, nz) if slab is None else slab
    rin = None if rays_in is None else np.ascontiguousarray(rays_in, dtype=np.uint32)
    samples = lib().orc_render_gmm(
        ctypes.byref(g), ctypes.byref(params), int(z_lo), int(z_hi),
        None if rin is None else rin.ctypes.data, n_in,
        None if rays_out is None else rays_out.ctypes.data, ctypes.byref(n_out),
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _fp(out_f),
        out_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
        None if mark is None else mark.ctypes.data)
    res = dict(out=out, out_f=out_f, out_n=out_n, samples=int(samples),
               rays_out=None if rays_out is None else rays_out[:n_out.value].copy())
    if mark is not None:
        res["U"] = int(np.unpackbits(mark.view(np.uint8)).sum())
    return res


def render_gmm_rows(wm, sg, dims, params, row_lo, row_hi, nthreads=0):
    """CPU-baseline GMM render of rows [row_lo, row_hi) (OpenMP); returns
    (out (H, W) uint32, samples)"""
    nx, ny, nz = (int(v) for v in dims)
    g = Gmm(_fp(wm), _fp(sg), nx, ny, nz, int(sg.shape[-1]), 0, int(sg.shape[0]))
    out = np.zeros((params.height, params.width), np.uint32)
    s = lib().orc_render_gmm_rows(ctypes.byref(g), ctypes.byref(params), int(row_lo), int(row_hi),
                                  out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), nthreads)
    return out, int(s)


def render_gmm_rows_proc(dims, K, params, rows, seed=20261015, nthreads=0):
    """whole-volume GMM render of the given frame rows with every record computed
    from its voxel index as a sample reads it (the generator of synth_gmm, no
    resident volume): for frames of volumes no host holds (config 5, 2048^3 x 16
    = 1.65 TB).  Returns (out (len(rows), W) uint32, out_n (len(rows), W) int32,
    -1 where the ray misses the box), samples"""
    nx, ny, nz = (int(v) for v in dims)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    if rows.size and (rows.min() < 0 or rows.max() >= params.height):
        raise ValueError("row outside the frame")
    W = params.width
    out = np.zeros((rows.size, W), np.uint32)
    out_n = np.zeros((rows.size, W), np.int32)
    g = lib().orc_gmm_proc_new(nx, ny, nz, int(K), int(seed))
    if not g:
        raise MemoryError("orc_gmm_proc_new")
    try:
        s = lib().orc_render_gmm_rows_proc(
            g, ctypes.byref(params), rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            int(rows.size), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
            out_n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), int(nthreads))
    finally:
        lib().orc_gmm_proc_free(g)
    if s < 0:
        raise ValueError(f"K = {K}: the GMM march takes 4..32 components")
    return out, out_n, int(s)
