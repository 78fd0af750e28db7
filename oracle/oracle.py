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
        L.orc_synth_fill.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint64, fp, ctypes.c_int]
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
