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
        L.orc_splitmix64.argtypes = [ctypes.c_uint64]
        L.orc_splitmix64.restype = ctypes.c_uint64
        L.orc_synth_fill.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint64, fp, ctypes.c_int]
        _lib = L
    return _lib


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
