"""Python mirror of the reference's host/launch API (volumeRender.cpp:156-170).

The functions keep the reference's names, argument order and meaning and call
straight into libvr.so.  Device buffers are passed as torch CUDA tensors or as
raw device addresses (int).  Where the reference's checkCudaErrors /
getLastCudaError would have printed and exited (C:201-216, 1070), these
functions raise VRError.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import VR_ERR_ARG, Dim3, Extent, RenderDesc, VRError, check, check_last

PAD = 0xFFFFFFFF


def _ptr(buf) -> int:
    if buf is None:
        return 0
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):
        if not buf.is_cuda:
            raise ValueError("device buffer expected (a CUDA/HIP tensor)")
        if not buf.is_contiguous():
            raise ValueError("device buffer must be contiguous")
        return int(buf.data_ptr())
    raise TypeError(f"cannot take a device pointer of {type(buf)!r}")


def _extent(e) -> Extent:
    if isinstance(e, Extent):
        return e
    w, h, d = (int(v) for v in e)
    return Extent(w, h, d)


def _dim3(d) -> Dim3:
    if isinstance(d, Dim3):
        return d
    d = tuple(int(v) for v in d) + (1, 1, 1)
    return Dim3(d[0], d[1], d[2])


# ---------------------------------------------------------------- reference API

def render_kernel(gridSize, blockSize, d_output, imageW: int, imageH: int, density: float,
                  brightness: float, transferOffset: float, transferScale: float,
                  queryMethod: int, volumeSize) -> None:
    """render_kernel, K:2387-2401 (asynchronous; raises on a recorded error)."""
    _lib.load().render_kernel(_dim3(gridSize), _dim3(blockSize), _ptr(d_output), int(imageW),
                              int(imageH), float(density), float(brightness),
                              float(transferOffset), float(transferScale), int(queryMethod),
                              _extent(volumeSize))
    check_last()


def copyInvViewMatrix(invViewMatrix, sizeofMatrix: int = 48) -> None:
    """copyInvViewMatrix, K:2403-2406."""
    m = np.ascontiguousarray(np.asarray(invViewMatrix, dtype=np.float32).reshape(-1))
    if m.nbytes < sizeofMatrix:
        raise ValueError("matrix smaller than sizeofMatrix")
    _lib.load().copyInvViewMatrix(m.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                  int(sizeofMatrix))
    check_last()


def initCuda(h_histogram, volumeSize, histogramSize, h_codebook=None, codebookSize=None,
             h_templates=None, templatesSize=None, h_errorsbook=None, errorsbookSize=None,
             *flexible_arrays) -> None:
    """initCuda, K:1893-2358.  h_histogram: host fp32 array of B-bin records in
    AoS order (record = x + X*(y + Y*z)).  h_codebook (int32 [..., 4]),
    h_templates (fp32 [T, B]) and h_errorsbook (fp32 [..., slots, 2]) make the
    codec volume of methods 4/5/6 resident (sizes as the reference passes them:
    codebookSize = volumeSize, templatesSize = (B, T, 1), errorsbookSize =
    (slots, rows, layers)).  flexible_arrays: the nine span-table arrays of
    arguments 10-18 (codebookSpanLow, codebookSpanHigh, flexibleCodebook,
    flexibleErrorsbook, simpleLow, simpleHigh, simpleCount, simpleHistogram,
    flexibleTemplates) at the reference's fixed sizes (vr_init_flex)."""
    h = np.ascontiguousarray(np.asarray(h_histogram, dtype=np.float32))
    L = _lib.load()
    z = Extent(0, 0, 0)
    keep = []

    def arr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(np.asarray(a, dtype=dt))
        keep.append(a)
        return a.ctypes.data

    L.initCuda(h.ctypes.data, _extent(volumeSize), _extent(histogramSize),
               arr(h_codebook, np.int32), _extent(codebookSize) if codebookSize else z,
               arr(h_templates, np.float32), _extent(templatesSize) if templatesSize else z,
               arr(h_errorsbook, np.float32), _extent(errorsbookSize) if errorsbookSize else z,
               *_flex_initcuda_args(flexible_arrays, arr))
    check_last()


def _flex_initcuda_args(flexible_arrays, arr):
    if not flexible_arrays:
        return [None] * 9
    if len(flexible_arrays) != 9:
        raise ValueError("initCuda takes all nine flexible-block arrays or none")
    types = [np.int32] * 3 + [np.float32] + [np.int32] * 3 + [np.float32] * 2
    return [arr(a, t) for a, t in zip(flexible_arrays, types)]


def init_flex(tables: dict) -> None:
    """Make flexible-block span tables resident (methods 8/9/0; vr_init_flex).
    tables: dim, nbins, fractal_low/high/code int32 (n, 4), fractal_err float32
    (n, nbins, 2), simple_low/high int32 (m, 4), simple_count int32 (m,),
    simple_hist float32 (m, nbins, 2), templates float32 (T, nbins)."""
    keep = {}
    for k, dt in (("fractal_low", np.int32), ("fractal_high", np.int32),
                  ("fractal_code", np.int32), ("fractal_err", np.float32),
                  ("simple_low", np.int32), ("simple_high", np.int32),
                  ("simple_count", np.int32), ("simple_hist", np.float32),
                  ("templates", np.float32)):
        keep[k] = np.ascontiguousarray(tables[k], dtype=dt)
    t = _lib.FlexTables()
    t.dim, t.nbins = int(tables["dim"]), int(tables["nbins"])
    t.n_fractal, t.n_simple = keep["fractal_low"].shape[0], keep["simple_low"].shape[0]
    t.ntemplates = keep["templates"].shape[0]
    t.fractal_low, t.fractal_high = keep["fractal_low"].ctypes.data, keep["fractal_high"].ctypes.data
    t.fractal_code, t.fractal_errors = keep["fractal_code"].ctypes.data, keep["fractal_err"].ctypes.data
    t.simple_low, t.simple_high = keep["simple_low"].ctypes.data, keep["simple_high"].ctypes.data
    t.simple_count, t.simple_hist = keep["simple_count"].ctypes.data, keep["simple_hist"].ctypes.data
    t.templates = keep["templates"].ctypes.data
    check(_lib.load().vr_init_flex(ctypes.byref(t)))


def load_flex_files(span_list, fractal, simple_counts, simple_bin_ids, simple_bin_freqs,
                    templates, dim: int = 64, nbins: int = 64) -> None:
    """The reference's flexible-block files (spanList.bin, codebook0.bin, nzbCounts0.bin,
    nzbBinIds0.bin, nzbFreqs0.bin, domainList.bin; C:79-84) -> resident span tables."""
    args = [str(a).encode() for a in (span_list, fractal, simple_counts, simple_bin_ids,
                                      simple_bin_freqs, templates)]
    check(_lib.load().vr_load_flex_files(*args, int(dim), int(nbins)))


def parse_flex_files(span_list, fractal, simple_counts, simple_bin_ids, simple_bin_freqs,
                     templates, dim: int = 64, nbins: int = 64) -> dict:
    """Parse the flexible-block files on the host into the table dict init_flex takes."""
    L = _lib.load()
    sp = str(span_list).encode()
    n = L.vr_parse_span_list(sp, 0, None, None)
    if n < 0:
        raise VRError(VR_ERR_ARG, f"span list: {n}")
    sl, sh = np.zeros((n, 4), np.int32), np.zeros((n, 4), np.int32)
    L.vr_parse_span_list(sp, n, sl.ctypes.data, sh.ctypes.data)
    fp = str(fractal).encode()
    nf = L.vr_parse_fractal_histogram(fp, sl.ctypes.data, sh.ctypes.data, n, nbins, 0,
                                      None, None, None, None)
    if nf < 0:
        raise VRError(VR_ERR_ARG, f"fractal spans: {nf}")
    t = {"dim": dim, "nbins": nbins,
         "fractal_low": np.zeros((nf, 4), np.int32), "fractal_high": np.zeros((nf, 4), np.int32),
         "fractal_code": np.zeros((nf, 4), np.int32),
         "fractal_err": np.zeros((nf, nbins, 2), np.float32)}
    L.vr_parse_fractal_histogram(fp, sl.ctypes.data, sh.ctypes.data, n, nbins, nf,
                                 t["fractal_low"].ctypes.data, t["fractal_high"].ctypes.data,
                                 t["fractal_code"].ctypes.data, t["fractal_err"].ctypes.data)
    paths = [str(p).encode() for p in (simple_counts, simple_bin_ids, simple_bin_freqs)]
    ns = L.vr_parse_simple_histogram(*paths, nbins, 0, None, None, None, None)
    if ns < 0:
        raise VRError(VR_ERR_ARG, f"simple spans: {ns}")
    t.update({"simple_low": np.zeros((ns, 4), np.int32), "simple_high": np.zeros((ns, 4), np.int32),
              "simple_count": np.zeros(ns, np.int32),
              "simple_hist": np.zeros((ns, nbins, 2), np.float32)})
    L.vr_parse_simple_histogram(*paths, nbins, ns, t["simple_low"].ctypes.data,
                                t["simple_high"].ctypes.data, t["simple_count"].ctypes.data,
                                t["simple_hist"].ctypes.data)
    tp = str(templates).encode()
    nt = L.vr_parse_templates(tp, nbins, 0, None)
    if nt <= 0:
        raise VRError(VR_ERR_ARG, f"flexible templates: {nt}")
    t["templates"] = np.zeros((nt, nbins), np.float32)
    L.vr_parse_templates(tp, nbins, nt, t["templates"].ctypes.data)
    return t


def flex_process(block: int) -> int:
    """dataProcessing with `block`-voxel blocks (vr_flex_process); returns blocks per axis."""
    return int(check(_lib.load().vr_flex_process(int(block))))


def flex_info():
    """(blocks per axis, bins, device pointer of the float4 block statistics)"""
    n, nb, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
    check(_lib.load().vr_flex_info(ctypes.byref(n), ctypes.byref(nb), ctypes.byref(p)))
    return n.value, nb.value, p.value


def init_codec(codebook, templates, errors) -> None:
    """Make a fractal/template codec volume resident (methods 4/5/6).
    codebook int32 (nz, ny, nx, 4) = (template id, shift, flip, NE); templates fp32
    (T, B); errors fp32 (nz, ny, nx, slots, 2) = (bin id, value).  Host numpy arrays
    or CUDA tensors (copied)."""
    L = _lib.load()
    if hasattr(codebook, "data_ptr") and getattr(codebook, "is_cuda", False):
        nz, ny, nx, _ = codebook.shape
        check(L.vr_init_codec(_ptr(codebook), _extent((nx, ny, nz)), _ptr(templates),
                              int(templates.shape[0]), _ptr(errors), int(errors.shape[-2]),
                              int(templates.shape[1]), 1))
        return
    cb = np.ascontiguousarray(codebook, dtype=np.int32)
    tp = np.ascontiguousarray(templates, dtype=np.float32)
    er = np.ascontiguousarray(errors, dtype=np.float32)
    nz, ny, nx, _ = cb.shape
    check(L.vr_init_codec(cb.ctypes.data, _extent((nx, ny, nz)), tp.ctypes.data, tp.shape[0],
                          er.ctypes.data, er.shape[-2], tp.shape[1], 0))


def freeCudaBuffers() -> None:
    """freeCudaBuffers, K:2360-2385."""
    _lib.load().freeCudaBuffers()
    check_last()


def setTextureFilterMode(bLinearFilter: bool) -> None:
    """setTextureFilterMode, K:1889-1891 (no effect on methods 1/2/3/7)."""
    _lib.load().setTextureFilterMode(bool(bLinearFilter))


def basicDataProcessing() -> None:
    """basicDataProcessing, K:1798-1887: bakes the per-voxel statistics of the resident
    raw / codec volumes (originalQueryTex / fractalQueryTex, K:722-871) into float
    planes; methods 1-7 then read the planes (bit-identical to the per-step decode)."""
    _lib.load().basicDataProcessing()
    check_last()


def bake_stats() -> None:
    """vr_bake_stats: basicDataProcessing with a status (raises VRError)."""
    check(_lib.load().vr_bake_stats())


def release_stats() -> None:
    """Drop the baked planes: methods 1-7 decode the records per step again."""
    check(_lib.load().vr_release_stats())


def stats_info():
    """((d_raw, raw_plane_floats), (d_codec, codec_plane_floats)); pointer None = not baked"""
    a, c = ctypes.c_void_p(), ctypes.c_void_p()
    na, nc = ctypes.c_uint64(), ctypes.c_uint64()
    check(_lib.load().vr_stats_info(ctypes.byref(a), ctypes.byref(na), ctypes.byref(c),
                                    ctypes.byref(nc)))
    return (a.value, na.value), (c.value, nc.value)


def set_layout_budget(nbytes=None) -> None:
    """Cap the HBM the library spends on layout copies (micro-brick and
    axis-rows copies of the records, baked-plane copies; include/vr.h): None =
    the default budget, 0 = never make one."""
    check(_lib.load().vr_set_layout_budget(0xFFFFFFFFFFFFFFFF if nbytes is None else int(nbytes)))


def layout_info() -> dict:
    """Layout copies: bytes resident, copies made since load, and the time (ms)
    and size of the last one made -- the extra cost of the first frame of a view
    that needs a copy."""
    b, n = ctypes.c_uint64(), ctypes.c_int()
    ms, lb = ctypes.c_float(), ctypes.c_uint64()
    check(_lib.load().vr_layout_info(ctypes.byref(b), ctypes.byref(n), ctypes.byref(ms),
                                     ctypes.byref(lb)))
    return {"resident_bytes": b.value, "builds": n.value, "last_build_ms": round(ms.value, 3),
            "last_build_bytes": lb.value}


def dataProcessing() -> None:
    """dataProcessing, K:1735-1796: flexible-block pre-pass with 6-voxel blocks."""
    _lib.load().dataProcessing()
    check_last()


# ---------------------------------------------------------------- extensions

def init_distribution(bins, nbins: Optional[int] = None, dims=None, adopt: bool = False):
    """Make a distribution volume resident.

    bins: numpy array (nz, ny, nx, B) -> copied from host; or a torch CUDA tensor
    of the same shape -> copied device-to-device (adopt=False) or used in place
    (adopt=True, the caller keeps it alive)."""
    L = _lib.load()
    if hasattr(bins, "data_ptr") and getattr(bins, "is_cuda", False):
        shp = tuple(bins.shape)
        if dims is None:
            nz, ny, nx, nb = shp
            dims = (nx, ny, nz)
        nb = nbins if nbins is not None else shp[-1]
        check(L.vr_init_distribution(_ptr(bins), _extent(dims), int(nb), 2 if adopt else 1))
        return
    a = np.ascontiguousarray(np.asarray(bins, dtype=np.float32))
    if dims is None:
        nz, ny, nx, nb = a.shape
        dims = (nx, ny, nz)
    nb = nbins if nbins is not None else a.shape[-1]
    check(L.vr_init_distribution(a.ctypes.data, _extent(dims), int(nb), 0))


def synthesize_codec(dims, nbins: int, ntemplates: int = 64, slots: int = 4,
                     seed: int = 20261015) -> None:
    """Generate the seeded synthetic codec volume (methods 4/5/6) directly in HBM."""
    check(_lib.load().vr_synthesize_codec(_extent(dims), int(nbins), int(ntemplates), int(slots),
                                          int(seed)))


def codec_info():
    """((X, Y, Z), nbins, ntemplates, slots, codebook_ptr, templates_ptr, errors_ptr)"""
    e = Extent()
    nb, nt, sl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    cb, tp, er = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    check(_lib.load().vr_codec_info(ctypes.byref(e), ctypes.byref(nb), ctypes.byref(nt),
                                    ctypes.byref(sl), ctypes.byref(cb), ctypes.byref(tp),
                                    ctypes.byref(er)))
    return ((e.width, e.height, e.depth), nb.value, nt.value, sl.value, cb.value, tp.value,
            er.value)


def synthesize(dims, nbins: int, seed: int = 20261015) -> None:
    """Generate the seeded synthetic distribution volume directly in HBM."""
    check(_lib.load().vr_synthesize(_extent(dims), int(nbins), int(seed)))


def volume_info():
    e = Extent()
    nb = ctypes.c_int()
    p = ctypes.c_void_p()
    check(_lib.load().vr_volume_info(ctypes.byref(e), ctypes.byref(nb), ctypes.byref(p)))
    return (e.width, e.height, e.depth), nb.value, p.value


def volume_layout():
    """(row_pitch, slice_pitch) of the resident volume, in records."""
    a, b = ctypes.c_size_t(), ctypes.c_size_t()
    check(_lib.load().vr_volume_layout(ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def set_stream(stream) -> None:
    """Stream for subsequent launches: a torch.cuda.Stream, a raw hipStream_t, or None."""
    raw = 0 if stream is None else (stream.cuda_stream if hasattr(stream, "cuda_stream")
                                    else int(stream))
    check(_lib.load().vr_set_stream(raw))


def set_tuning(key: str, value=None) -> None:
    """Set (value not None) or remove a tuning knob (include/vr.h vr_set_tuning):
    kernel-path overrides and occupancy caps for tests and tools.  Knobs change
    which kernel computes a frame, never its pixels; the library reads no
    environment variables."""
    L = _lib.load()
    check(L.vr_set_tuning(str(key).encode(), None if value is None else str(value).encode()))


def clear_tuning() -> None:
    """Remove every tuning knob (back to the default dispatch)."""
    _lib.load().vr_clear_tuning()


def make_desc(d_output, width: int, height: int, inv_view, density=0.05, brightness=1.0,
              transfer_offset=0.0, transfer_scale=1.0, query_method=1, volume_size=None,
              d_output_f=None, d_steps=None, d_tile_list=None, n_tiles=0) -> RenderDesc:
    d = RenderDesc()
    d.d_output = _ptr(d_output)
    d.d_output_f = _ptr(d_output_f)
    d.d_steps = _ptr(d_steps)
    d.width, d.height = int(width), int(height)
    m = np.asarray(inv_view, dtype=np.float32).reshape(12)
    for i in range(12):
        d.inv_view[i] = float(m[i])
    d.density, d.brightness = float(density), float(brightness)
    d.transfer_offset, d.transfer_scale = float(transfer_offset), float(transfer_scale)
    d.query_method = int(query_method)
    if volume_size is None:  # method 7's grid defaults to the resident volume's dims
        try:
            volume_size = volume_info()[0]
        except VRError:
            _lib.load().vr_clear_error()
            volume_size = codec_info()[0]
    d.volume_size = _extent(volume_size)
    d.d_tile_list = _ptr(d_tile_list)
    d.n_tiles = int(n_tiles)
    return d


def render(desc: RenderDesc) -> None:
    """Launch the march for an explicit descriptor (asynchronous)."""
    check(_lib.load().vr_render(ctypes.byref(desc)))


def count_footprint(desc: RenderDesc) -> int:
    """U: distinct records under all trilinear footprints (synchronous)."""
    return int(check(_lib.load().vr_count_footprint(ctypes.byref(desc))))


def footprint_bytes(desc: RenderDesc) -> int:
    """algorithmic volume bytes of one launch (methods 1-6; synchronous)"""
    return int(check(_lib.load().vr_footprint_bytes(ctypes.byref(desc))))


def unscatter_tiles(d_packed, d_tile_lists, n_ranks: int, n_slots: int, d_frame, width: int,
                    height: int) -> None:
    check(_lib.load().vr_unscatter_tiles(_ptr(d_packed), _ptr(d_tile_lists), int(n_ranks),
                                         int(n_slots), _ptr(d_frame), int(width), int(height)))


def last_kernel() -> str:
    """The march kernel (and its template arguments) the last render launched."""
    return _lib.load().vr_last_kernel().decode()


def stream_read(reps: int = 5):
    """Measured read ceiling: the resident record volume streamed by a coalesced
    16-B-per-lane read kernel (vr_stream_read).  Returns (bytes per pass,
    fastest ms, mean ms)."""
    ms = (ctypes.c_float * 2)()
    nbytes = ctypes.c_uint64(0)
    check(_lib.load().vr_stream_read(int(reps), ms, ctypes.byref(nbytes)))
    return int(nbytes.value), float(ms[0]), float(ms[1])


def debug_wave_clock(d_buf) -> None:
    """Tooling: per-wave {start, end, __smid} clocks of the pipelined, quad and
    ray-segmented marches into a device uint64 buffer of 48 * n_slots values
    (include/vr.h: up to 16 waves of 3 words per launch slot; None = off)."""
    check(_lib.load().vr_debug_wave_clock(None if d_buf is None else _ptr(d_buf)))


# ------------------------------------------- GMM volumes (config 5)

def init_gmm(wm, sigma, dims=None, z_base: int = 0, adopt: bool = False) -> None:
    """Make a K-component GMM volume resident.

    wm: (nzs, ny, nx, K, 2) float32 (w, mu) pairs; sigma: (nzs, ny, nx, K).  numpy
    arrays are copied from the host, torch CUDA tensors device-to-device (or used
    in place with adopt=True).  dims: the whole volume's (X, Y, Z) when only the
    slices [z_base, z_base + nzs) are given (default: wm's own shape)."""
    L = _lib.load()
    on_device = hasattr(wm, "data_ptr") and getattr(wm, "is_cuda", False)
    if not on_device:  # lists and other array-likes, as np.asarray takes them
        wm = np.asarray(wm, dtype=np.float32)
        sigma = np.asarray(sigma, dtype=np.float32)
    if len(wm.shape) != 5 or int(wm.shape[4]) != 2:
        raise ValueError(f"wm must have shape (nzs, ny, nx, K, 2), got {tuple(wm.shape)}")
    nzs, ny, nx, K = (int(v) for v in wm.shape[:4])
    if dims is None:
        dims = (nx, ny, nzs)
    if tuple(int(v) for v in sigma.shape) != (nzs, ny, nx, K):
        raise ValueError(f"sigma must have shape wm.shape[:4] = {(nzs, ny, nx, K)}, "
                         f"got {tuple(sigma.shape)}")
    if on_device:
        import torch
        for name, t in (("wm", wm), ("sigma", sigma)):
            if not getattr(t, "is_cuda", False):
                raise ValueError(f"{name} must be a CUDA tensor like wm")
            if t.device != wm.device:
                raise ValueError(f"{name} is on {t.device}, wm on {wm.device}: both must be on "
                                 "the library's device")
            if t.dtype != torch.float32:
                raise ValueError(f"{name} must be float32, got {t.dtype}")
            if not t.is_contiguous():
                raise ValueError(f"{name} must be contiguous (the march reads dense planes)")
        check(L.vr_init_gmm(_ptr(wm), _ptr(sigma), _extent(dims), K, int(z_base), nzs,
                            2 if adopt else 1))
        return
    a = np.ascontiguousarray(np.asarray(wm, dtype=np.float32))
    b = np.ascontiguousarray(np.asarray(sigma, dtype=np.float32))
    check(L.vr_init_gmm(a.ctypes.data, b.ctypes.data, _extent(dims), K, int(z_base), nzs, 0))


def synthesize_gmm(dims, ncomp: int = 16, seed: int = 20261015, z_base: int = 0,
                   nslices: Optional[int] = None) -> None:
    """Generate slices [z_base, z_base + nslices) of the seeded synthetic GMM volume in HBM."""
    if nslices is None:
        nslices = int(tuple(dims)[2]) - int(z_base)
    check(_lib.load().vr_synthesize_gmm(_extent(dims), int(ncomp), int(seed), int(z_base),
                                        int(nslices)))


def gmm_info():
    """((X, Y, Z), K, z_base, nslices, wm_ptr, sigma_ptr) of the resident GMM volume"""
    e = Extent()
    k, zb, ns = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    a, b = ctypes.c_void_p(), ctypes.c_void_p()
    check(_lib.load().vr_gmm_info(ctypes.byref(e), ctypes.byref(k), ctypes.byref(zb),
                                  ctypes.byref(ns), ctypes.byref(a), ctypes.byref(b)))
    return (e.width, e.height, e.depth), k.value, zb.value, ns.value, a.value, b.value


def free_gmm() -> None:
    check(_lib.load().vr_free_gmm())


def gmm_select(slot: int) -> None:
    """Select GMM slot 0 or 1 (include/vr.h vr_gmm_select): the GMM calls act on it"""
    check(_lib.load().vr_gmm_select(int(slot)))


def gmm_slab(z_lo: int, z_hi: int, d_rays_out, d_n_rays_out, d_rays_in=None,
             n_rays_in: int = 0) -> _lib.GmmSlab:
    s = _lib.GmmSlab()
    s.z_lo, s.z_hi = int(z_lo), int(z_hi)
    s.d_rays_in = _ptr(d_rays_in) or None
    s.n_rays_in = int(n_rays_in)
    s.d_rays_out = _ptr(d_rays_out) or None
    s.d_n_rays_out = _ptr(d_n_rays_out) or None
    return s


def render_gmm(desc: RenderDesc, slab: Optional[_lib.GmmSlab] = None) -> None:
    """Launch the GMM march: the whole frame (slab None) or one slab of a chain."""
    L = _lib.load()
    check(L.vr_render_gmm(ctypes.byref(desc), None if slab is None else ctypes.byref(slab)))


def gmm_count_footprint(desc: RenderDesc, slab: Optional[_lib.GmmSlab] = None) -> int:
    """U of a whole-volume GMM render, or of one slab of a chain (synchronous)"""
    L = _lib.load()
    if slab is None:
        return int(check(L.vr_gmm_count_footprint(ctypes.byref(desc))))
    return int(check(L.vr_gmm_count_footprint_slab(ctypes.byref(desc), ctypes.byref(slab))))


def version() -> str:
    return _lib.load().vr_version().decode()


__all__ = [
    "render_kernel", "copyInvViewMatrix", "initCuda", "freeCudaBuffers", "setTextureFilterMode",
    "basicDataProcessing", "dataProcessing", "init_distribution", "init_codec", "init_flex",
    "flex_process", "flex_info", "load_flex_files", "parse_flex_files", "synthesize", "synthesize_codec", "codec_info",
    "volume_info",
    "volume_layout",
    "set_stream", "set_tuning", "clear_tuning", "make_desc", "render", "count_footprint", "footprint_bytes", "unscatter_tiles", "last_kernel", "debug_wave_clock", "stream_read", "version",
    "init_gmm", "synthesize_gmm", "gmm_info", "free_gmm", "gmm_select", "gmm_slab", "render_gmm",
    "gmm_count_footprint", "bake_stats", "release_stats", "stats_info", "set_layout_budget",
    "layout_info",
    "VRError", "PAD",
]
