"""C-ABI checks that need no GPU: libvr.so loads, exports every entry point that
include/vr.h declares, and reports argument/state errors without exiting
(no compute call is made)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vr.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src)
    return sorted(set(n for n in names if n not in ("if", "sizeof")))


def test_header_declares_reference_entry_points():
    names = declared_functions()
    for ref in ("render_kernel", "copyInvViewMatrix", "initCuda", "freeCudaBuffers",
                "setTextureFilterMode", "basicDataProcessing", "dataProcessing"):
        assert ref in names


def test_library_exports_every_declared_symbol(pkg):
    lib = ctypes.CDLL(pkg.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"libvr.so lacks {missing}"
    assert set(pkg._lib.EXPORTS) == set(declared_functions())


def test_struct_layouts():
    from ctypes import sizeof
    import __graft_entry__ as g
    L = g.load_package()._lib
    assert sizeof(L.Dim3) == 12           # dim3
    assert sizeof(L.Extent) == 24         # cudaExtent / hipExtent
    # vr_render_desc: 3 pointers, 2 u32, 12 f32, 4 f32, int, (pad), extent, ptr, u32 (+pad)
    assert sizeof(L.RenderDesc) == 8 * 3 + 4 * 2 + 4 * 12 + 4 * 4 + 4 + 4 + 24 + 8 + 8


def test_errors_without_gpu(pkg):
    L = pkg._lib.load()
    L.vr_clear_error()
    assert L.vr_render(None) == pkg._lib.VR_ERR_ARG
    assert b"null" in L.vr_last_error()
    L.vr_clear_error()
    # no volume resident: render_kernel records a state error instead of exiting
    pkg._lib.load().freeCudaBuffers()
    with pytest.raises(pkg.VRError) as e:
        pkg.render_kernel((1, 1, 1), (16, 16, 1), 0x1000, 4, 4, 0.05, 1.0, 0.0, 1.0, 1,
                          (4, 4, 4))
    assert e.value.status == pkg._lib.VR_ERR_STATE
    with pytest.raises(pkg.VRError) as e:
        pkg.dataProcessing()  # no span tables resident
    assert e.value.status == pkg._lib.VR_ERR_STATE
    with pytest.raises(pkg.VRError):
        pkg.basicDataProcessing()
    with pytest.raises(pkg.VRError):
        pkg.initCuda(np.zeros(10, np.float32), (2, 2, 2), (4, 3, 1))  # 3 records != 8 voxels
    with pytest.raises(pkg.VRError):
        pkg.copyInvViewMatrix(np.zeros(16, np.float32), 64)            # > 48 bytes
    pkg.setTextureFilterMode(True)  # stored only
    assert pkg._lib.load().vr_tiles_x(1920) == pkg.tiles.tiles_x(1920) == 30
    assert pkg._lib.load().vr_tiles_y(1080) == pkg.tiles.tiles_y(1080) == 270
    assert "gfx950" in pkg.version()


def test_flex_table_validation_without_gpu(pkg, orc):
    """vr_init_flex rejects out-of-range tables before touching the device"""
    t = orc.synth_flex(12, 5, 16, ntemplates=6, extra=0, dup=False)
    bad = [("dim", 0), ("dim", 127), ("nbins", 65)]
    for k, v in bad:
        u = dict(t)
        u[k] = v
        with pytest.raises(pkg.VRError) as e:
            pkg.init_flex(u)
        assert e.value.status == pkg._lib.VR_ERR_ARG
    for col, v in ((0, 6), (0, -1), (1, 16), (3, 17)):  # template id, shift, NE
        u = dict(t)
        u["fractal_code"] = t["fractal_code"].copy()
        u["fractal_code"][3, col] = v
        with pytest.raises(pkg.VRError, match="fractal entry 3"):
            pkg.init_flex(u)
    u = dict(t)
    u["simple_count"] = t["simple_count"].copy()
    u["simple_count"][2] = 17
    with pytest.raises(pkg.VRError, match="simple entry 2"):
        pkg.init_flex(u)


def test_render_kernel_launch_configuration_without_gpu(pkg):
    """render_kernel validates gridSize / blockSize like a CUDA launch would
    (K:2397): an empty grid or block, > 1024 threads per block, a block
    dimension beyond (1024, 1024, 64) or a grid beyond (2^31 - 1, 65535, 65535)
    is an invalid configuration, recorded before any device call"""
    L = pkg._lib.load()
    for grid, block in (((0, 1, 1), (16, 16, 1)), ((4, 0, 1), (16, 16, 1)),
                        ((4, 4, 1), (16, 16, 0)), ((4, 4, 1), (64, 32, 1)),
                        ((4, 4, 1), (1, 1, 65)), ((4, 4, 1), (1, 1025, 1)),
                        ((4, 65536, 1), (16, 16, 1)), ((4, 4, 65536), (16, 16, 1)),
                        ((2 ** 31, 1, 1), (16, 16, 1))):
        with pytest.raises(pkg.VRError) as e:
            pkg.render_kernel(grid, block, 0x1000, 64, 64, 0.05, 1.0, 0.0, 1.0, 1, (4, 4, 4))
        assert e.value.status == pkg._lib.VR_ERR_ARG
        assert "launch configuration" in str(e.value)
    L.vr_clear_error()


def test_tuning_knobs_are_explicit(pkg):
    """knobs go through vr_set_tuning only (no environment reads in the default
    build); an empty key is rejected, None removes a knob"""
    pkg.set_tuning("VR_PATH", "2")
    pkg.set_tuning("VR_PATH", None)
    pkg.clear_tuning()
    with pytest.raises(pkg.VRError) as e:
        pkg.set_tuning("", "1")
    assert e.value.status == pkg._lib.VR_ERR_ARG
    src = open(os.path.join(ROOT, "volume-rendering-based-on-distribution-data_amd", "csrc",
                            "vr_api.cpp")).read()
    # the only getenv sits behind the tooling build flag
    assert src.count("getenv(") == 1
    i = src.index("getenv(")
    assert src.rfind("#ifdef VR_TUNING", 0, i) > src.rfind("#endif", 0, i)
    for f in ("vr_kernels.hip", "vr_seg.hip", "vr_gmm.hip", "vr_stats.hip", "vr_flex.hip"):
        assert "getenv(" not in open(os.path.join(ROOT, "volume-rendering-based-on-"
                                                  "distribution-data_amd", "csrc", f)).read()


def test_init_gmm_validates_array_likes_without_gpu(pkg):
    """init_gmm takes lists like numpy arrays (converted before the shape checks) and
    rejects mismatched shapes with ValueError before any device call"""
    wm = np.zeros((2, 3, 4, 8, 2), np.float32).tolist()
    with pytest.raises(ValueError, match="sigma must have shape"):
        pkg.init_gmm(wm, np.zeros((2, 3, 4, 7), np.float32).tolist())
    with pytest.raises(ValueError, match="wm must have shape"):
        pkg.init_gmm(np.zeros((2, 3, 4, 8), np.float32).tolist(), [[0.0]])
