"""GPU parity of the baked-statistics path (basicDataProcessing, vr_stats.hip).

basicDataProcessing bakes each voxel's mean / variance / entropy once into float
planes (the reference's originalQueryTex / fractalQueryTex, K:722-871); frames
of methods 1-6 then filter the planes.  Bar: the planes equal the oracle's
per-record statistics bit for bit, and every baked frame equals the oracle's
render (packed RGBA8 identical, float RGBA within 1e-4, samples identical).
"""
import ctypes

import numpy as np
import pytest

from test_gpu_parity import assert_parity, codec_render, gpu_render

pytestmark = pytest.mark.gpu


@pytest.fixture
def baked(pkg):
    yield
    pkg.release_stats()


def _d2h(ptr, n):
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.zeros(n, np.float32)
    torch.cuda.synchronize()
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr),
                         ctypes.c_size_t(out.nbytes), 2) == 0
    return out


def plane_geometry(nx, ny):
    """pitches of a baked plane (vr_device.h plane_pitches): 16 x 2 x 1 bricks, x runs
    of 16 starting every 15 voxels (one apron voxel)"""
    sy = ((nx - 1) // 15 + 1) * 32
    return sy, ((ny + 1) // 2) * sy


def plane_index(x, y, z, sy, sz):
    """vr_device.h plane_index: voxel (x, y, z) at its home brick (x // 15)"""
    kx = x // 15
    return z * sz + (y >> 1) * sy + (y & 1) * 16 + kx * 32 + (x - 15 * kx)


@pytest.mark.parametrize("nx,ny,nz", [(9, 7, 5), (31, 6, 3), (46, 3, 2)])
@pytest.mark.parametrize("nb", [1, 3, 4, 8, 32])
def test_planes_equal_oracle_stats(pkg, orc, gpu, baked, nb, nx, ny, nz, tune):
    """plane k < 3 at plane_index(x, y, z) = statistic k+1 of record (x, y, z)
    (orc_record_stats), plane 3 = method 7's corner mean (orc_corner_mean), bit for bit;
    x = 15 k also in the apron (offset 15) of brick k - 1; records with padded rows /
    slices"""
    tune.set("VR_PAD", "3,5")
    vol = orc.synth_volume(nx, ny, nz, nb)
    pkg.init_distribution(vol)
    assert pkg.stats_info()[0][0] is None
    pkg.basicDataProcessing()
    (ptr, plane), _ = pkg.stats_info()
    sy, sz = plane_geometry(nx, ny)
    assert ptr and plane == sz * nz
    got = _d2h(ptr, 4 * plane).reshape(4, plane)
    for z in range(nz):
        for y in range(ny):
            for x in range(nx):
                want = np.append(orc.record_stats(vol[z, y, x]),
                                 np.float32(orc.corner_mean(vol[z, y, x]))).astype(np.float32)
                i = plane_index(x, y, z, sy, sz)
                assert np.array_equal(got[:, i].view(np.uint32), want.view(np.uint32)), (x, y, z)
                if x > 0 and x % 15 == 0:
                    assert np.array_equal(got[:, i - 32 + 15].view(np.uint32),
                                          want.view(np.uint32)), ("apron", x, y, z)


@pytest.mark.parametrize("nb", [1, 4, 5, 8, 32])
def test_baked_render_parity(pkg, orc, gpu, baked, nb):
    """methods 1/2/3 on both cameras from the baked planes: the oracle's frame"""
    import torch
    vol = orc.synth_volume(24, 20, 16, nb)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    for cam in ("C0", "C1"):
        m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, 96, 72, m, method, torch)
            ref = orc.render(vol, orc.make_params(96, 72, m, query_method=method))[:3]
            assert_parity(got, ref, f"baked 24x20x16x{nb} {cam} m{method}")
            # oblique views read the plane's 8 x 2 x 2 brick copy (round 5)
            want = "k_march_pipe<B=1,M=0>" if cam == "C0" else "k_march_seg4_plane8<B=1,M=0>"
            assert pkg.last_kernel() == want, pkg.last_kernel()


@pytest.mark.parametrize("path,env", [
    ("1", {}), ("1", {"VR_BOX_MAX": "64"}), ("7", {"VR_SEG": "-2"}), ("7", {"VR_SEG": "4"}),
    ("7", {"VR_SEG": "-4"}), ("2", {"VR_WG_PER_CU": "2"}), ("7", {"VR_SEG": "2"}),
    ("7", {"VR_SEG": "4", "VR_SEG_MAP": "1"}), ("7", {"VR_SEG": "-2", "VR_SEG_MAP": "1"}),
    ("2", {"VR_SEG_MAP": "1"}),
])
def test_baked_paths(pkg, orc, gpu, baked, path, env, tune):
    """every kernel a baked frame can take (VR_PATH 2 / 7; 1, the LDS-box march over x
    rows, is ignored for the bricked planes) is bit-identical"""
    import torch
    tune.set("VR_PATH", path)
    for k, v in env.items():
        tune.set(k, v)
    vol = orc.synth_volume(20, 18, 16, 8)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))):
        for method in (1, 3):
            got = gpu_render(pkg, None, 80, 64, cam, method, torch)
            ref = orc.render(vol, orc.make_params(80, 64, cam, query_method=method))[:3]
            assert_parity(got, ref, f"baked path {path} {env} m{method}")
            assert "M=0" in pkg.last_kernel() or "M=-1" in pkg.last_kernel(), pkg.last_kernel()


@pytest.mark.parametrize("dims", [(23, 19, 17), (29, 14, 21), (8, 9, 10), (15, 2, 3)])
def test_baked_plane8_copy(pkg, orc, gpu, baked, dims, tune):
    """oblique baked frames filter the method's plane in 8 x 2 x 2 bricks (k_plane8,
    gather8 MODE 6): ragged x (7-voxel brick runs with one apron voxel), odd y and
    z (a half brick pair at the far edge), methods 1/2/3, several oblique views,
    full frames through the segmented and the one-lane marches and rank lists,
    bit-identical to the oracle; VR_PLANE8=0 keeps the 16 x 2 x 1 plane; the copy
    counts in layout_info and goes with the planes"""
    import torch
    vol = orc.synth_volume(*dims, 4)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    W, H = 88, 64
    for rot in ((30.0, 45.0), (-25.0, 130.0), (60.0, -20.0), (180.0, 33.0)):
        m = pkg.camera.display_inv_view(rot)
        for path in ("", "2"):
            if path:
                tune.set("VR_PATH", path)
            else:
                tune.clear("VR_PATH")
            for method in (1, 2, 3):
                got = gpu_render(pkg, None, W, H, m, method, torch)
                assert "plane8" in pkg.last_kernel(), (rot, path, pkg.last_kernel())
                ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
                assert_parity(got, ref, f"plane8 {dims} {rot} path {path} m{method}")
        tune.clear("VR_PATH")
        lists = pkg.tiles.tile_lists(W, H, 3, m)
        n_slots = lists.shape[1]
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        for r in range(3):
            pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=2, d_tile_list=dl[r],
                                     n_tiles=n_slots))
            assert "plane8" in pkg.last_kernel(), pkg.last_kernel()
        frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
        torch.cuda.synchronize()
        ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=2), want_float=False,
                          want_steps=False)[0]
        assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref8), rot
    assert pkg.layout_info()["resident_bytes"] > 0
    tune.set("VR_PLANE8", "0")
    m = pkg.camera.display_inv_view((30.0, 45.0))
    got = gpu_render(pkg, None, W, H, m, 1, torch)
    assert "plane8" not in pkg.last_kernel()
    assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3], "plane8 off")
    pkg.release_stats()
    assert pkg.layout_info()["resident_bytes"] == 0


def test_baked_plane_copies_kept_per_method(pkg, orc, gpu, baked):
    """a client alternating methods 1/2/3 on oblique baked frames builds
    each method's 8 x 2 x 2 plane copy once (one copy per (axis, method) while the
    layout budget holds them), every frame still bit-identical; a budget that
    holds one copy only keeps replacing it, and the frames stay exact"""
    import torch
    vol = orc.synth_volume(30, 26, 22, 8)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    W, H = 96, 64
    m = pkg.camera.display_inv_view((30.0, 45.0))
    refs = {q: orc.render(vol, orc.make_params(W, H, m, query_method=q))[:3] for q in (1, 2, 3)}
    b0 = pkg.layout_info()["builds"]
    for _ in range(3):
        for q in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, q, torch)
            assert "plane8" in pkg.last_kernel(), pkg.last_kernel()
            assert_parity(got, refs[q], f"alternating m{q}")
    info = pkg.layout_info()
    assert info["builds"] - b0 == 3, info  # one copy per method, made once
    one = info["resident_bytes"] // 3
    pkg.set_layout_budget(one + one // 2)  # room for one copy: drops all three
    assert pkg.layout_info()["resident_bytes"] == 0
    for q in (1, 2, 1):
        got = gpu_render(pkg, None, W, H, m, q, torch)
        assert_parity(got, refs[q], f"one-copy budget m{q}")
        assert pkg.layout_info()["resident_bytes"] <= one + one // 2
    pkg.set_layout_budget(None)
    pkg.release_stats()


def test_baked_tile_lists(pkg, orc, gpu, baked):
    """multi-GPU tile lists over the baked planes (segmented march for short lists):
    packed tiles unscatter to the oracle's frame"""
    import torch
    vol = orc.synth_volume(20, 18, 16, 8)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    W, H, world = 130, 70, 3
    m = pkg.camera.single_test_inv_view()
    lists = pkg.tiles.tile_lists(W, H, world)
    n_slots = lists.shape[1]
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=2, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert "M=0" in pkg.last_kernel()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    ref = orc.render(vol, orc.make_params(W, H, m, query_method=2), want_float=False,
                     want_steps=False)[0]
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref)


@pytest.mark.parametrize("nb", [4, 8, 32])
def test_baked_codec(pkg, orc, gpu, baked, nb):
    """methods 4/5/6: codec voxels decoded once into planes (fractalQueryTex, K:775-871)"""
    import torch
    cb, t, e = orc.synth_codec(22, 18, 14, nb, seed=nb)
    pkg.init_codec(cb, t, e)
    pkg.basicDataProcessing()
    _, (ptr, plane) = pkg.stats_info()
    sy, sz = plane_geometry(22, 18)
    assert ptr and plane == sz * 14
    got = _d2h(ptr, 3 * plane).reshape(3, plane)
    for v in range(0, 22 * 18 * 14, 7):
        want = orc.codec_stats(cb, t, e, v)
        x, y, z = v % 22, (v // 22) % 18, v // (22 * 18)
        i = plane_index(x, y, z, sy, sz)
        assert np.array_equal(got[:, i].view(np.uint32), want.view(np.uint32)), v
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view()):
        for method in (4, 5, 6):
            got_f = codec_render(pkg, 72, 56, cam, method, torch)
            ref = orc.render_codec(cb, t, e, orc.make_params(72, 56, cam, query_method=method))[:3]
            assert_parity(got_f, ref, f"baked codec nb={nb} m{method}")
            assert "B=1,M=0>" in pkg.last_kernel(), pkg.last_kernel()


def test_release_reupload_and_errors(pkg, orc, gpu, baked):
    """release_stats returns to the per-step decode; a new volume drops stale planes;
    no volume -> VRError"""
    import torch
    vol = orc.synth_volume(16, 16, 16, 8)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    m = pkg.camera.single_test_inv_view()
    gpu_render(pkg, None, 64, 48, m, 1, torch)
    assert pkg.last_kernel() == "k_march_pipe<B=1,M=0>"
    got = gpu_render(pkg, None, 64, 48, m, 7, torch, m7=(16, 16, 16))
    ref = orc.render(vol, orc.make_params(64, 48, m, query_method=7, m7_dims=(16, 16, 16)))[:3]
    assert_parity(got, ref, "m7 from the baked corner means")
    assert pkg.last_kernel() == "k_march_m7<B=1,M=-7>", pkg.last_kernel()
    pkg.release_stats()
    assert pkg.stats_info()[0][0] is None
    gpu_render(pkg, None, 64, 48, m, 1, torch)
    assert "M=1" in pkg.last_kernel()
    pkg.bake_stats()
    vol2 = orc.synth_volume(12, 10, 8, 4, seed=7)
    pkg.init_distribution(vol2)  # re-upload: the old planes must not be used
    assert pkg.stats_info()[0][0] is None
    got = gpu_render(pkg, None, 64, 48, m, 1, torch)
    ref = orc.render(vol2, orc.make_params(64, 48, m, query_method=1))[:3]
    assert_parity(got, ref, "re-uploaded volume")
    pkg.freeCudaBuffers()
    with pytest.raises(pkg.VRError):
        pkg.bake_stats()


@pytest.mark.parametrize("nb", [1, 4, 8, 32])
def test_baked_method7(pkg, orc, gpu, baked, nb):
    """method 7 from the baked corner means (plane 3): the corner cache and double lerps of
    K:395-480 over 4-byte corners (k_march_m7<1, baked>), grid = volume and grid != volume"""
    import torch
    vol = orc.synth_volume(18, 16, 14, nb)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))):
        for grid in ((18, 16, 14), (10, 12, 20)):
            got = gpu_render(pkg, None, 72, 56, cam, 7, torch, m7=grid)
            ref = orc.render(vol, orc.make_params(72, 56, cam, query_method=7, m7_dims=grid))[:3]
            assert_parity(got, ref, f"baked m7 nb={nb} grid {grid}")
            assert "B=1,M=-7>" in pkg.last_kernel(), pkg.last_kernel()
