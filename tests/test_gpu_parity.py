"""GPU parity: the HIP march (through the C-ABI) against the CPU oracle.

Bar (BASELINE.json north_star): packed RGBA8 identical, float RGBA within
1e-4 per channel, samples-per-pixel identical, on the same seeded inputs.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4  # max per-channel |RGBA - oracle| (north_star)


def gpu_render(pkg, vol_or_none, W, H, m, method, torch, density=0.05, brightness=1.0,
               toff=0.0, tscale=1.0, m7=None, tile_list=None):
    if vol_or_none is not None:
        pkg.init_distribution(vol_or_none)
    dims = (1, 1, 1) if m7 or method in (8, 9, 0) else pkg.volume_info()[0]
    out = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    out_f = torch.zeros(H * W * 4, dtype=torch.float32, device="cuda")
    steps = torch.full((H * W,), -2, dtype=torch.int32, device="cuda")
    d = pkg.make_desc(out, W, H, m, density=density, brightness=brightness,
                      transfer_offset=toff, transfer_scale=tscale, query_method=method,
                      volume_size=m7 or dims, d_output_f=out_f, d_steps=steps)
    pkg.render(d)
    torch.cuda.synchronize()
    return (out.cpu().numpy().view(np.uint32).reshape(H, W),
            out_f.cpu().numpy().reshape(H, W, 4), steps.cpu().numpy().reshape(H, W))


def assert_parity(got, ref, what):
    g8, gf, gn = got
    r8, rf, rn = ref
    hit = rn >= 0
    assert np.array_equal(gn[hit], rn[hit]), f"{what}: samples per pixel differ"
    assert np.all(gn[~hit] == -1), f"{what}: miss pixels must report -1"
    assert np.array_equal(g8, r8), (
        f"{what}: {int(np.sum(g8 != r8))} RGBA8 pixels differ from the oracle")
    err = float(np.max(np.abs(gf - rf))) if gf.size else 0.0
    assert err <= TOL, f"{what}: max |RGBA - oracle| = {err}"


@pytest.mark.parametrize("method", [1, 2, 3, 7])
@pytest.mark.parametrize("cam", ["C0", "C1"])
@pytest.mark.parametrize("nb", [1, 4, 8])
def test_small_scene(pkg, orc, gpu, method, cam, nb):
    import torch
    vol = orc.synth_volume(24, 20, 16, nb)
    m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
    W, H = 96, 72
    got = gpu_render(pkg, vol, W, H, m, method, torch)
    p = orc.make_params(W, H, m, query_method=method, m7_dims=(24, 20, 16))
    ref = orc.render(vol, p)[:3]
    assert_parity(got, ref, f"24x20x16x{nb} {cam} m{method}")


@pytest.mark.parametrize("nb", [2, 3, 5, 16, 32])
def test_bin_counts(pkg, orc, gpu, nb):
    """compiled specialisations (2, 16, 32) and the runtime-B path (3, 5)"""
    import torch
    vol = orc.synth_volume(12, 14, 10, nb)
    m = pkg.camera.display_inv_view((20.0, -35.0))
    for method in (1, 2, 3, 7):
        got = gpu_render(pkg, vol, 48, 40, m, method, torch)
        ref = orc.render(vol, orc.make_params(48, 40, m, query_method=method,
                                              m7_dims=(12, 14, 10)))[:3]
        assert_parity(got, ref, f"nb={nb} m{method}")


@pytest.mark.parametrize("wide", ["", "1", "2"])
@pytest.mark.parametrize("nb", [16, 32])
@pytest.mark.parametrize("cam", ["C0", "C1"])
def test_wide_records_take_batched_march(pkg, orc, gpu, nb, cam, wide, tune):
    """16 / 32 bins (the reference's record width), mean and variance: the quad-
    cooperative march (k_march_wq; the lane-per-record k_march_wide for row-aligned
    16-bin views; VR_WIDE=1 / 2 force either), full
    frames and packed tile lists bit-identical to the oracle; VR_PATH=1 keeps the
    LDS-box march; entropy takes the quad march (the LDS-box march for oblique
    views of a coarse volume)"""
    import torch
    tune.set("VR_WIDE", wide)
    kind = wide or ("1" if nb == 16 and cam == "C0" else "2")
    want = "k_march_wide<" if kind == "1" else "k_march_wq<"
    vol = orc.synth_volume(21, 18, 15, nb)
    m = pkg.camera.single_test_inv_view() if cam == "C0" else pkg.camera.display_inv_view()
    W, H = 88, 60
    pkg.init_distribution(vol)
    for method in (1, 2):
        got = gpu_render(pkg, None, W, H, m, method, torch)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
        assert_parity(got, ref, f"{nb} bins {cam} m{method}")
        assert pkg.last_kernel().startswith(want), pkg.last_kernel()
    # a rank's packed tile list (multi-GPU path) through the same kernel
    lists = pkg.tiles.tile_lists(W, H, 3, m)
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    for r in range(3):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert pkg.last_kernel().startswith(want), pkg.last_kernel()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
    torch.cuda.synchronize()
    ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref8)
    got = gpu_render(pkg, None, W, H, m, 3, torch)
    assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=3))[:3],
                  f"{nb} bins {cam} m3")
    # (oblique entropy of this coarse volume: the LDS-box march, round 6)
    want3 = "k_march<" if cam == "C1" else "k_march_wq<"
    assert pkg.last_kernel().startswith(want3), pkg.last_kernel()
    # method 7: quad-cooperative corner refreshes, method-7 grid = volume or not
    for grid in ((21, 18, 15), (10, 12, 20)):
        got = gpu_render(pkg, None, W, H, m, 7, torch, m7=grid)
        assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=7,
                                                           m7_dims=grid))[:3],
                      f"{nb} bins {cam} m7 grid {grid}")
        assert pkg.last_kernel().startswith("k_march_m7wq<"), pkg.last_kernel()
    tune.set("VR_M7_WQ", "0")
    got = gpu_render(pkg, None, W, H, m, 7, torch, m7=(21, 18, 15))
    assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=7,
                                                       m7_dims=(21, 18, 15)))[:3],
                  f"{nb} bins {cam} m7 lane-owned")
    assert pkg.last_kernel().startswith("k_march_m7<"), pkg.last_kernel()
    tune.set("VR_PATH", "1")
    got = gpu_render(pkg, None, W, H, m, 1, torch)
    assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3],
                  f"{nb} bins {cam} m1 box")
    assert pkg.last_kernel().startswith("k_march<"), pkg.last_kernel()


def test_reference_isabel_shape_via_reference_api(pkg, orc, gpu):
    """The reference's own shape: 50x50x10 blocks x 32 bins, initCuda + render_kernel at
    512x512 with the runSingleTest camera (C:1016-1067)."""
    import torch
    vol = orc.synth_volume(50, 50, 10, 32)
    W = H = 512
    pkg.initCuda(vol.reshape(-1), (50, 50, 10), (32, 2500, 10))
    m = pkg.camera.single_test_inv_view()
    pkg.copyInvViewMatrix(m, 48)
    pkg.basicDataProcessing()
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for method in (1, 2, 3, 7):
        out.zero_()  # C:208 / C:1022
        pkg.render_kernel((32, 32, 1), (16, 16, 1), out, W, H, 0.05, 1.0, 0.0, 1.0, method,
                          (50, 50, 10))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32).reshape(H, W)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method,
                                              m7_dims=(50, 50, 10)), want_float=False,
                         want_steps=False)[0]
        assert np.array_equal(got, ref), f"m{method}: {int(np.sum(got != ref))} pixels differ"
    pkg.freeCudaBuffers()


@pytest.mark.parametrize("params", [
    dict(density=0.2, brightness=1.5, toff=0.1, tscale=1.3),
    dict(density=1.0, brightness=0.7, toff=-0.2, tscale=0.5),
    dict(density=0.01, brightness=2.0, toff=0.05, tscale=2.0),
])
def test_render_parameters(pkg, orc, gpu, params):
    """density / brightness / transfer offset+scale (keyboard parameters, C:315-345)"""
    import torch
    vol = orc.synth_volume(20, 20, 20, 4)
    m = pkg.camera.display_inv_view((10.0, 70.0))
    for method in (1, 3):
        got = gpu_render(pkg, vol, 64, 64, m, method, torch, **params)
        ref = orc.render(vol, orc.make_params(
            64, 64, m, density=params["density"], brightness=params["brightness"],
            transfer_offset=params["toff"], transfer_scale=params["tscale"],
            query_method=method))[:3]
        assert_parity(got, ref, f"{params} m{method}")


def test_method7_grid_differs_from_volume(pkg, orc, gpu):
    """render_kernel's volumeSize drives only the method-7 corner grid (K:322-352)."""
    import torch
    vol = orc.synth_volume(16, 16, 16, 4)
    m = pkg.camera.display_inv_view((25.0, 15.0))
    got = gpu_render(pkg, vol, 64, 64, m, 7, torch, m7=(10, 12, 20))
    ref = orc.render(vol, orc.make_params(64, 64, m, query_method=7, m7_dims=(10, 12, 20)))[:3]
    assert_parity(got, ref, "m7 grid 10x12x20 over 16^3")
    # B = 8, oblique, grid != volume: the quad march does not apply
    vol8 = orc.synth_volume(16, 16, 16, 8)
    got = gpu_render(pkg, vol8, 64, 64, m, 7, torch, m7=(10, 12, 20))
    ref = orc.render(vol8, orc.make_params(64, 64, m, query_method=7, m7_dims=(10, 12, 20)))[:3]
    assert_parity(got, ref, "m7 grid 10x12x20 over 16^3 x 8")
    assert pkg.last_kernel().startswith("k_march_m7_pipe")


def test_oblique_coarse_volume_takes_segmented_march(pkg, orc, gpu):
    """>= 4 pixels per voxel of the x-y face on an oblique view: methods 1/2 take the
    pipelined 2-lane segmented march, bit-identical"""
    import torch
    vol = orc.synth_volume(20, 18, 16, 8)
    m = pkg.camera.display_inv_view((30.0, 45.0))
    for method, W, H, kern in ((1, 96, 64, "k_march_segp2"), (2, 96, 64, "k_march_segp2"),
                               (1, 32, 24, "k_march_quad")):
        got = gpu_render(pkg, vol, W, H, m, method, torch)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
        assert_parity(got, ref, f"coarse oblique m{method} {W}x{H}")
        assert pkg.last_kernel().startswith(kern), pkg.last_kernel()


def test_row_aligned_coarse_volume_takes_box_march(pkg, orc, gpu, tune):
    """row-aligned full frame, >= 4 pixels per voxel, more rays than the segmented
    threshold: methods 1/2 stage the wave's footprint box in LDS (path 1),
    bit-identical; 8-bin entropy takes it too (round 4: the rolled LDS-column entropy);
    a frame below the threshold takes the ray-segmented march"""
    import torch
    tune.set("VR_SEG_RAYS", "1000")
    vol = orc.synth_volume(20, 18, 16, 8)
    m = pkg.camera.display_inv_view((0.0, 0.0), translation=(0.05, -0.1, 0.0))
    # (8-bin mean / variance: two samples per box, k_march_duo)
    for method, W, H, kern in ((1, 96, 64, "k_march_duo<"), (2, 96, 64, "k_march_duo<"),
                               (3, 96, 64, "k_march<"), (1, 32, 24, "k_march_segp4")):
        got = gpu_render(pkg, vol, W, H, m, method, torch)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
        assert_parity(got, ref, f"coarse rows m{method} {W}x{H}")
        assert pkg.last_kernel().startswith(kern), pkg.last_kernel()


@pytest.mark.parametrize("nb", [16, 32])
def test_wide_coarse_rows_take_box_march(pkg, orc, gpu, nb, tune):
    """16 / 32 bins, >= 4 pixels per voxel: row-aligned full frames above the
    segmented threshold stage the wave's footprint box (k_march, entropy included;
    box rows loaded by the quad gathers), oblique ones keep the quad-cooperative
    march; bit-identical"""
    import torch
    tune.set("VR_SEG_RAYS", "1000")
    vol = orc.synth_volume(20, 18, 16, nb)
    pkg.init_distribution(vol)
    rows = pkg.camera.display_inv_view((0.0, 0.0), translation=(0.05, -0.1, 0.0))
    for m, kern in ((rows, "k_march<"), (pkg.camera.display_inv_view(), "k_march_wq<")):
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, 96, 64, m, method, torch)
            ref = orc.render(vol, orc.make_params(96, 64, m, query_method=method))[:3]
            assert_parity(got, ref, f"coarse {nb} bins m{method}")
            # (oblique entropy too takes the box, round 6)
            want = "k_march<" if method == 3 else kern
            assert pkg.last_kernel().startswith(want), pkg.last_kernel()


@pytest.mark.parametrize("nb", [16, 32])
def test_wide_axis_views_take_box_march(pkg, orc, gpu, nb):
    """16 / 32 bins, views along the volume's z or y (side / top, no axis copy for
    B > 8): full frames take the LDS-box march on the x rows (round 6), methods
    1/2/3, bit-identical; rank tile lists keep the quad-cooperative march"""
    import torch
    vol = orc.synth_volume(22, 19, 17, nb)
    pkg.init_distribution(vol)
    W, H = 72, 56
    for rot in ((0.0, 90.0), (90.0, 90.0), (-10.0, -80.0)):
        m = pkg.camera.display_inv_view(rot)
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            assert_parity(got, ref, f"wide axis view {rot} {nb} bins m{method}")
            assert pkg.last_kernel().startswith("k_march<"), (rot, pkg.last_kernel())
    lists = pkg.tiles.tile_lists(W, H, 3, m)
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    for r in range(3):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert not pkg.last_kernel().startswith("k_march<"), pkg.last_kernel()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
    torch.cuda.synchronize()
    ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref8)


def test_edge_images(pkg, orc, gpu):
    """ragged image sizes: 1x1, odd sizes, partial tiles"""
    import torch
    vol = orc.synth_volume(16, 16, 16, 4)
    pkg.init_distribution(vol)
    m = pkg.camera.single_test_inv_view()
    for W, H in [(1, 1), (17, 3), (33, 65), (250, 7)]:
        got = gpu_render(pkg, None, W, H, m, 1, torch)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3]
        assert_parity(got, ref, f"{W}x{H}")


def test_camera_inside_volume(pkg, orc, gpu):
    """eye inside the box: tnear < 0 is clamped to 0 (K:305-306)"""
    import torch
    vol = orc.synth_volume(16, 16, 16, 4)
    m = pkg.camera.display_inv_view((0.0, 0.0), translation=(0.1, -0.2, -0.3))
    got = gpu_render(pkg, vol, 64, 64, m, 1, torch)
    ref = orc.render(vol, orc.make_params(64, 64, m, query_method=1))[:3]
    assert_parity(got, ref, "eye inside")


def test_synth_matches_oracle(pkg, orc, gpu):
    """the on-device generator writes the same volume as the oracle generator"""
    import torch
    for dims, nb in [((16, 12, 10), 1), ((16, 12, 10), 4), ((9, 7, 5), 8), ((8, 8, 8), 3),
                     ((8, 6, 4), 32)]:
        pkg.synthesize(dims, nb, seed=20261015)
        (nx, ny, nz), b, ptr = pkg.volume_info()
        sy, sz = pkg.volume_layout()
        n = sz * nz * b
        t = torch.empty(n, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        # device-to-device copy of the library-owned (pitched) volume into a torch tensor
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr),
                             ctypes.c_size_t(n * 4), 3) == 0
        flat = t.cpu().numpy()
        got = np.stack([flat[z * sz * b:(z * sz + ny * sy) * b].reshape(ny, sy, b)[:, :nx]
                        for z in range(nz)])
        ref = orc.synth_volume(nx, ny, nz, b)
        assert np.array_equal(got, ref), f"synth {dims}x{nb} differs"


def test_footprint_count(pkg, orc, gpu):
    import torch
    vol = orc.synth_volume(40, 36, 32, 4)
    pkg.init_distribution(vol)
    for cam, m in [("C0", pkg.camera.single_test_inv_view()),
                   ("C1", pkg.camera.display_inv_view())]:
        for method in (1, 2, 3):
            out = torch.zeros(128 * 96, dtype=torch.int32, device="cuda")
            d = pkg.make_desc(out, 128, 96, m, query_method=method)
            u = pkg.count_footprint(d)
            ref = orc.count_footprint(vol, orc.make_params(128, 96, m, query_method=method))
            assert u == ref, f"{cam} m{method}: U {u} != oracle {ref}"


@pytest.mark.parametrize("world", [2, 3, 8])
def test_tile_split_and_unscatter(pkg, orc, gpu, world):
    """multi-GPU path on one device: each 'rank' renders its tile list into a packed
    buffer, rank 0 unscatters -> identical to the full-frame render"""
    import torch
    vol = orc.synth_volume(32, 32, 32, 8)
    pkg.init_distribution(vol)
    W, H = 200, 136
    m = pkg.camera.display_inv_view()
    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.render(pkg.make_desc(full, W, H, m, query_method=1))
    lists = pkg.tiles.tile_lists(W, H, world)
    n_slots = lists.shape[1]
    # garbage-filled: tile-list renders write every in-image pixel (misses as 0)
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)
    ref = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                     want_steps=False)[0]
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_cost_dealt_tile_split(pkg, orc, gpu, world):
    """measured-cost dealing (bench.py at N > 1): per-pixel steps of the estimate
    split -> summed tile costs -> tile_lists_by_cost; the re-dealt ranks (PAD
    slots inside the XCD sublists included) assemble the same frame"""
    import torch
    vol = orc.synth_volume(32, 32, 32, 8)
    pkg.init_distribution(vol)
    W, H = 200, 136
    m = pkg.camera.display_inv_view()
    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    fsteps = torch.full((W * H,), -1, dtype=torch.int32, device="cuda")
    pkg.render(pkg.make_desc(full, W, H, m, query_method=1, d_steps=fsteps))
    lists = pkg.tiles.tile_lists(W, H, world, m)
    n_slots = lists.shape[1]
    ntiles = pkg.tiles.tiles_x(W) * pkg.tiles.tiles_y(H)
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    cost = np.zeros(ntiles, np.int64)
    for r in range(world):
        buf = torch.zeros(n_slots * 256, dtype=torch.int32, device="cuda")
        st = torch.full((n_slots * 256,), -1, dtype=torch.int32, device="cuda")
        pkg.render(pkg.make_desc(buf, W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots, d_steps=st))
        torch.cuda.synchronize()
        cost += pkg.tiles.tile_costs_from_steps(st.cpu().numpy(), lists[r], ntiles)
    torch.cuda.synchronize()
    # the split's steps are the full frame's steps
    assert np.array_equal(cost, pkg.tiles.tile_costs_from_frame(fsteps.cpu().numpy(), W, H))
    lists2 = pkg.tiles.tile_lists_by_cost(W, H, world, cost)
    n2 = lists2.shape[1]
    packed = torch.full((world, n2 * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl2 = torch.from_numpy(lists2.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl2[r],
                                 n_tiles=n2))
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl2, world, n2, frame, W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)


@pytest.mark.parametrize("adapt", [True, False])
def test_adaptive_frame_order_renders_identical_frames(pkg, orc, gpu, adapt, tune):
    """full frames: the 1st render of a view uses the estimate order and records
    tile costs, the 2nd re-deals the tiles by them; every frame is the oracle's;
    a new view / new volume starts over"""
    import torch
    tune.set("VR_SEG_RAYS", "0")  # keep this small frame on the recording march
    if not adapt:
        tune.set("VR_NO_ADAPT", "1")
    vol = orc.synth_volume(48, 40, 36, 8)
    pkg.init_distribution(vol)
    W, H = 320, 200
    for m in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((10.0, 20.0))):
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                         want_steps=False)[0]
        for _ in range(4):
            out = torch.full((W * H,), 0, dtype=torch.int32, device="cuda")
            pkg.render(pkg.make_desc(out, W, H, m, query_method=1))
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref)
    vol2 = orc.synth_volume(48, 40, 36, 8, seed=7)
    pkg.init_distribution(vol2)
    ref2 = orc.render(vol2, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    for _ in range(3):
        out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        pkg.render(pkg.make_desc(out, W, H, m, query_method=1))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref2)


def test_errors_do_not_exit(pkg, gpu):
    import torch
    pkg.freeCudaBuffers()  # no codec volume resident either
    vol = np.zeros((4, 4, 4, 2), np.float32)
    pkg.init_distribution(vol)
    out = torch.zeros(16, dtype=torch.int32, device="cuda")
    for bad in (4, 5, 6, 8, 9, 0, 11):
        with pytest.raises(pkg.VRError):
            pkg.render_kernel((1, 1, 1), (16, 16, 1), out, 4, 4, 0.05, 1.0, 0.0, 1.0, bad,
                              (4, 4, 4))
    with pytest.raises(pkg.VRError):
        pkg.dataProcessing()
    pkg.freeCudaBuffers()
    with pytest.raises(pkg.VRError):
        pkg.render_kernel((1, 1, 1), (16, 16, 1), out, 4, 4, 0.05, 1.0, 0.0, 1.0, 1, (4, 4, 4))


@pytest.mark.parametrize("path,env", [
    ("0", {}), ("1", {}), ("2", {}), ("4", {}),
    ("1", {"VR_BOX_MAX": "0"}), ("1", {"VR_BOX_MAX": "64"}), ("0", {"VR_WG_PER_CU": "1"}),
    ("7", {"VR_SEG": "2"}), ("7", {"VR_SEG": "4"}), ("7", {"VR_SEG": "-4"}),
    ("7", {"VR_SEG": "-2"}),
    # occupancy caps (LDS requests) on the ray-segmented, LDS-box and pipelined launches
    ("7", {"VR_SEG": "-2", "VR_WG_PER_CU": "3"}), ("1", {"VR_BOX_MAX": "64", "VR_WG_PER_CU": "3"}),
    ("2", {"VR_WG_PER_CU": "2"}), ("0", {"VR_WG_PER_CU": "3"}),
    ("0", {"VR_QUAD2": "1"}), ("0", {"VR_QUAD2": "1", "VR_WG_PER_CU": "1"}),
    # K samples per footprint box (k_march_duo m1/m2; m3 takes k_march), with
    # direct-path fallbacks
    ("1", {"VR_DUO": "2"}), ("1", {"VR_DUO": "2", "VR_BOX_MAX": "64"}),
    ("1", {"VR_DUO": "3"}), ("1", {"VR_DUO": "4", "VR_BOX_MAX": "64"}),
    # a wave's rays as a compact pixel block (segmented and one-lane pipelined marches)
    ("7", {"VR_SEG": "4", "VR_SEG_MAP": "1"}), ("7", {"VR_SEG": "-2", "VR_SEG_MAP": "1"}),
    ("7", {"VR_SEG": "-4", "VR_SEG_MAP": "1"}), ("2", {"VR_SEG_MAP": "1"}),
])
@pytest.mark.parametrize("nb", [4, 8])
def test_every_kernel_path(pkg, orc, gpu, path, env, nb, tune):
    """each march variant (quad / LDS-staged box with fallback / per-ray pipelined) is
    bit-identical to the oracle on both cameras and all three statistics"""
    import torch
    tune.set("VR_PATH", path)
    for k, v in env.items():
        tune.set(k, v)
    vol = orc.synth_volume(26, 22, 18, nb)
    pkg.init_distribution(vol)
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0)),
                pkg.camera.display_inv_view((-60.0, 110.0))):
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, 80, 64, cam, method, torch)
            ref = orc.render(vol, orc.make_params(80, 64, cam, query_method=method))[:3]
            assert_parity(got, ref, f"path {path} {env} nb={nb} m{method}")


@pytest.mark.parametrize("k", ["2", "3", "4"])
@pytest.mark.parametrize("nb", [1, 2, 8])
def test_duo_march_early_exit(pkg, orc, gpu, nb, k, tune):
    """k_march_duo (K samples per footprint box; mean and variance -- entropy keeps
    one sample per box, k_march<B, 3>): rays ending on any sample of a box
    (opacity, tfar), full frames and tile lists, bit-identical to the oracle"""
    import torch
    tune.set("VR_PATH", "1")
    tune.set("VR_DUO", k)
    vol = orc.synth_volume(30, 26, 22, nb)
    pkg.init_distribution(vol)
    cams = [pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0)),
            pkg.camera.display_inv_view((0.0, 90.0))]
    for cam in cams:
        for density, bright in ((0.05, 1.0), (0.6, 1.3), (3.0, 0.7)):
            for method in (1, 2, 3):
                got = gpu_render(pkg, None, 72, 40, cam, method, torch, density=density,
                                 brightness=bright)
                want = ("k_march<" if method == 3 else "k_march_duo<" if k == "2"
                        else f"k_march_duo{k}<")
                assert pkg.last_kernel().startswith(want), pkg.last_kernel()
                ref = orc.render(vol, orc.make_params(72, 40, cam, query_method=method,
                                                      density=density, brightness=bright))[:3]
                assert_parity(got, ref, f"duo nb={nb} m{method} d={density}")
    W, H, m = 72, 40, cams[0]
    lists = pkg.tiles.tile_lists(W, H, 3, m)
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    for r in range(3):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert pkg.last_kernel().startswith("k_march_duo"), pkg.last_kernel()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
    torch.cuda.synchronize()
    got = frame.cpu().numpy().view(np.uint32).reshape(H, W)
    ref8 = orc.render(vol, orc.make_params(72, 40, cams[0], query_method=1), want_float=False,
                      want_steps=False)[0]
    assert np.array_equal(got, ref8)


@pytest.mark.parametrize("seg", ["2", "4", "-2", "-4"])
@pytest.mark.parametrize("nb", [1, 2, 8])
def test_segmented_march_early_exit(pkg, orc, gpu, seg, nb, tune):
    """ray-segmented march (S lanes per ray): early exits inside a window, rays that end
    on any lane of a window and tile lists give the one-lane march's results bit for bit"""
    import torch
    tune.set("VR_PATH", "7")
    tune.set("VR_SEG", seg)
    vol = orc.synth_volume(30, 26, 22, nb)
    pkg.init_distribution(vol)
    cams = [pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))]
    for cam in cams:
        for density, bright in ((0.05, 1.0), (0.6, 1.3), (3.0, 0.7)):
            for method in (1, 2, 3):
                got = gpu_render(pkg, None, 72, 40, cam, method, torch, density=density,
                                 brightness=bright)
                ref = orc.render(vol, orc.make_params(72, 40, cam, query_method=method,
                                                      density=density, brightness=bright))[:3]
                assert_parity(got, ref, f"seg {seg} nb={nb} m{method} d={density}")
    # tile lists (multi-GPU ranks): packed slots, misses cleared
    W, H = 136, 72
    m = cams[1]
    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    tune.set("VR_PATH", "2")
    pkg.render(pkg.make_desc(full, W, H, m, query_method=1))
    tune.set("VR_PATH", "7")
    world = 3
    lists = pkg.tiles.tile_lists(W, H, world, m)
    n_slots = lists.shape[1]
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
    name = f"k_march_segp{seg[1:]}" if seg.startswith("-") else f"k_march_seg{seg}"
    assert pkg.last_kernel().startswith(name)
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)


@pytest.mark.parametrize("brick", ["1", "0"])
def test_quad_two_lanes_per_ray(pkg, orc, gpu, brick, tune):
    """k_march_quad2 (the quad march with two lanes per ray: halves of a wave take
    alternate steps and composite both in order): early exits on even and odd
    steps, frames whose edges cut tiles and workgroups, and tile lists whose slot
    count is not a multiple of 8 give the one-lane march's results bit for bit,
    on the x rows and on the micro-brick copy"""
    import torch
    tune.set("VR_PATH", "0")
    tune.set("VR_QUAD2", "1")
    tune.set("VR_BRICK", brick)
    vol = orc.synth_volume(30, 26, 22, 8)
    pkg.init_distribution(vol)
    cams = [pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0)),
            pkg.camera.display_inv_view((-60.0, 110.0))]
    for cam in cams:
        for density, bright in ((0.05, 1.0), (0.6, 1.3), (3.0, 0.7)):
            for method in (1, 2, 3):
                got = gpu_render(pkg, None, 72, 42, cam, method, torch, density=density,
                                 brightness=bright)
                ref = orc.render(vol, orc.make_params(72, 42, cam, query_method=method,
                                                      density=density, brightness=bright))[:3]
                assert_parity(got, ref, f"quad2 brick={brick} m{method} d={density}")
                assert pkg.last_kernel().startswith("k_march_quad2")
    # tile lists (multi-GPU ranks): packed slots, misses cleared, 3 ranks
    W, H = 136, 72
    m = cams[1]
    full = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    tune.set("VR_QUAD2", "0")
    pkg.render(pkg.make_desc(full, W, H, m, query_method=1))
    tune.set("VR_QUAD2", "1")
    world = 3
    lists = pkg.tiles.tile_lists(W, H, world, m)
    n_slots = lists.shape[1]
    assert n_slots % 8 != 0 or world == 3
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert pkg.last_kernel().startswith("k_march_quad2")
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)


@pytest.mark.parametrize("path", ["", "0"])
def test_padded_layout(pkg, orc, gpu, path, tune):
    """pitched rows / slices (VR_PAD) change only addresses, never results (path 0: the
    quad march on the micro-brick copy made from the pitched records)"""
    import torch
    if path:
        tune.set("VR_PATH", path)
    vol = orc.synth_volume(20, 18, 16, 8)
    ref = orc.render(vol, orc.make_params(64, 48, pkg.camera.display_inv_view(), query_method=1))[:3]
    for pad in ("4,0", "3,77"):
        tune.set("VR_PAD", pad)
        got = gpu_render(pkg, vol, 64, 48, pkg.camera.display_inv_view(), 1, torch)
        assert_parity(got, ref, f"pad {pad}")
        pkg.synthesize((20, 18, 16), 8)
        got = gpu_render(pkg, None, 64, 48, pkg.camera.display_inv_view(), 1, torch)
        assert_parity(got, ref, f"synth pad {pad}")
        if path == "0":
            assert pkg.last_kernel().startswith("k_march_quad_brick<")


def test_fast_log_is_exact_for_every_float(pkg, gpu):
    """the entropy decode's logf_canon == (float)log((double)x) for all 2^31 - 2^23
    positive finite floats, series and table forms (exhaustive, on the device)"""
    import ctypes
    L = pkg._lib.load()
    counts = (ctypes.c_uint64 * 2)()
    assert L.vr_selftest_logf(counts) == 0, L.vr_last_error()
    assert counts[0] == 0, f"{counts[0]} floats differ"
    assert counts[1] < 1 << 17, f"{counts[1]} fallbacks (both forms)"


# ---- methods 4/5/6: fractal/template codec ----

def codec_render(pkg, W, H, m, method, torch):
    out = torch.zeros(H * W, dtype=torch.int32, device="cuda")
    out_f = torch.zeros(H * W * 4, dtype=torch.float32, device="cuda")
    steps = torch.full((H * W,), -2, dtype=torch.int32, device="cuda")
    d = pkg.make_desc(out, W, H, m, query_method=method, volume_size=(1, 1, 1), d_output_f=out_f,
                      d_steps=steps)
    pkg.render(d)
    torch.cuda.synchronize()
    return (out.cpu().numpy().view(np.uint32).reshape(H, W),
            out_f.cpu().numpy().reshape(H, W, 4), steps.cpu().numpy().reshape(H, W))


@pytest.mark.parametrize("method", [4, 5, 6])
@pytest.mark.parametrize("nb", [4, 8, 32])
def test_codec_methods(pkg, orc, gpu, method, nb):
    import torch
    cb, t, e = orc.synth_codec(22, 18, 14, nb, seed=nb + method)
    pkg.init_codec(cb, t, e)
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view()):
        got = codec_render(pkg, 72, 56, cam, method, torch)
        ref = orc.render_codec(cb, t, e, orc.make_params(72, 56, cam, query_method=method))[:3]
        assert_parity(got, ref, f"codec nb={nb} m{method}")
    assert pkg.last_kernel().startswith("k_march_codec")


@pytest.mark.parametrize("nb", [4, 8, 32])
def test_codec_block_map(pkg, orc, gpu, nb, tune):
    """VR_CODEC_MAP=1: the one-lane codec march with a 16x4 pixel block per wave,
    row-aligned and oblique views, methods 4/5/6, bit-identical"""
    import torch
    tune.set("VR_CODEC_MAP", "1")
    cb, t, e = orc.synth_codec(22, 18, 14, nb, seed=nb + 11)
    pkg.init_codec(cb, t, e)
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view()):
        for method in (4, 5, 6):
            got = codec_render(pkg, 72, 56, cam, method, torch)
            ref = orc.render_codec(cb, t, e, orc.make_params(72, 56, cam, query_method=method))[:3]
            assert_parity(got, ref, f"codec block map nb={nb} m{method}")


@pytest.mark.parametrize("cap", ["1", "3"])
def test_codec_occupancy_cap(pkg, orc, gpu, cap, tune):
    """VR_WG_PER_CU reaches the codec march (its LDS request holds the template table at
    the front): results stay bit-identical, with and without the staged table"""
    import torch
    tune.set("VR_WG_PER_CU", cap)
    cb, t, e = orc.synth_codec(20, 16, 12, 8, seed=7)
    pkg.init_codec(cb, t, e)
    for lds in ("1", "0"):
        tune.set("VR_CODEC_LDS", lds)
        for method in (4, 5, 6):
            cam = pkg.camera.display_inv_view((30.0, 45.0))
            got = codec_render(pkg, 64, 48, cam, method, torch)
            ref = orc.render_codec(cb, t, e, orc.make_params(64, 48, cam, query_method=method))[:3]
            assert_parity(got, ref, f"codec cap {cap} lds {lds} m{method}")


def test_codec_via_reference_initCuda(pkg, orc, gpu):
    """the reference's own shapes: 50x50x10 voxels, 32 bins, templatesSize (32, T, 1),
    errorsbookSize (32, 2500, 10) -- initCuda with all codec arrays, then render_kernel
    with queryMethod 4/5/6 (C:1200-1203, K:1893-2050)"""
    import torch
    cb, t, e = orc.synth_codec(50, 50, 10, 32, ntemplates=40, seed=9)
    vol = orc.synth_volume(50, 50, 10, 32)
    pkg.initCuda(vol.reshape(-1), (50, 50, 10), (32, 2500, 10), cb.reshape(-1, 4), (50, 50, 10),
                 t, (32, 40, 1), e.reshape(-1, 2), (32, 2500, 10))
    m = pkg.camera.single_test_inv_view()
    pkg.copyInvViewMatrix(m, 48)
    W = H = 128
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for method in (4, 5, 6):
        out.zero_()
        pkg.render_kernel((W // 16, H // 16, 1), (16, 16, 1), out, W, H, 0.05, 1.0, 0.0, 1.0,
                          method, (50, 50, 10))
        torch.cuda.synchronize()
        ref = orc.render_codec(cb, t, e, orc.make_params(W, H, m, query_method=method))[0]
        assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref), method
    # methods 1/2/3 still read the raw histograms
    out.zero_()
    pkg.render_kernel((W // 16, H // 16, 1), (16, 16, 1), out, W, H, 0.05, 1.0, 0.0, 1.0, 1,
                      (50, 50, 10))
    torch.cuda.synchronize()
    ref = orc.render(vol, orc.make_params(W, H, m, query_method=1))[0]
    assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref)


def test_codec_validation(pkg, orc, gpu):
    cb, t, e = orc.synth_codec(6, 5, 4, 8)
    for field, value in ((0, 24), (1, 8), (1, -1), (3, 9)):
        bad = cb.copy()
        bad[1, 2, 3, field] = value
        with pytest.raises(pkg.VRError):
            pkg.init_codec(bad, t, e)
    pkg.init_codec(cb[..., :4], t, e)  # the unmodified volume is accepted


def test_synth_codec_matches_oracle(pkg, orc, gpu):
    """the on-device codec generator writes the oracle's codec volume, and methods 4/5/6
    render it identically"""
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    for (nx, ny, nz), nb, nt, slots in [((14, 11, 9), 8, 64, 4), ((9, 7, 5), 32, 16, 2),
                                        ((8, 8, 8), 4, 8, 0)]:
        pkg.synthesize_codec((nx, ny, nz), nb, nt, slots, seed=20261015)
        dims, b, t, s, pcb, ptp, per = pkg.codec_info()
        assert dims == (nx, ny, nz) and (b, t, s) == (nb, nt, slots)
        cb, tp, er = orc.synth_codec_field(nx, ny, nz, nb, nt, slots)
        got_cb = np.zeros_like(cb)
        got_tp = np.zeros_like(tp)
        got_er = np.zeros_like(er)
        torch.cuda.synchronize()
        assert hip.hipMemcpy(ctypes.c_void_p(got_cb.ctypes.data), ctypes.c_void_p(pcb),
                             ctypes.c_size_t(got_cb.nbytes), 2) == 0
        assert hip.hipMemcpy(ctypes.c_void_p(got_tp.ctypes.data), ctypes.c_void_p(ptp),
                             ctypes.c_size_t(got_tp.nbytes), 2) == 0
        if slots:
            assert hip.hipMemcpy(ctypes.c_void_p(got_er.ctypes.data), ctypes.c_void_p(per),
                                 ctypes.c_size_t(got_er.nbytes), 2) == 0
        assert np.array_equal(got_cb, cb) and np.array_equal(got_tp, tp)
        assert np.array_equal(got_er, er)
        for method in (4, 5, 6):
            m = pkg.camera.display_inv_view((20.0, 60.0))
            got = codec_render(pkg, 48, 40, m, method, torch)
            ref = orc.render_codec(cb, tp, er, orc.make_params(48, 40, m, query_method=method))[:3]
            assert_parity(got, ref, f"synth codec {nb} m{method}")


def test_codec_footprint_bytes(pkg, orc, gpu):
    """vr_footprint_bytes for methods 4/5/6 = sum over the distinct footprint voxels
    (numpy restatement) of 16 + 8 NE, plus the template table; methods 1/2/3 = U*B*4"""
    import torch
    import ref_numpy as R
    cb, t, e = orc.synth_codec(20, 16, 12, 8, seed=5)
    pkg.init_codec(cb, t, e)
    m = pkg.camera.display_inv_view()
    out = torch.zeros(64 * 48, dtype=torch.int32, device="cuda")
    for method in (4, 6):
        fp = set()
        R.render(R.codec_decode(cb, t, e), 64, 48, m, method, footprint=fp)
        ne = cb.reshape(-1, 4)[:, 3]
        expect = sum(16 + 8 * int(ne[v]) for v in fp) + t.size * 4
        d = pkg.make_desc(out, 64, 48, m, query_method=method, volume_size=(1, 1, 1))
        assert pkg.footprint_bytes(d) == expect
    vol = orc.synth_volume(20, 16, 12, 8)
    pkg.init_distribution(vol)
    d = pkg.make_desc(out, 64, 48, m, query_method=1)
    assert pkg.footprint_bytes(d) == pkg.count_footprint(d) * 8 * 4


def test_large_volume_64bit_offsets(pkg, orc, gpu):
    """4096 x 4096 x 36 voxels x 8 bins = 4.8e9 floats: record offsets and float
    offsets beyond 2^32, device-generated volume against the oracle's"""
    import torch
    nx, ny, nz, nb = 4096, 4096, 36, 8
    pkg.synthesize((nx, ny, nz), nb)
    m = pkg.camera.display_inv_view((25.0, -40.0))
    got = gpu_render(pkg, None, 96, 64, m, 1, torch)
    vol = orc.synth_volume(nx, ny, nz, nb)
    ref = orc.render(vol, orc.make_params(96, 64, m, query_method=1))[:3]
    del vol
    assert_parity(got, ref, "4096x4096x36x8")
    pkg.freeCudaBuffers()


# ---- flexible blocks (methods 8/9/0) ----

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

def _flex_blocks_from_device(pkg):
    import ctypes
    n, nb, ptr = pkg.flex_info()
    got = np.zeros((n, n, n, 4), np.float32)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), ctypes.c_void_p(ptr),
                         ctypes.c_size_t(got.nbytes), 2) == 0
    return got


@pytest.mark.parametrize("dim,block,nb", [(12, 5, 16), (20, 6, 64), (16, 3, 8), (9, 9, 4),
                                          (64, 6, 64)])
def test_flex_prepass_matches_oracle(pkg, orc, gpu, dim, block, nb):
    """vr_flex_process (sorted-key lookups, one workgroup per corner) == the oracle's
    linear-scan restatement of dataProcessing, bit for bit; 64^3 with 6-voxel blocks
    is the reference's own configuration (K:106, 1737)"""
    t = orc.synth_flex(dim, block, nb, ntemplates=9, seed=dim + 31 * block)
    ref = orc.flex_process(t)
    pkg.init_flex(t)
    assert pkg.flex_process(block) == orc.flex_blocks_per_axis(dim, block)
    got = _flex_blocks_from_device(pkg)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("method", [8, 9, 0])
def test_flex_render_matches_oracle(pkg, orc, gpu, method):
    """methods 8/9/0 through render_kernel after initCuda-free vr_init_flex + the
    reference entry point dataProcessing (6-voxel blocks), both cameras, early exits"""
    import torch
    t = orc.synth_flex(22, 6, 32, ntemplates=11, seed=5)
    pkg.init_flex(t)
    pkg.dataProcessing()
    blocks = orc.flex_process({**t, "block": 6})
    ts = {9: 1 / 255, 0: 1 / 4000, 8: 1.0}[method]
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0)),
                pkg.camera.display_inv_view((-60.0, 110.0))):
        for density in (0.05, 0.6):
            got = gpu_render(pkg, None, 72, 56, cam, method, torch, density=density, tscale=ts)
            ref = orc.render_flex(blocks, orc.make_params(72, 56, cam, density=density,
                                                          transfer_scale=ts,
                                                          query_method=method))[:3]
            assert_parity(got, ref, f"flex m{method} d={density}")
    assert pkg.last_kernel().startswith("k_march_flex")


def test_flex_golden_fixtures(pkg, gpu):
    """the committed flex fixtures (tables in the fixture, tests/golden/make_golden.py)"""
    import glob
    import torch
    files = sorted(glob.glob(os.path.join(GOLDEN_DIR, "flex*.npz")))
    assert files
    for path in files:
        z = np.load(path, allow_pickle=False)
        dim, block, nb = (int(v) for v in z["flex_dims"])
        pkg.init_flex({"dim": dim, "nbins": nb, **{k: z[k] for k in (
            "fractal_low", "fractal_high", "fractal_code", "fractal_err", "simple_low",
            "simple_high", "simple_count", "simple_hist", "templates")}})
        pkg.flex_process(block)
        assert np.array_equal(_flex_blocks_from_device(pkg).view(np.uint32),
                              z["blocks"].view(np.uint32)), path
        W, H = (int(v) for v in z["image"])
        got = gpu_render(pkg, None, W, H, z["inv_view"], int(z["method"]), torch,
                         density=float(z["density"]), tscale=float(z["tscale"]))
        assert_parity(got, (z["rgba8"], z["rgba_f"], z["steps"].astype(np.int32)), path)


def test_flex_through_initcuda(pkg, orc, gpu):
    """initCuda's arguments 10-18 at the reference's fixed sizes (64x64x32 entries,
    64 bins, 469 templates, 64^3 volume) then dataProcessing, as main() does
    (C:1200-1221)"""
    import torch
    t = orc.synth_flex(64, 6, 64, ntemplates=469, seed=11, extra=0, dup=False)
    N = 64 * 64 * 32

    def pad(a, fill=0):
        out = np.full((N,) + a.shape[1:], fill, a.dtype)
        out[:a.shape[0]] = a
        return out
    arrays = [pad(t["fractal_low"], -1), pad(t["fractal_high"], -1), pad(t["fractal_code"]),
              pad(t["fractal_err"]), pad(t["simple_low"], -1), pad(t["simple_high"], -1),
              pad(t["simple_count"]), pad(t["simple_hist"]), t["templates"]]
    vol = orc.synth_volume(8, 8, 8, 4)
    pkg.initCuda(vol, (8, 8, 8), (4, 512, 1), None, None, None, None, None, None, *arrays)
    pkg.dataProcessing()
    n, nb, _ = pkg.flex_info()
    assert (n, nb) == (11, 64)
    ref = orc.flex_process(t)
    assert np.array_equal(_flex_blocks_from_device(pkg).view(np.uint32), ref.view(np.uint32))
    m = pkg.camera.display_inv_view((30.0, 45.0))
    got = gpu_render(pkg, None, 48, 40, m, 8, torch)
    assert_parity(got, orc.render_flex(ref, orc.make_params(48, 40, m, query_method=8))[:3],
                  "flex via initCuda")
    # the histogram volume initCuda made resident is still there for methods 1/2/3
    got = gpu_render(pkg, None, 48, 40, m, 1, torch)
    assert_parity(got, orc.render(vol, orc.make_params(48, 40, m, query_method=1))[:3],
                  "method 1 next to flex")


def test_flex_errors(pkg, orc, gpu):
    import torch
    pkg.freeCudaBuffers()
    out = torch.zeros(16, dtype=torch.int32, device="cuda")
    for m in (8, 9, 0):
        with pytest.raises(pkg.VRError):
            pkg.render_kernel((1, 1, 1), (16, 16, 1), out, 4, 4, 0.05, 1.0, 0.0, 1.0, m,
                              (4, 4, 4))
    t = orc.synth_flex(10, 4, 8, dup=False, extra=0)
    pkg.init_flex(t)
    with pytest.raises(pkg.VRError):
        pkg.flex_process(11)  # block > dim
    with pytest.raises(pkg.VRError):  # tables resident but no statistics yet
        pkg.render_kernel((1, 1, 1), (16, 16, 1), out, 4, 4, 0.05, 1.0, 0.0, 1.0, 8, (4, 4, 4))
    for k in ("simple_low", "simple_high", "simple_count", "simple_hist"):
        t[k] = t[k][1:]
    pkg.init_flex(t)
    with pytest.raises(pkg.VRError, match="no table"):
        pkg.flex_process(4)
    pkg.freeCudaBuffers()


@pytest.mark.parametrize("quad", ["1", "0"])
def test_method7_oblique_kernels(pkg, orc, gpu, quad, tune):
    """method 7 on oblique views: the quad-cooperative march (grid = volume) and the
    one-lane pipelined march give the oracle's result bit for bit, including views
    where neighbouring rays refresh their cells at different steps"""
    import torch
    tune.set("VR_M7_QUAD", quad)
    vol = orc.synth_volume(30, 26, 22, 8)
    pkg.init_distribution(vol)
    for rot in ((30.0, 45.0), (-60.0, 110.0), (12.0, -70.0)):
        m = pkg.camera.display_inv_view(rot)
        for density in (0.05, 0.8):
            got = gpu_render(pkg, None, 88, 60, m, 7, torch, density=density)
            ref = orc.render(vol, orc.make_params(88, 60, m, query_method=7, density=density,
                                                  m7_dims=(30, 26, 22)))[:3]
            assert_parity(got, ref, f"m7 quad={quad} {rot} d={density}")
    assert pkg.last_kernel().startswith("k_march_m7_quad" if quad == "1" else "k_march_m7_pipe")


@pytest.mark.parametrize("dims", [(26, 22, 18), (25, 21, 17), (1, 3, 5), (7, 1, 4)])
@pytest.mark.parametrize("brick", ["1", "0"])
def test_quad_march_brick_layout(pkg, orc, gpu, dims, brick, tune):
    """oblique views of 8-bin volumes: the quad march reads the library's 2x2 (x, y)
    micro-brick copy of the records (odd widths / heights are padded to even in the
    copy); VR_BRICK=0 keeps the x rows.  Both bit-identical to the oracle, also for
    the tile lists of a multi-GPU rank"""
    import torch
    tune.set("VR_PATH", "0")
    tune.set("VR_BRICK", brick)
    vol = orc.synth_volume(*dims, 8)
    pkg.init_distribution(vol)
    want = "k_march_quad_brick<" if brick == "1" else "k_march_quad<"
    for rot in ((30.0, 45.0), (-60.0, 110.0), (12.0, -70.0)):
        m = pkg.camera.display_inv_view(rot)
        for method in (1, 2, 3, 7):
            got = gpu_render(pkg, None, 88, 60, m, method, torch)
            ref = orc.render(vol, orc.make_params(88, 60, m, query_method=method,
                                                  m7_dims=dims))[:3]
            assert_parity(got, ref, f"{dims} brick={brick} {rot} m{method}")
            assert pkg.last_kernel().startswith(want if method != 7 else
                                                want.replace("quad", "m7_quad"))
    W, H = 136, 72
    m = pkg.camera.display_inv_view((30.0, 45.0))
    full = gpu_render(pkg, None, W, H, m, 1, torch)[0]
    world = 3
    lists = pkg.tiles.tile_lists(W, H, world, m)
    n_slots = lists.shape[1]
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        # a short list takes two lanes per ray (k_march_quad2)
        assert pkg.last_kernel().startswith(want.replace("quad", "quad2"))
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), full)


@pytest.mark.parametrize("dims,nb,W,H,want", [
    ((40, 36, 32), 1, 256, 256, "k_march_segp4<"), ((40, 36, 32), 4, 512, 320, None),
    ((40, 36, 32), 8, 256, 200, "k_march_segp4<")])
def test_small_frames_take_segmented_march(pkg, orc, gpu, dims, nb, W, H, want):
    """small full frames run the pipelined ray-segmented march: 4 lanes per ray up to
    128 K rays; oblique views (B < 8) 4 lanes up to 400 K (round 4), 2 up to 700 K;
    row-aligned 4- and 8-bin frames above 128 K rays of a coarse volume take the box
    march with four samples per box (k_march_duo4, round 4); bit-identical"""
    import torch
    vol = orc.synth_volume(*dims, nb)
    pkg.init_distribution(vol)
    for cam in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))):
        for method in (1, 2):
            got = gpu_render(pkg, None, W, H, cam, method, torch)
            ref = orc.render(vol, orc.make_params(W, H, cam, query_method=method))[:3]
            assert_parity(got, ref, f"{dims}x{nb} {W}x{H} m{method}")
            rows = abs(float(cam[0])) >= 0.95
            k = want or ("k_march_duo4<" if rows else
                         "k_march_segp4<" if W * H <= 400000 else "k_march_segp2<")
            if nb < 8 or rows:
                assert pkg.last_kernel().startswith(k), pkg.last_kernel()


@pytest.mark.parametrize("nb,want", [(2, "k_march_pipe<"), (4, "k_march_duo4<"),
                                     (8, "k_march_duo4<")])
def test_midsize_rows_take_box_march_with_four_samples(pkg, orc, gpu, nb, want):
    """row-aligned full frames between 128 K and 700 K rays of a volume with >= 4
    pixels per voxel face (BASELINE config 2's shape): 4 and 8 bins, methods 1/2, on
    k_march_duo with four samples per box, 2 bins on the one-lane march; 8-bin
    entropy on k_march, 2- and 4-bin entropy on the one-lane march (round 6); rays
    ending on any sample of a box; bit-identical"""
    import torch
    vol = orc.synth_volume(44, 38, 30, nb)
    pkg.init_distribution(vol)
    W, H = 400, 360
    m = pkg.camera.single_test_inv_view()
    for method, density in ((1, 0.05), (2, 0.05), (1, 2.5), (2, 0.8), (3, 0.05)):
        got = gpu_render(pkg, None, W, H, m, method, torch, density=density)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method, density=density))[:3]
        assert_parity(got, ref, f"nb={nb} m{method} d={density}")
        # entropy: the one-sample box (8 bins); 2 and 4 bins the one-lane pipelined
        # march (round 6)
        k = want if method != 3 else "k_march<" if nb == 8 else "k_march_pipe<"
        assert pkg.last_kernel().startswith(k), (method, pkg.last_kernel())


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_small_frame_entropy_dispatch(pkg, orc, gpu, nb):
    """entropy of small and mid-size full frames with 1-4 bins (round 4): 2-lane
    windows for frames up to 128 K rays and for oblique frames up to 700 K, the LDS
    box for row-aligned frames of a coarse volume above 128 K rays; 2 and 4 bins
    on the one-lane pipelined march (round 6); bit-identical, dense and sparse
    (early exit) transfer"""
    import torch
    vol = orc.synth_volume(36, 30, 28, nb)
    pkg.init_distribution(vol)
    rows, obl = pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))
    # round 6: 2 and 4 bins on the one-lane pipelined march
    cases = ((rows, 200, 150, "k_march_segp2<"), (obl, 200, 150, "k_march_segp2<"),
             (rows, 400, 360, "k_march<"), (obl, 400, 360, "k_march_segp2<"))
    if nb != 1:
        cases = tuple((m, W, H, "k_march_pipe<") for m, W, H, _ in cases)
    for m, W, H, want in cases:
        for density in (0.05, 2.0):
            got = gpu_render(pkg, None, W, H, m, 3, torch, density=density)
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=3, density=density))[:3]
            assert_parity(got, ref, f"nb={nb} {W}x{H} d={density}")
            assert pkg.last_kernel().startswith(want), (W, H, pkg.last_kernel())


def test_environment_does_not_change_the_kernel(pkg, orc, gpu, monkeypatch):
    """the library reads no environment variables: a knob left set in the shell
    (VR_PATH, VR_SEG, VR_WG_PER_CU) changes nothing; vr_set_tuning does"""
    import torch
    vol = orc.synth_volume(26, 22, 18, 8)
    pkg.init_distribution(vol)
    pkg.clear_tuning()
    m = pkg.camera.single_test_inv_view()
    ref = orc.render(vol, orc.make_params(80, 64, m, query_method=1))[:3]
    got = gpu_render(pkg, None, 80, 64, m, 1, torch)
    default = pkg.last_kernel()
    assert_parity(got, ref, "default")
    for k, v in (("VR_PATH", "0"), ("VR_SEG", "4"), ("VR_WG_PER_CU", "1"), ("VR_BRICK", "0")):
        monkeypatch.setenv(k, v)
    got = gpu_render(pkg, None, 80, 64, m, 1, torch)
    assert pkg.last_kernel() == default, pkg.last_kernel()
    assert_parity(got, ref, "environment set")
    pkg.set_tuning("VR_PATH", "0")
    try:
        got = gpu_render(pkg, None, 80, 64, m, 1, torch)
        assert pkg.last_kernel().startswith("k_march_quad"), pkg.last_kernel()
        assert_parity(got, ref, "VR_PATH=0 through vr_set_tuning")
    finally:
        pkg.clear_tuning()



@pytest.mark.parametrize("nb", [1, 2, 4, 8])
def test_axis_views_segmented(pkg, orc, gpu, nb):
    """small frames and rank tile lists of views along the volume's z or y take the
    pipelined ray-segmented march over the axis-rows copy (k_march_segp4_zrows /
    segp2 / _yrows) by the default dispatch: bit-identical
    to the oracle, method 3 keeping the one-lane march (8 bins: the LDS-box march)"""
    import torch
    vol = orc.synth_volume(48, 40, 44, nb)
    pkg.init_distribution(vol)
    W, H = 88, 68
    for rot, kern in (((0.0, 90.0), "zrows"), ((90.0, 90.0), "yrows"), ((-10.0, -80.0), "zrows")):
        m = pkg.camera.display_inv_view(rot)
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            # (8-bin entropy: the LDS-box march on the x rows, no copy)
            want = (f"k_march_segp4_{kern}<" if method < 3 else "k_march<" if nb == 8
                    else f"k_march_pipe_{kern}<")
            assert pkg.last_kernel().startswith(want), pkg.last_kernel()
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            assert_parity(got, ref, f"segmented axis view {rot} nb={nb} m{method}")
        # a 3-rank split: each rank's packed list through the 2-lane windows
        lists = pkg.tiles.tile_lists(W, H, 3, m)
        n_slots = lists.shape[1]
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        for method in (1, 2):
            for r in range(3):
                pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=method,
                                         d_tile_list=dl[r], n_tiles=n_slots))
                assert pkg.last_kernel().startswith(f"k_march_segp2_{kern}<"), pkg.last_kernel()
            frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
            pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
            torch.cuda.synchronize()
            ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=method),
                              want_float=False, want_steps=False)[0]
            assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref8), (
                f"segmented axis lists {rot} nb={nb} m{method}")


@pytest.mark.parametrize("nb", [1, 2, 4, 8])
def test_axis_views_take_an_axis_rows_copy(pkg, orc, gpu, nb, tune):
    """views whose screen x runs along the volume's z or y (|M[8]| or |M[4]| >= 0.95)
    march an axis-rows copy with the per-ray pipelined march (ensure_axis_copy):
    full frames and rank tile lists bit-identical to the oracle, the copy
    dropped with the volume (a new volume renders its own frame) and by
    vr_release_stats, VR_ZROWS=0 keeps the x rows.  (Frames below the ray-segmented
    thresholds keep that march, so this small frame sets VR_SEG_RAYS=0 and a volume
    finer than the frame)"""
    import torch
    tune.set("VR_SEG_RAYS", "0")
    vol = orc.synth_volume(48, 40, 44, nb)
    pkg.init_distribution(vol)
    W, H = 88, 68
    # M[8] = cos rx sin ry (screen x along z), M[4] = sin rx sin ry (along y): the
    # copies of both axes, one resident at a time, alternating views rebuild them
    for rot, kern in (((0.0, 90.0), "zrows"), ((12.0, 95.0), "zrows"), ((90.0, 90.0), "yrows"),
                      ((-10.0, -80.0), "zrows"), ((80.0, 95.0), "yrows"),
                      ((-85.0, 80.0), "yrows"), ((8.0, 265.0), "zrows")):
        m = pkg.camera.display_inv_view(rot)
        assert abs(m[8 if kern == "zrows" else 4]) >= 0.95
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            # 8-bin entropy takes the LDS-box march on the x rows (the pipelined
            # march's unrolled 64 logarithms per step spill)
            want = "k_march<" if method == 3 and nb == 8 else f"k_march_pipe_{kern}<"
            assert pkg.last_kernel().startswith(want), pkg.last_kernel()
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            assert_parity(got, ref, f"axis view {rot} nb={nb} m{method}")
    # a rank's packed tile list
    m = pkg.camera.display_inv_view((0.0, 90.0))
    lists = pkg.tiles.tile_lists(W, H, 3, m)
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    packed = torch.full((3, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    for r in range(3):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        assert pkg.last_kernel().startswith("k_march_pipe_zrows<"), pkg.last_kernel()
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, 3, n_slots, frame, W, H)
    torch.cuda.synchronize()
    ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    assert np.array_equal(frame.cpu().numpy().view(np.uint32).reshape(H, W), ref8)
    # the copy follows the volume
    vol2 = orc.synth_volume(48, 40, 44, nb, seed=5)
    pkg.init_distribution(vol2)
    got = gpu_render(pkg, None, W, H, m, 1, torch)
    assert_parity(got, orc.render(vol2, orc.make_params(W, H, m, query_method=1))[:3], "vol2")
    pkg.release_stats()
    got = gpu_render(pkg, None, W, H, m, 2, torch)
    assert pkg.last_kernel().startswith("k_march_pipe_zrows<"), pkg.last_kernel()
    assert_parity(got, orc.render(vol2, orc.make_params(W, H, m, query_method=2))[:3], "rebuilt")
    tune.set("VR_ZROWS", "0")
    got = gpu_render(pkg, None, W, H, m, 1, torch)
    assert not pkg.last_kernel().startswith("k_march_pipe_zrows"), pkg.last_kernel()
    assert_parity(got, orc.render(vol2, orc.make_params(W, H, m, query_method=1))[:3], "x rows")


def test_wide32_row_aligned_frames_take_box_march(pkg, orc, gpu, tune):
    """32-bin records, row-aligned full frames above the segmented threshold, a
    volume fine for the frame: the LDS-box march with 16x4-pixel wave blocks
    (decode once per wave-step), methods 1/2/3, bit-identical; the 64-pixel-row
    box (VR_BOX_MAP=0) too"""
    import torch
    tune.set("VR_SEG_RAYS", "1000")
    vol = orc.synth_volume(60, 50, 20, 32)
    pkg.init_distribution(vol)
    m = pkg.camera.display_inv_view((0.0, 0.0), translation=(0.05, -0.1, 0.0))
    W, H = 96, 64  # 6144 rays < 4 x 60 x 50 pixels per voxel face
    for bmap in ("1", "0"):
        tune.set("VR_BOX_MAP", bmap)
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            assert pkg.last_kernel().startswith("k_march<B=32"), pkg.last_kernel()
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            assert_parity(got, ref, f"32 bins box map {bmap} m{method}")


@pytest.mark.parametrize("nb", [2, 8, 16, 32])
def test_block_map_m7_and_wide(pkg, orc, gpu, nb, tune):
    """VR_M7_MAP=1 / VR_WIDE_MAP=1: the one-lane method-7 marches and the 16-bin
    row march with a 16x4 pixel block per wave, bit-identical (method-7 grid equal
    to the volume and not; row-aligned and oblique views)"""
    import torch
    tune.set("VR_M7_MAP", "1")
    tune.set("VR_WIDE_MAP", "1")
    tune.set("VR_M7_WQ", "0")
    tune.set("VR_M7_QUAD", "0")
    vol = orc.synth_volume(21, 18, 15, nb)
    pkg.init_distribution(vol)
    W, H = 80, 56
    for m in (pkg.camera.single_test_inv_view(), pkg.camera.display_inv_view((30.0, 45.0))):
        for grid in ((21, 18, 15), (10, 12, 20)):
            got = gpu_render(pkg, None, W, H, m, 7, torch, m7=grid)
            assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=7,
                                                               m7_dims=grid))[:3],
                          f"{nb} bins m7 grid {grid} block map")
            assert pkg.last_kernel().startswith("k_march_m7"), pkg.last_kernel()
    if nb == 16:
        tune.set("VR_WIDE", "1")
        tune.set("VR_PATH", "2")
        m = pkg.camera.single_test_inv_view()
        for method in (1, 2):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            assert pkg.last_kernel().startswith("k_march_wide<"), pkg.last_kernel()
            assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3],
                          f"wide block map m{method}")
