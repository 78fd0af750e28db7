"""Seeded random parity sweep: every case draws a volume shape, bin count, camera
(any rotation, translations that put the eye outside, at the edge of or inside
the volume), image size, method, render parameters, kernel path override and
statistics source (per-step decode / baked), renders through the C-ABI and
compares with the oracle.  Same bar as test_gpu_parity.py: packed RGBA8 and
samples per pixel identical, float RGBA within 1e-4.  Cases are reproducible
from their seed (printed in the failure message)."""
import numpy as np
import pytest

from test_gpu_parity import assert_parity, codec_render, gpu_render

pytestmark = pytest.mark.gpu

# kernel-path overrides a case may take (vr_api.cpp fill_params / baked_path)
PATHS = [{}, {}, {"VR_PATH": "0"}, {"VR_PATH": "1"}, {"VR_PATH": "1", "VR_BOX_MAX": "64"},
         {"VR_PATH": "2"}, {"VR_PATH": "4"}, {"VR_PATH": "7", "VR_SEG": "-4"},
         {"VR_PATH": "7", "VR_SEG": "-2"}, {"VR_PATH": "7", "VR_SEG": "4"}, {"VR_WG_PER_CU": "2"},
         {"VR_PATH": "0", "VR_QUAD2": "1"}]


def draw_camera(pkg, rng):
    kind = rng.integers(0, 4)
    if kind == 0:  # row-aligned (runSingleTest family), shifted / zoomed
        return pkg.camera.display_inv_view(
            (0.0, 0.0), (rng.uniform(-0.6, 0.6), rng.uniform(-0.6, 0.6), -rng.uniform(1.2, 6.0)))
    if kind == 1:  # axis-aligned quarter turns
        rx, ry = (float(rng.choice([0, 90, 180, 270])) for _ in range(2))
        return pkg.camera.display_inv_view((rx, ry), (0.0, 0.0, -rng.uniform(2.5, 5.0)))
    if kind == 2:  # eye inside the volume
        return pkg.camera.display_inv_view(
            (rng.uniform(-180, 180), rng.uniform(-180, 180)),
            (rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5)))
    return pkg.camera.display_inv_view(
        (rng.uniform(-180, 180), rng.uniform(-180, 180)),
        (rng.uniform(-0.4, 0.4), rng.uniform(-0.4, 0.4), -rng.uniform(1.5, 6.0)))


def draw_params(rng):
    return dict(density=float(np.float32(rng.uniform(0.01, 1.0))),
                brightness=float(np.float32(rng.uniform(0.5, 2.0))),
                toff=float(np.float32(rng.uniform(-0.2, 0.2))),
                tscale=float(np.float32(rng.uniform(0.5, 2.0))))


@pytest.mark.parametrize("seed", range(200))
def test_random_histogram_case(pkg, orc, gpu, seed, tune):
    import torch
    rng = np.random.default_rng(1000 + seed)
    dims = tuple(int(v) for v in rng.integers(2, 41, 3))
    nb = int(rng.choice([1, 2, 3, 4, 5, 8, 8, 8, 16, 32]))
    W, H = int(rng.integers(1, 161)), int(rng.integers(1, 121))
    method = int(rng.choice([1, 2, 3, 7]))
    m = draw_camera(pkg, rng)
    prm = draw_params(rng)
    env = PATHS[int(rng.integers(0, len(PATHS)))]
    baked = bool(rng.integers(0, 3) == 0)
    m7 = tuple(int(v) for v in rng.integers(2, 41, 3)) if rng.integers(0, 2) else dims
    for k, v in env.items():
        tune.set(k, v)
    vol = orc.synth_volume(*dims, nb, seed=seed)
    pkg.init_distribution(vol)
    if baked:
        pkg.bake_stats()
    try:
        got = gpu_render(pkg, None, W, H, m, method, torch, m7=m7 if method == 7 else None, **prm)
        ref = orc.render(vol, orc.make_params(
            W, H, m, density=prm["density"], brightness=prm["brightness"],
            transfer_offset=prm["toff"], transfer_scale=prm["tscale"], query_method=method,
            m7_dims=m7))[:3]
        assert_parity(got, ref, f"seed {seed}: {dims}x{nb} {W}x{H} m{method} env {env} "
                                f"baked {baked} kernel {pkg.last_kernel()}")
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("seed", range(40))
def test_random_tile_list_case(pkg, orc, gpu, seed, tune):
    """a multi-GPU split of a random frame: every rank's tile list rendered through
    the kernel the library picks for a list of that size (or a random path
    override), the packed slots assembled by k_unscatter, equals the oracle frame"""
    import torch
    rng = np.random.default_rng(3000 + seed)
    dims = tuple(int(v) for v in rng.integers(2, 41, 3))
    nb = int(rng.choice([1, 2, 4, 8, 8, 8]))
    W, H = int(rng.integers(1, 321)), int(rng.integers(1, 201))
    method = int(rng.choice([1, 2, 3]))
    world = int(rng.integers(2, 9))
    m = draw_camera(pkg, rng)
    prm = draw_params(rng)
    env = PATHS[int(rng.integers(0, len(PATHS)))]
    for k, v in env.items():
        tune.set(k, v)
    vol = orc.synth_volume(*dims, nb, seed=seed)
    pkg.init_distribution(vol)
    ref = orc.render(vol, orc.make_params(
        W, H, m, density=prm["density"], brightness=prm["brightness"],
        transfer_offset=prm["toff"], transfer_scale=prm["tscale"], query_method=method),
        want_float=False, want_steps=False)[0]
    lists = pkg.tiles.tile_lists(W, H, world, m)
    n_slots = lists.shape[1]
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    kernels = set()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=method, d_tile_list=dl[r],
                                 n_tiles=n_slots, density=prm["density"],
                                 brightness=prm["brightness"], transfer_offset=prm["toff"],
                                 transfer_scale=prm["tscale"]))
        kernels.add(pkg.last_kernel())
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    got = frame.cpu().numpy().view(np.uint32).reshape(H, W)
    assert np.array_equal(got, ref), (
        f"seed {seed}: {dims}x{nb} {W}x{H} m{method} world {world} env {env} {kernels}: "
        f"{int(np.sum(got != ref))} pixels differ")


@pytest.mark.parametrize("seed", range(48))
def test_random_codec_case(pkg, orc, gpu, seed):
    import torch
    rng = np.random.default_rng(2000 + seed)
    dims = tuple(int(v) for v in rng.integers(2, 33, 3))
    nb = int(rng.choice([1, 2, 4, 8, 16, 32]))
    W, H = int(rng.integers(1, 129)), int(rng.integers(1, 97))
    method = int(rng.choice([4, 5, 6]))
    m = draw_camera(pkg, rng)
    baked = bool(rng.integers(0, 3) == 0)
    cb, t, e = orc.synth_codec(*dims, nb, ntemplates=int(rng.integers(1, 40)),
                               slots=int(rng.integers(0, nb + 1)), seed=seed)
    pkg.init_codec(cb, t, e)
    if baked:
        pkg.bake_stats()
    try:
        got = codec_render(pkg, W, H, m, method, torch)
        ref = orc.render_codec(cb, t, e, orc.make_params(W, H, m, query_method=method))[:3]
        assert_parity(got, ref, f"seed {seed}: codec {dims}x{nb} {W}x{H} m{method} baked {baked}")
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("seed", range(40))
def test_random_gmm_case(pkg, orc, gpu, seed):
    import torch
    from test_gpu_gmm import check, gmm_render
    rng = np.random.default_rng(3000 + seed)
    dims = tuple(int(v) for v in rng.integers(2, 31, 3))
    K = int(rng.choice([8, 16, 32]))
    W, H = int(rng.integers(1, 129)), int(rng.integers(1, 97))
    method = int(rng.choice([1, 2]))
    m = draw_camera(pkg, rng)
    density = float(np.float32(rng.uniform(0.02, 0.8)))
    wm, sg = orc.synth_gmm(*dims, K, seed=seed)
    pkg.init_gmm(wm, sg)
    got = gmm_render(pkg, W, H, m, method, torch, density=density)
    ref = orc.render_gmm(wm, sg, dims, orc.make_params(W, H, m, query_method=method,
                                                       density=density))
    check(got, ref, f"seed {seed}: GMM {dims} K={K} {W}x{H} m{method}")
    pkg.free_gmm()


def draw_dispatch_camera(pkg, rng):
    """views around the library's kernel-choice thresholds (vr_api.cpp fill_params):
    screen x near the voxel rows' 0.95 cosine, along the volume's z (side views) or
    y (top views), row-aligned and oblique"""
    kind = int(rng.integers(0, 5))
    dist = -float(rng.uniform(2.2, 4.5))
    if kind == 0:  # yaw across the 18.2 deg row-aligned / oblique threshold
        ang = (float(rng.uniform(-12, 12)), float(rng.choice([-1, 1]) * rng.uniform(14, 23)))
    elif kind == 1:  # side views: screen x along z
        ang = (float(rng.uniform(-12, 12)), float(rng.choice([90, 270]) + rng.uniform(-12, 12)))
    elif kind == 2:  # top views: screen x along y
        ang = (float(rng.choice([90, 270]) + rng.uniform(-12, 12)),
               float(90 + rng.uniform(-12, 12)))
    elif kind == 3:
        ang = (0.0, 0.0)
    else:
        ang = (float(rng.uniform(-180, 180)), float(rng.uniform(-180, 180)))
    return pkg.camera.display_inv_view(ang, (float(rng.uniform(-0.3, 0.3)),
                                             float(rng.uniform(-0.3, 0.3)), dist)), kind, ang


@pytest.mark.parametrize("seed", range(48))
def test_random_midsize_default_dispatch(pkg, orc, gpu, seed):
    """mid-size volumes (64-192 voxels an axis) and frames (up to 800 x 600) through
    the library's own kernel choice -- no tuning knobs -- so the size- and
    view-dependent dispatch (LDS box for coarse row-aligned frames, micro-brick and
    axis-rows copies, wide-record marches, baked planes) is exercised at the shapes
    it is tuned for, whole frames against the oracle"""
    import torch
    rng = np.random.default_rng(3000 + seed)
    dims = tuple(int(v) for v in rng.integers(64, 193, 3))
    nb = int(rng.choice([1, 2, 4, 8, 8, 8, 16, 32]))
    W, H = int(rng.integers(320, 801)), int(rng.integers(240, 601))
    method = int(rng.choice([1, 1, 2, 3, 7]))
    m, kind, ang = draw_dispatch_camera(pkg, rng)
    baked = bool(rng.integers(0, 3) == 0)
    vol = orc.synth_volume(*dims, nb, seed=seed)
    pkg.init_distribution(vol)
    if baked:
        pkg.bake_stats()
    try:
        got = gpu_render(pkg, None, W, H, m, method, torch, m7=dims if method == 7 else None)
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method, m7_dims=dims))[:3]
        what = (f"seed {seed}: {dims}x{nb} {W}x{H} m{method} view {kind} "
                f"({ang[0]:.1f}, {ang[1]:.1f}) baked {baked} kernel {pkg.last_kernel()}")
        print(what)
        assert_parity(got, ref, what)
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("seed", range(24))
def test_random_midsize_tile_lists_default_dispatch(pkg, orc, gpu, seed):
    """multi-GPU splits of mid-size frames (up to 1280 x 800, 1-8 ranks: tile lists
    of ~30 K to ~1 M rays, across the library's 400 K / 700 K ray thresholds for
    the ray-segmented, two-lanes-per-ray quad and one-lane marches) through the
    default dispatch, per-step or baked, assembled by k_unscatter, against the
    oracle frame"""
    import torch
    rng = np.random.default_rng(4000 + seed)
    dims = tuple(int(v) for v in rng.integers(64, 161, 3))
    nb = int(rng.choice([1, 4, 8, 8, 8]))
    W, H = int(rng.integers(480, 1281)), int(rng.integers(320, 801))
    method = int(rng.choice([1, 1, 2, 3]))
    world = int(rng.choice([1, 2, 3, 4, 8]))
    m, kind, ang = draw_dispatch_camera(pkg, rng)
    baked = bool(rng.integers(0, 3) == 0)
    vol = orc.synth_volume(*dims, nb, seed=seed)
    pkg.init_distribution(vol)
    if baked:
        pkg.bake_stats()
    try:
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=method),
                         want_float=False, want_steps=False)[0]
        lists = pkg.tiles.tile_lists(W, H, world, m)
        n_slots = lists.shape[1]
        packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        kernels = set()
        for r in range(world):
            pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=method, d_tile_list=dl[r],
                                     n_tiles=n_slots))
            kernels.add(pkg.last_kernel())
        frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
        torch.cuda.synchronize()
        got = frame.cpu().numpy().view(np.uint32).reshape(H, W)
        what = (f"seed {seed}: {dims}x{nb} {W}x{H} m{method} world {world} "
                f"({n_slots * 256} rays a list) view {kind} ({ang[0]:.1f}, {ang[1]:.1f}) "
                f"baked {baked} {sorted(kernels)}")
        print(what)
        assert np.array_equal(got, ref), f"{what}: {int(np.sum(got != ref))} pixels differ"
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("seed", range(16))
def test_random_midsize_codec_default_dispatch(pkg, orc, gpu, seed):
    """fractal/template codec volumes (methods 4/5/6) of 48-128 voxels an axis at
    frames up to 640 x 480 through the default dispatch (codec marches chosen by
    view and bin count), per-step or baked, against the oracle"""
    import torch
    rng = np.random.default_rng(5000 + seed)
    dims = tuple(int(v) for v in rng.integers(48, 129, 3))
    nb = int(rng.choice([4, 8, 8, 16, 32]))
    W, H = int(rng.integers(240, 641)), int(rng.integers(160, 481))
    method = int(rng.choice([4, 5, 6]))
    m, kind, ang = draw_dispatch_camera(pkg, rng)
    baked = bool(rng.integers(0, 3) == 0)
    cb, t, e = orc.synth_codec(*dims, nb, ntemplates=int(rng.integers(8, 65)),
                               slots=int(rng.integers(0, min(nb, 8) + 1)), seed=seed)
    pkg.init_codec(cb, t, e)
    if baked:
        pkg.bake_stats()
    try:
        got = codec_render(pkg, W, H, m, method, torch)
        ref = orc.render_codec(cb, t, e, orc.make_params(W, H, m, query_method=method))[:3]
        what = (f"seed {seed}: codec {dims}x{nb} {W}x{H} m{method} view {kind} "
                f"({ang[0]:.1f}, {ang[1]:.1f}) baked {baked} kernel {pkg.last_kernel()}")
        print(what)
        assert_parity(got, ref, what)
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("seed", range(12))
def test_random_midsize_gmm_default_dispatch(pkg, orc, gpu, seed):
    """GMM volumes (K = 8 / 16 / 32) of 40-96 voxels an axis at frames up to
    512 x 384 against the oracle's GMM march"""
    import torch
    from test_gpu_gmm import check, gmm_render
    rng = np.random.default_rng(6000 + seed)
    dims = tuple(int(v) for v in rng.integers(40, 97, 3))
    K = int(rng.choice([8, 16, 32]))
    W, H = int(rng.integers(192, 513)), int(rng.integers(128, 385))
    method = int(rng.choice([1, 2]))
    m, kind, ang = draw_dispatch_camera(pkg, rng)
    wm, sg = orc.synth_gmm(*dims, K, seed=seed)
    pkg.init_gmm(wm, sg)
    try:
        got = gmm_render(pkg, W, H, m, method, torch)
        ref = orc.render_gmm(wm, sg, dims, orc.make_params(W, H, m, query_method=method))
        what = (f"seed {seed}: GMM {dims} K={K} {W}x{H} m{method} view {kind} "
                f"({ang[0]:.1f}, {ang[1]:.1f}) kernel {pkg.last_kernel()}")
        print(what)
        check(got, ref, what)
    finally:
        pkg.free_gmm()
