"""Parity at the BASELINE.json sizes: whole frames at the benchmark resolutions.

The reference's only automated check compares its whole benchmark frame with a
golden image (runSingleTest, C:1073-1077, sdkComparePPM with the constants of
C:57-58).  Here every BASELINE config that fits one GPU renders its whole frame
through the library's DEFAULT kernel dispatch (no tuning knobs: the kernels the
bench and a user get at these sizes) and is compared with the oracle's frame of
the same seeded volume:
  config 1  128^3 x 1  at 256 x 256      (the reference's CPU plumbing case)
  config 2  256^3 x 4  at 512 x 512
  config 3  512^3 x 8  at 1920 x 1080
  config 4  1024^3 x 8 at 1920 x 1080    (the headline: 32 GiB volume)
Bar (BASELINE.json north_star): packed RGBA8 identical, float RGBA within 1e-4
per channel, samples per pixel identical -- for the first frame of a view
(estimate tile order) and the second (the order re-dealt by measured tile
costs).  Config 4 also checks the rank lists of the 8-GPU image split and the
baked statistics.  Config 5 (2048^3 x 16 GMM, 1.65 TB) cannot be resident on one
GPU; its slab chain is checked bit-exactly at smaller sizes (test_gpu_gmm.py).
"""
import numpy as np
import pytest

from test_gpu_parity import TOL, assert_parity

pytestmark = pytest.mark.gpu

SEED = 20261015
CONFIGS = {  # name: (edge, bins, W, H)
    "128x1": (128, 1, 256, 256),
    "256x4": (256, 4, 512, 512),
    "512x8": (512, 8, 1920, 1080),
    "1024x8": (1024, 8, 1920, 1080),
}


class _Scene:
    """one resident config at a time: the library's synthetic volume in HBM and
    the oracle's identical host copy (32 GiB at 1024^3)"""
    name = None
    vol = None


_scene = _Scene()


def scene(pkg, orc, name):
    if _scene.name != name:
        _scene.vol = None
        n, nb, _, _ = CONFIGS[name]
        pkg.clear_tuning()
        pkg.freeCudaBuffers()
        pkg.synthesize((n, n, n), nb, SEED)
        _scene.vol = orc.synth_volume(n, n, n, nb, SEED)
        _scene.name = name
    return _scene.vol


@pytest.fixture(scope="module", autouse=True)
def _release(pkg):
    yield
    _scene.vol = None
    _scene.name = None
    pkg.freeCudaBuffers()


def camera(pkg, cam):
    """C0 runSingleTest (C:1024-1043), C1 display() at (30, 45) deg, S a side view
    (display() at yaw 90: screen x along the volume's z, the z-rows copy)"""
    if cam == "C0":
        return pkg.camera.single_test_inv_view()
    return pkg.camera.display_inv_view((0.0, 90.0) if cam == "S" else (30.0, 45.0))


def render_frames(pkg, torch, W, H, m, method, n_frames=2, volume_size=None):
    """n_frames consecutive renders of one view (caller-zeroed output, C:208)"""
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    out_f = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
    steps = torch.full((W * H,), -2, dtype=torch.int32, device="cuda")
    frames = []
    for _ in range(n_frames):
        out.zero_()
        out_f.zero_()
        steps.fill_(-2)
        pkg.render(pkg.make_desc(out, W, H, m, query_method=method, volume_size=volume_size,
                                 d_output_f=out_f, d_steps=steps))
        torch.cuda.synchronize()
        frames.append((out.cpu().numpy().view(np.uint32).reshape(H, W).copy(),
                       out_f.cpu().numpy().reshape(H, W, 4).copy(),
                       steps.cpu().numpy().reshape(H, W).copy(), pkg.last_kernel()))
    return frames


@pytest.mark.parametrize("name,cam,method", [
    ("128x1", "C0", 1), ("128x1", "C1", 1), ("128x1", "C0", 2), ("128x1", "C1", 7),
    ("256x4", "C0", 1), ("256x4", "C1", 1), ("256x4", "C0", 3), ("256x4", "C1", 2),
    ("512x8", "C0", 1), ("512x8", "C1", 1), ("512x8", "C0", 2), ("512x8", "C1", 2),
    ("512x8", "C0", 3), ("512x8", "C1", 7), ("512x8", "S", 1),
    ("1024x8", "C0", 1), ("1024x8", "C1", 1), ("1024x8", "C0", 2), ("1024x8", "C1", 2),
    ("1024x8", "C0", 7), ("1024x8", "S", 1), ("1024x8", "S", 3),
])
def test_full_frame(pkg, orc, gpu, name, cam, method):
    import torch
    n, nb, W, H = CONFIGS[name]
    vol = scene(pkg, orc, name)
    m = camera(pkg, cam)
    ref = orc.render(vol, orc.make_params(W, H, m, query_method=method, m7_dims=(n, n, n)))[:3]
    assert int(np.sum(ref[2] >= 0)) > W * H // 4  # the box covers ~44 % of the frame
    for k, got in enumerate(render_frames(pkg, torch, W, H, m, method,
                                          volume_size=(n, n, n))):
        assert_parity(got[:3], ref, f"{name} {cam} m{method} frame {k} ({got[3]})")


@pytest.mark.parametrize("name,cam", [("256x4", "C0"), ("512x8", "C0"), ("512x8", "C1"),
                                      ("1024x8", "C0"), ("1024x8", "C1"), ("1024x8", "S")])
def test_footprint_count_at_size(pkg, orc, gpu, name, cam):
    """U of SURVEY.md 8(d) -- the distinct records under every sample's footprint,
    the numerator of the bench's roofline -- counted on the GPU
    (vr_count_footprint) equals the oracle's count of the same frame at the
    BASELINE size (1024^3 x 8 C0: 220 435 750, C1: 399 031 053;
    tools/oracle_footprint.py, profiles/r03/oracle_U_1024x8.log)"""
    import torch
    n, nb, W, H = CONFIGS[name]
    vol = scene(pkg, orc, name)
    m = camera(pkg, cam)
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for method in (1, 3):
        u = pkg.count_footprint(pkg.make_desc(out, W, H, m, query_method=method))
        ref = orc.count_footprint(vol, orc.make_params(W, H, m, query_method=method))
        assert u == ref, f"{name} {cam} m{method}: GPU U {u} != oracle {ref}"
        if (name, cam, method) == ("1024x8", "C0", 1):
            assert u == 220435750
        if (name, cam, method) == ("1024x8", "C1", 1):
            assert u == 399031053


@pytest.mark.parametrize("cam", ["C0", "C1", "S"])
def test_full_frame_baked(pkg, orc, gpu, cam):
    """config 4 after basicDataProcessing (the reference's own order, C:1200-1221):
    frames filter the baked statistics planes (the side view S: the method's
    plane's z-rows copy, round 4)"""
    import torch
    n, nb, W, H = CONFIGS["1024x8"]
    vol = scene(pkg, orc, "1024x8")
    pkg.bake_stats()
    try:
        m = camera(pkg, cam)
        for method in (1, 3):
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            got = render_frames(pkg, torch, W, H, m, method, n_frames=1)[0]
            assert_parity(got[:3], ref, f"baked 1024x8 {cam} m{method} ({got[3]})")
            if cam == "S":
                assert "plane_zrows" in got[3], got[3]
            if cam == "C1":  # the 8 x 2 x 2 brick copy (round 5)
                assert "plane8" in got[3], got[3]
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("cam", ["C0", "C1", "S"])
def test_rank_lists_of_eight_gpus(pkg, orc, gpu, cam):
    """config 4 split over 8 ranks as bench.py deals it (estimate lists, then the
    measured-cost re-deal): each rank's packed tiles through the kernel the rank
    would run, assembled by k_unscatter, equal the oracle's frame"""
    import torch
    n, nb, W, H = CONFIGS["1024x8"]
    vol = scene(pkg, orc, "1024x8")
    m = camera(pkg, cam)
    ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    world = 8
    ntiles = pkg.tiles.tiles_x(W) * pkg.tiles.tiles_y(H)
    lists = pkg.tiles.tile_lists(W, H, world, m)
    for deal in ("estimate", "cost"):
        n_slots = lists.shape[1]
        dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
        packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32,
                            device="cuda")
        steps = torch.full((world, n_slots * 256), -1, dtype=torch.int32, device="cuda")
        kernels = set()
        for r in range(world):
            pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=1, d_tile_list=dl[r],
                                     n_tiles=n_slots, d_steps=steps[r]))
            kernels.add(pkg.last_kernel())
        frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
        torch.cuda.synchronize()
        got = frame.cpu().numpy().view(np.uint32).reshape(H, W)
        assert np.array_equal(got, ref8), (
            f"{cam} {deal} deal ({kernels}): {int(np.sum(got != ref8))} pixels differ")
        st = steps.cpu().numpy()
        cost = sum(pkg.tiles.tile_costs_from_steps(st[r], lists[r], ntiles) for r in range(world))
        lists = pkg.tiles.tile_lists_by_cost(W, H, world, cost)


def test_render_kernel_grid_covers_the_frame(pkg, orc, gpu):
    """render_kernel with the reference's launch shape (C:122, 1231: 16x16 blocks,
    ceil(W/16) x ceil(H/16)) at config 3 renders the oracle's whole frame; a grid
    that covers only part of the image renders exactly that part (K:282-286)"""
    import torch
    n, nb, W, H = CONFIGS["512x8"]
    vol = scene(pkg, orc, "512x8")
    m = camera(pkg, "C0")
    pkg.copyInvViewMatrix(m, 48)
    ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                      want_steps=False)[0]
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for grid, block, cw, ch in (((120, 68, 1), (16, 16, 1), W, H),
                                ((50, 30, 1), (16, 16, 1), 800, 480),
                                ((7, 1, 1), (256, 1, 1), 1792, 1),
                                ((200, 200, 1), (16, 16, 1), W, H)):
        out.zero_()
        pkg.render_kernel(grid, block, out, W, H, 0.05, 1.0, 0.0, 1.0, 1, (n, n, n))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32).reshape(H, W)
        want = np.zeros_like(ref8)
        want[:ch, :cw] = ref8[:ch, :cw]
        assert np.array_equal(got, want), f"grid {grid} block {block}: {int(np.sum(got != want))}"
    for grid, block in (((0, 1, 1), (16, 16, 1)), ((1, 1, 1), (64, 32, 1)), ((4, 4, 1), (0, 1, 1))):
        out.zero_()
        with pytest.raises(pkg.VRError):
            pkg.render_kernel(grid, block, out, W, H, 0.05, 1.0, 0.0, 1.0, 1, (n, n, n))
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(out)) == 0
    assert TOL == 1e-4


@pytest.mark.parametrize("cam", ["C0", "C1", "S"])
def test_wide_entropy_at_size(pkg, orc, gpu, cam):
    """32-bin records (the reference's width, C:86-87) at 1080p, entropy (method 3):
    the LDS-box march with the rolled per-bin sums over LDS record columns (round
    4) -- row-aligned, and since round 6 the oblique and side views of this coarse
    volume too -- every 8th row against the oracle"""
    import torch
    n, nb, W, H = 512, 32, 1920, 1080
    _scene.vol = None
    _scene.name = None
    pkg.freeCudaBuffers()
    pkg.synthesize((n, n, n), nb, SEED)
    vol = orc.synth_volume(n, n, n, nb, SEED)
    try:
        m = camera(pkg, cam)
        got = render_frames(pkg, torch, W, H, m, 3, n_frames=1)[0]
        want = "k_march<B=32,M=3>"
        assert got[3] == want, got[3]
        ref = orc.render(vol, orc.make_params(W, H, m, query_method=3), row_stride=8)[:3]
        rows = slice(0, None, 8)
        assert_parity(tuple(a[rows] for a in got[:3]), tuple(a[rows] for a in ref),
                      f"512x32 {cam} m3")
    finally:
        del vol
        pkg.freeCudaBuffers()
