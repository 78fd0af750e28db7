"""GPU: round-4 dispatch pieces against the oracle.

* the head split of a rank's tile list (k_march_seg_head / k_march_pipe_head:
  the first slots of every XCD sublist with more lanes per ray in the same
  launch) assembles the full frame bit for bit;
* layout copies obey vr_set_layout_budget, keep both axis copies when they
  fit, and report their build cost (vr_layout_info).
"""
import numpy as np
import pytest

from test_gpu_parity import assert_parity, gpu_render

pytestmark = pytest.mark.gpu


def _split_frame(pkg, torch, W, H, m, world, method, lists=None):
    lists = pkg.tiles.tile_lists(W, H, world, m) if lists is None else lists
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    packed = torch.full((world, n_slots * 256), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    kernels = set()
    for r in range(world):
        pkg.render(pkg.make_desc(packed[r], W, H, m, query_method=method, d_tile_list=dl[r],
                                 n_tiles=n_slots))
        kernels.add(pkg.last_kernel())
    frame = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    pkg.unscatter_tiles(packed, dl, world, n_slots, frame, W, H)
    torch.cuda.synchronize()
    return frame.cpu().numpy().view(np.uint32).reshape(H, W), kernels


@pytest.mark.parametrize("lanes", ["-2", "-4", "-8"])
@pytest.mark.parametrize("tail", ["0", "1"])
def test_head_split_tile_lists(pkg, orc, gpu, tune, lanes, tail):
    """VR_HEAD slots of each rank's list with VR_HEAD_SEG lanes per ray, the rest on
    2-lane windows (tail 0) or one lane per ray (tail 1), in one launch: the
    assembled frame equals the oracle's, row-aligned (x rows) and side views
    (z-rows copy), methods 1 and 2, heads shorter and longer than a list"""
    import torch
    vol = orc.synth_volume(40, 36, 44, 8)
    pkg.init_distribution(vol)
    W, H = 200, 136
    tune.set("VR_HEAD_SEG", lanes)
    tune.set("VR_HEAD_TAIL", tail)
    for rot in (None, (0.0, 90.0)):
        m = pkg.camera.single_test_inv_view() if rot is None else pkg.camera.display_inv_view(rot)
        for head in ("8", "16", "4096"):
            tune.set("VR_HEAD", head)
            for method in (1, 2):
                got, kernels = _split_frame(pkg, torch, W, H, m, 3, method)
                ref = orc.render(vol, orc.make_params(W, H, m, query_method=method),
                                 want_float=False, want_steps=False)[0]
                assert np.array_equal(got, ref), (rot, head, method, kernels)
                want = "_head_pipe" if tail == "1" else "_head_segp2"
                if head != "4096":  # a head covering the whole list: the plain march
                    assert all(want in k for k in kernels), kernels


def test_head_split_with_output_buffers(pkg, orc, gpu, tune):
    """float RGBA and samples per pixel of a head-split list land in the list's packed
    slots like the packed RGBA8 (the oracle's pixels of those tiles)"""
    import torch
    vol = orc.synth_volume(40, 36, 44, 8)
    pkg.init_distribution(vol)
    W, H = 200, 136
    m = pkg.camera.single_test_inv_view()
    tune.set("VR_HEAD", "8")
    lists = pkg.tiles.tile_lists(W, H, 2, m)
    n_slots = lists.shape[1]
    dl = torch.from_numpy(lists.view(np.int32).copy()).cuda()
    out = torch.zeros(n_slots * 256, dtype=torch.int32, device="cuda")
    out_f = torch.zeros(n_slots * 256 * 4, dtype=torch.float32, device="cuda")
    steps = torch.full((n_slots * 256,), -2, dtype=torch.int32, device="cuda")
    pkg.render(pkg.make_desc(out, W, H, m, query_method=1, d_tile_list=dl[0], n_tiles=n_slots,
                             d_output_f=out_f, d_steps=steps))
    torch.cuda.synchronize()
    assert "_head_" in pkg.last_kernel()
    r8, rf, rn, _ = orc.render(vol, orc.make_params(W, H, m, query_method=1))
    tx = pkg.tiles.tiles_x(W)
    o8, of, on = out.cpu().numpy().view(np.uint32), out_f.cpu().numpy().reshape(-1, 4), steps.cpu().numpy()
    for s, t in enumerate(lists[0]):
        if t == pkg.tiles.PAD:
            continue
        x0, y0 = (int(t) % tx) * 64, (int(t) // tx) * 4
        for ly in range(4):
            y = y0 + ly
            if y >= H:
                continue
            xs = slice(x0, min(x0 + 64, W))
            n = xs.stop - xs.start
            base = s * 256 + ly * 64
            assert np.array_equal(o8[base:base + n], r8[y, xs]), (s, ly)
            assert np.array_equal(on[base:base + n], rn[y, xs]), (s, ly)
            hit = rn[y, xs] >= 0
            assert float(np.max(np.abs(of[base:base + n][hit] - rf[y, xs][hit]), initial=0.0)) <= 1e-4


def test_layout_budget_and_both_axis_copies(pkg, orc, gpu, tune):
    """a zero budget makes no copy (oblique views on the x-row quad march, side views
    on the x rows), both axis copies stay resident when they fit, a lowered budget
    drops them, layout_info reports the copies and their build cost, and every
    frame stays bit-identical to the oracle"""
    import torch
    vol = orc.synth_volume(48, 40, 44, 8)
    tune.set("VR_SEG_RAYS", "0")  # small frame: the one-lane / quad marches that read copies
    pkg.init_distribution(vol)
    W, H = 88, 68
    rec = 48 * 40 * 44 * 8 * 4
    try:
        pkg.set_layout_budget(0)
        for rot in ((30.0, 45.0), (0.0, 90.0), (90.0, 90.0)):
            m = pkg.camera.display_inv_view(rot)
            got = gpu_render(pkg, None, W, H, m, 1, torch)
            assert "brick" not in pkg.last_kernel() and "rows" not in pkg.last_kernel(), (
                rot, pkg.last_kernel())
            assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3],
                          f"budget 0 {rot}")
        assert pkg.layout_info()["resident_bytes"] == 0
        pkg.set_layout_budget(None)
        builds0 = pkg.layout_info()["builds"]
        for rot, kern in (((0.0, 90.0), "zrows"), ((90.0, 90.0), "yrows"), ((0.0, 90.0), "zrows")):
            m = pkg.camera.display_inv_view(rot)
            got = gpu_render(pkg, None, W, H, m, 1, torch)
            assert kern in pkg.last_kernel(), pkg.last_kernel()
            assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3],
                          f"axis copy {rot}")
        info = pkg.layout_info()
        # y and z copies both resident; the third frame reused the z copy
        assert info["resident_bytes"] == 2 * rec and info["builds"] == builds0 + 2, info
        assert info["last_build_bytes"] == rec and info["last_build_ms"] > 0.0, info
        # a budget of one copy drops both; the next side view makes one again
        pkg.set_layout_budget(rec)
        assert pkg.layout_info()["resident_bytes"] == 0
        m = pkg.camera.display_inv_view((90.0, 90.0))
        gpu_render(pkg, None, W, H, m, 1, torch)
        assert "yrows" in pkg.last_kernel()
        m = pkg.camera.display_inv_view((0.0, 90.0))
        got = gpu_render(pkg, None, W, H, m, 1, torch)
        # the z copy replaced the y copy (room only after dropping it)
        assert "zrows" in pkg.last_kernel() and pkg.layout_info()["resident_bytes"] == rec
        assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3],
                      "budget of one copy")
    finally:
        pkg.set_layout_budget(None)


@pytest.mark.parametrize("nb", [1, 8])
def test_baked_axis_views_take_a_plane_copy(pkg, orc, gpu, tune, nb):
    """baked frames of views along z or y (side / top views) filter a copy of the
    method's plane with that axis in the brick rows (k_plane_axis, gather8 MODE 4 /
    5): full frames through the one-lane march, rank lists through the segmented
    ones, methods 1/2/3, bit-identical to the oracle; the copies count in
    layout_info and go with the planes (vr_release_stats)"""
    import torch
    vol = orc.synth_volume(52, 40, 47, nb)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    W, H = 120, 88
    tune.set("VR_SEG_RAYS", "0")  # this small frame on the one-lane march
    for rot, kern in (((0.0, 90.0), "plane_zrows"), ((90.0, 90.0), "plane_yrows"),
                      ((-8.0, -85.0), "plane_zrows")):
        m = pkg.camera.display_inv_view(rot)
        for method in (1, 2, 3):
            got = gpu_render(pkg, None, W, H, m, method, torch)
            assert kern in pkg.last_kernel(), (rot, pkg.last_kernel())
            ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
            assert_parity(got, ref, f"baked {rot} nb={nb} m{method}")
        # a 3-rank split (4-lane windows at this size)
        got, kernels = _split_frame(pkg, torch, W, H, m, 3, 1)
        assert all(kern in k for k in kernels), kernels
        ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=1), want_float=False,
                          want_steps=False)[0]
        assert np.array_equal(got, ref8), (rot, kernels)
    assert pkg.layout_info()["resident_bytes"] > 0
    pkg.release_stats()  # drops the planes with their copies (and the record copies)
    assert pkg.layout_info()["resident_bytes"] == 0
    got = gpu_render(pkg, None, W, H, pkg.camera.display_inv_view((0.0, 90.0)), 1, torch)
    assert "plane" not in pkg.last_kernel()


@pytest.mark.parametrize("seg", ["0", ""])
def test_baked_wide_planes_keep_plane_copies_on_their_modes(pkg, orc, gpu, tune, seg):
    """x-row planes too large for 32-bit indices march with method -1 (64-bit plane
    index); a plane's y- / z-rows copy must never go there (it is not an x-row
    plane): VR_PLANE_WIDE=1 forces the wide branch at a small size, and every view
    stays bit-identical to the oracle -- the row-aligned view on M=-1, the side and
    top views on their plane copies (M=0, MODE 4 / 5), full frames and rank lists"""
    import torch
    vol = orc.synth_volume(52, 40, 47, 4)
    pkg.init_distribution(vol)
    pkg.bake_stats()
    W, H = 120, 88
    if seg:
        tune.set("VR_SEG_RAYS", seg)
    tune.set("VR_PLANE_WIDE", "1")
    try:
        for rot, kern in ((None, "M=-1"), ((0.0, 90.0), "plane_zrows"),
                          ((90.0, 90.0), "plane_yrows")):
            m = (pkg.camera.single_test_inv_view() if rot is None
                 else pkg.camera.display_inv_view(rot))
            for method in (1, 3):
                got = gpu_render(pkg, None, W, H, m, method, torch)
                assert kern in pkg.last_kernel(), (rot, pkg.last_kernel())
                if rot is not None:
                    assert "M=0" in pkg.last_kernel(), pkg.last_kernel()
                ref = orc.render(vol, orc.make_params(W, H, m, query_method=method))[:3]
                assert_parity(got, ref, f"wide baked {rot} m{method}")
            got, kernels = _split_frame(pkg, torch, W, H, m, 3, 2)
            ref8 = orc.render(vol, orc.make_params(W, H, m, query_method=2), want_float=False,
                              want_steps=False)[0]
            assert np.array_equal(got, ref8), (rot, kernels)
    finally:
        pkg.release_stats()


@pytest.mark.parametrize("nb", [1, 2, 4, 8])
def test_axis_copy_tiles_pitched_and_ragged(pkg, orc, gpu, tune, nb):
    """the LDS-tiled axis copy (k_axis_copy, 32 x 32 record tiles): volumes whose x,
    y, z are not multiples of the tile, pitched rows / slices (VR_PAD), records of
    1-8 bins; side and top views through both copies bit-identical to the oracle"""
    import torch
    vol = orc.synth_volume(45, 33, 70, nb)
    W, H = 72, 56
    tune.set("VR_SEG_RAYS", "0")  # the one-lane march, which reads the copies
    for pad in ("", "3,77"):
        if pad:
            tune.set("VR_PAD", pad)
        for rot, kern in (((0.0, 90.0), "zrows"), ((90.0, 90.0), "yrows")):
            m = pkg.camera.display_inv_view(rot)
            got = gpu_render(pkg, vol, W, H, m, 1, torch)
            assert kern in pkg.last_kernel(), (pad, rot, pkg.last_kernel())
            assert_parity(got, orc.render(vol, orc.make_params(W, H, m, query_method=1))[:3],
                          f"nb={nb} pad={pad!r} {rot}")
