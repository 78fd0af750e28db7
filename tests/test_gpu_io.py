"""The reference's own input files through the library, and the headless
runSingleTest tool (vr_single_test) -- on the GPU."""
import os
import subprocess

import numpy as np
import pytest

import ref_files as F

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "volume-rendering-based-on-distribution-data_amd", "csrc", "build",
                    "vr_single_test")
C0 = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 4]


def _files(orc, tmp_path, nx=20, ny=18, nz=10, nb=32):
    vol = orc.synth_volume(nx, ny, nz, nb)
    cb, t, e = orc.synth_codec(nx, ny, nz, nb, ntemplates=30, seed=4)
    paths = {k: str(tmp_path / f"{k}.bin") for k in ("hist", "codebook", "templates")}
    F.write_histograms(paths["hist"], vol)
    F.write_codebook(paths["codebook"], cb, e)
    F.write_templates(paths["templates"], t)
    # what the loaders make of them: errors in float, unused pairs zero
    e2 = np.zeros_like(e)
    ne = cb[..., 3]
    for j in range(e.shape[-2]):
        e2[..., j, :] = np.where((j < ne)[..., None], e[..., j, :], 0)
    return vol, cb, t, e2, paths


def test_reference_files_render(pkg, orc, gpu, tmp_path):
    import torch
    vol, cb, t, e, p = _files(orc, tmp_path)
    L = pkg._lib.load()
    ext = pkg._lib.Extent(20, 18, 10)
    assert L.vr_load_reference_files(p["hist"].encode(), p["codebook"].encode(),
                                     p["templates"].encode(), ext, 32) == 0, L.vr_last_error()
    W, H = 96, 80
    out = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for method in (1, 3, 4, 6):
        out.zero_()
        pkg.render(pkg.make_desc(out, W, H, C0, query_method=method, volume_size=(20, 18, 10)))
        torch.cuda.synchronize()
        params = orc.make_params(W, H, C0, query_method=method)
        ref = (orc.render_codec(cb, t, e, params) if method >= 4 else orc.render(vol, params))[0]
        assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(H, W), ref), method


def _ppm(path):
    with open(path, "rb") as f:
        data = f.read()
    head = data.split(b"\n", 3)
    assert head[0] == b"P6"
    w, h = (int(v) for v in head[1].split())
    return np.frombuffer(head[3], np.uint8).reshape(h, w, 3)


def _rgb(rgba8):
    return np.stack([(rgba8 >> s) & 0xFF for s in (0, 8, 16)], -1).astype(np.uint8)


def test_single_test_tool(pkg, orc, gpu, tmp_path):
    """mirrors runSingleTest: throughput line, volume.ppm, sdkComparePPM-style check"""
    vol, cb, t, e, p = _files(orc, tmp_path)
    out = str(tmp_path / "volume.ppm")
    ref = str(tmp_path / "ref_volume.ppm")
    W = H = 128
    for method in (1, 4):
        img = (orc.render_codec(cb, t, e, orc.make_params(W, H, C0, query_method=method))
               if method == 4 else orc.render(vol, orc.make_params(W, H, C0, query_method=method)))[0]
        with open(ref, "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (W, H))
            f.write(_rgb(img).tobytes())
        cmd = [TOOL, f"--file={p['hist']}", f"--codebook={p['codebook']}",
               f"--templates={p['templates']}", "--xsize=20", "--ysize=18", "--zsize=10",
               "--bins=32", f"--method={method}", f"--width={W}", f"--height={H}", "--iters=3",
               f"--out={out}", f"--ref={ref}"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "volumeRender, Throughput = " in r.stdout and "PASSED" in r.stdout
        assert np.array_equal(_ppm(out), _rgb(img))
    # a reference image that differs in every byte by more than 5 fails
    with open(ref, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (W, H))
        f.write(((_rgb(img).astype(np.int32) + 100) % 256).astype(np.uint8).tobytes())
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "FAILED" in r.stdout
    # synthetic mode needs no files
    r = subprocess.run([TOOL, "--synthetic", "--xsize=32", "--ysize=32", "--zsize=32", "--bins=8",
                        "--width=64", "--height=64", f"--out={out}"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_flex_files_render(pkg, orc, gpu, tmp_path):
    """the six flexible-block files -> vr_load_flex_files -> dataProcessing (6-voxel
    blocks) -> methods 8/9/0 equal the oracle on the same tables"""
    import torch
    t = orc.synth_flex(20, 6, 32, ntemplates=8, seed=9)
    paths = F.write_flex_files(str(tmp_path), t)
    pkg.load_flex_files(*paths, dim=20, nbins=32)
    pkg.dataProcessing()
    blocks = orc.flex_process(t)
    m = pkg.camera.display_inv_view((30.0, 45.0))
    for method, ts in ((8, 1.0), (9, 1 / 255), (0, 1 / 4000)):
        out = torch.zeros(40 * 48, dtype=torch.int32, device="cuda")
        pkg.render(pkg.make_desc(out, 48, 40, m, density=0.3, transfer_scale=ts,
                                 query_method=method))
        torch.cuda.synchronize()
        ref = orc.render_flex(blocks, orc.make_params(48, 40, m, density=0.3, transfer_scale=ts,
                                                      query_method=method))[0]
        assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(40, 48), ref)
    pkg.freeCudaBuffers()
