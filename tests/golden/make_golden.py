#!/usr/bin/env python3
"""Generate the committed golden fixtures from the CPU oracle.

Each fixture holds the scene description (volume dims/bins/seed + a checksum of
the generated volume, camera matrix, render parameters) and the expected
outputs: packed RGBA8, samples per pixel and, for the small images, the float
RGBA.  The reference itself ships no golden image, so these pin
the oracle's restatement (cross-checked against tests/ref_numpy.py and the
analytic KATs in tests/test_oracle.py) against accidental drift, and the GPU
tests compare the HIP kernel with them too.

  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import __graft_entry__ as graft  # noqa: E402

SEED = 20261015


def scenes(cam):
    c0, c1 = cam.single_test_inv_view(), cam.display_inv_view((30.0, 45.0))
    out = []
    for method in (1, 2, 3, 7):
        out.append((f"vol16x4_c0_m{method}", (16, 16, 16, 4), (64, 64), c0, method, True))
        out.append((f"vol16x4_c1_m{method}", (16, 16, 16, 4), (64, 64), c1, method, True))
        # the reference's own data shape: Isabel 50x50x10 blocks x 32 bins (C:86-87)
        out.append((f"isabel50x50x10x32_c0_m{method}", (50, 50, 10, 32), (128, 128), c0,
                    method, False))
    out.append(("vol24x20x16x8_c1_m1_256x160", (24, 20, 16, 8), (256, 160), c1, 1, False))
    out.append(("vol32x1_c0_m1", (32, 32, 32, 1), (64, 64), c0, 1, True))
    return out


def codec_scenes(cam):
    c0, c1 = cam.single_test_inv_view(), cam.display_inv_view((30.0, 45.0))
    return [(f"codec12x10x9x8_{c}_m{m}", (12, 10, 9, 8), (48, 40), mat, m)
            for c, mat in (("c0", c0), ("c1", c1)) for m in (4, 5, 6)]


def main_codec(orc, cam):
    """methods 4/5/6: the codec inputs are stored in the fixture itself"""
    for name, (nx, ny, nz, nb), (W, H), m, method in codec_scenes(cam):
        cb, t, e = orc.synth_codec(nx, ny, nz, nb, seed=SEED)
        p = orc.make_params(W, H, m, query_method=method)
        out, f, n, _ = orc.render_codec(cb, t, e, p)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), codebook=cb, templates=t, errors=e,
            image=np.array([W, H]), inv_view=np.asarray(m, np.float32), density=np.float32(0.05),
            brightness=np.float32(1.0), toff=np.float32(0.0), tscale=np.float32(1.0),
            method=np.int32(method), rgba8=out, steps=n.astype(np.int16), rgba_f=f)
        print(name, "hit", int(np.sum(n >= 0)), "samples", int(np.sum(n[n > 0])))


FLEX_TSCALE = {9: 1.0 / 255.0, 0: 1.0 / 4000.0, 8: 1.0}  # mean ~[0,255], variance, entropy


def flex_scenes(cam):
    c0, c1 = cam.single_test_inv_view(), cam.display_inv_view((30.0, 45.0))
    return [(f"flex20b6x16_{c}_m{m}", (20, 6, 16), (48, 40), mat, m)
            for c, mat in (("c0", c0), ("c1", c1)) for m in (8, 9, 0)]


def main_flex(orc, cam):
    """methods 8/9/0: the span tables are stored in the fixture, with the block
    statistics of the pre-pass"""
    for name, (dim, block, nb), (W, H), m, method in flex_scenes(cam):
        t = orc.synth_flex(dim, block, nb, seed=SEED)
        blocks = orc.flex_process(t)
        p = orc.make_params(W, H, m, density=0.2, transfer_scale=FLEX_TSCALE[method],
                            query_method=method)
        out, f, n, _ = orc.render_flex(blocks, p)
        arrays = {k: t[k] for k in orc.FLEX_KEYS}
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), flex_dims=np.array([dim, block, nb]), blocks=blocks,
            image=np.array([W, H]), inv_view=np.asarray(m, np.float32), density=np.float32(0.2),
            brightness=np.float32(1.0), toff=np.float32(0.0),
            tscale=np.float32(FLEX_TSCALE[method]), method=np.int32(method), rgba8=out,
            steps=n.astype(np.int16), rgba_f=f, **arrays)
        print(name, "hit", int(np.sum(n >= 0)), "samples", int(np.sum(n[n > 0])))


def gmm_scenes(cam):
    c0, c1 = cam.single_test_inv_view(), cam.display_inv_view((30.0, 45.0))
    return [(f"gmm14x12x10x16_{c}_m{m}", (14, 12, 10, 16), (48, 40), mat, m)
            for c, mat in (("c0", c0), ("c1", c1)) for m in (1, 2)]


def main_gmm(orc, cam):
    """GMM volumes (config 5 record type): the mixture planes are
    regenerated from the seed; their checksums pin the generator"""
    for name, (nx, ny, nz, K), (W, H), m, method in gmm_scenes(cam):
        wm, sg = orc.synth_gmm(nx, ny, nz, K, SEED)
        p = orc.make_params(W, H, m, density=0.3, query_method=method)
        r = orc.render_gmm(wm, sg, (nx, ny, nz), p)
        n = r["out_n"]
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), gmm_dims=np.array([nx, ny, nz, K]),
            seed=np.uint64(SEED),
            wm_crc=np.uint32(np.bitwise_xor.reduce(wm.view(np.uint32).ravel())),
            sg_crc=np.uint32(np.bitwise_xor.reduce(sg.view(np.uint32).ravel())),
            image=np.array([W, H]), inv_view=np.asarray(m, np.float32), density=np.float32(0.3),
            brightness=np.float32(1.0), toff=np.float32(0.0), tscale=np.float32(1.0),
            method=np.int32(method), rgba8=r["out"], steps=n.astype(np.int16), rgba_f=r["out_f"])
        print(name, "hit", int(np.sum(n >= 0)), "samples", int(np.sum(n[n > 0])))


def main():
    orc = graft.load_oracle()
    cam = graft.load_package().camera
    for name, (nx, ny, nz, nb), (W, H), m, method, keep_f in scenes(cam):
        vol = orc.synth_volume(nx, ny, nz, nb, SEED)
        p = orc.make_params(W, H, m, query_method=method, m7_dims=(nx, ny, nz))
        out, f, n, _ = orc.render(vol, p)
        arrays = dict(
            dims=np.array([nx, ny, nz, nb]), seed=np.uint64(SEED),
            vol_crc=np.uint32(np.bitwise_xor.reduce(vol.view(np.uint32).ravel())),
            image=np.array([W, H]), inv_view=np.asarray(m, np.float32),
            density=np.float32(0.05), brightness=np.float32(1.0), toff=np.float32(0.0),
            tscale=np.float32(1.0), method=np.int32(method),
            m7_dims=np.array([nx, ny, nz]), rgba8=out, steps=n.astype(np.int16))
        if keep_f:
            arrays["rgba_f"] = f
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        print(name, "hit", int(np.sum(n >= 0)), "samples", int(np.sum(n[n > 0])))
    main_codec(orc, cam)
    main_flex(orc, cam)
    main_gmm(orc, cam)


if __name__ == "__main__":
    if sys.argv[1:] == ["gmm"]:  # only the GMM fixtures
        main_gmm(graft.load_oracle(), graft.load_package().camera)
    else:
        main()
