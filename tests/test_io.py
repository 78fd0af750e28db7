"""The reference's input-file readers (vr_parse_codebook / vr_parse_templates) on
files written in its formats (tests/ref_files.py).  Host-only: no GPU needed."""
import ctypes
import os
import struct

import numpy as np

import ref_files as F


def _parse_codebook(L, path, nb, n):
    cb = np.zeros((n, 4), np.int32)
    er = np.zeros((n, nb, 2), np.float32)
    got = L.vr_parse_codebook(str(path).encode(), nb, n, cb.ctypes.data, er.ctypes.data)
    return got, cb, er


def test_codebook_round_trip(pkg, orc, tmp_path):
    L = pkg._lib.load()
    cb, t, e = orc.synth_codec(5, 4, 3, 8, seed=11)
    path = tmp_path / "codebook.bin"
    F.write_codebook(path, cb, e)
    got, gcb, ger = _parse_codebook(L, path, 8, 60)
    assert got == 60
    assert np.array_equal(gcb, cb.reshape(-1, 4))
    ne = cb.reshape(-1, 4)[:, 3]
    for i in range(60):  # used pairs as written (doubles rounded to float), the rest zero
        k = ne[i]
        assert np.array_equal(ger[i, :k], e.reshape(60, 8, 2)[i, :k].astype(np.float64).astype(np.float32))
        assert not ger[i, k:].any()


def test_templates_round_trip(pkg, orc, tmp_path):
    L = pkg._lib.load()
    _, t, _ = orc.synth_codec(2, 2, 2, 32, ntemplates=7)
    path = tmp_path / "templates.bin"
    F.write_templates(path, t)
    out = np.zeros_like(t)
    assert L.vr_parse_templates(str(path).encode(), 32, 7, out.ctypes.data) == 7
    assert np.array_equal(out, t)


def test_codebook_rejections(pkg, tmp_path):
    L = pkg._lib.load()
    path = tmp_path / "bad.bin"
    with open(path, "wb") as f:  # one block with NE = 9 > 8 bins: the loader refuses (C:611-614)
        f.write(struct.pack("<iiiiiBi", 1, 1, 0, 0, 0, 0, 9))
    assert L.vr_parse_codebook(str(path).encode(), 8, 1, None, None) == -2
    with open(path, "wb") as f:  # truncated: 2 blocks announced, 1 present
        f.write(struct.pack("<iiiiiBi", 1, 2, 0, 0, 0, 0, 0))
    assert L.vr_parse_codebook(str(path).encode(), 8, 2, None, None) == -1
    assert L.vr_parse_codebook(str(tmp_path / "missing.bin").encode(), 8, 1, None, None) == -1
    assert L.vr_parse_templates(str(tmp_path / "missing.bin").encode(), 8, 1, None) == -1
