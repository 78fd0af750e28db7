"""The reference's input-file readers (vr_parse_codebook / vr_parse_templates) on
files written in its formats (tests/ref_files.py).  Host-only: no GPU needed."""
import ctypes
import os
import struct

import numpy as np
import pytest

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


def _flex_tables_for_files(orc):
    """synthetic tables whose values survive the files' float64 / int32 round trip
    and the loaders' checks (bin ids <= nbins, frequencies in [0, 1])"""
    return orc.synth_flex(12, 5, 16, ntemplates=6, seed=3)


def test_flex_files_round_trip(pkg, orc, tmp_path):
    """the flexible-block files parse back into the tables they were written from
    (C:709-997); fractal spans come from the span list through spanId"""
    import ref_files
    t = _flex_tables_for_files(orc)
    paths = ref_files.write_flex_files(str(tmp_path), t)
    got = pkg.parse_flex_files(*paths, dim=12, nbins=16)
    for k in ("fractal_low", "fractal_high", "fractal_code", "simple_low", "simple_high",
              "simple_count"):
        assert np.array_equal(got[k][:, :3] if got[k].ndim == 2 else got[k],
                              np.asarray(t[k])[:, :3] if np.asarray(t[k]).ndim == 2 else t[k]), k
    for k, n in (("fractal_err", t["fractal_code"][:, 3]), ("simple_hist", t["simple_count"])):
        for i, c in enumerate(n):
            assert np.array_equal(got[k][i, :c], np.asarray(t[k])[i, :c]), (k, i)
            assert not got[k][i, c:].any()
    assert np.array_equal(got["templates"], np.asarray(t["templates"], np.float32))
    # parsed tables give the same pre-pass (oracle) as the originals: unused pairs differ only
    tt = dict(got, block=5)
    assert np.array_equal(orc.flex_process(tt), orc.flex_process(t))


def test_flex_file_rejections(pkg, orc, tmp_path):
    import struct
    import ref_files
    t = _flex_tables_for_files(orc)
    paths = ref_files.write_flex_files(str(tmp_path), t)
    L = pkg._lib.load()
    # a span with low > high fails checkSpanLimit (C:693-699)
    bad = tmp_path / "badspan.bin"
    bad.write_bytes(struct.pack("<i6i", 1, 5, 4, 1, 1, 1, 1))
    assert L.vr_parse_span_list(str(bad).encode(), 0, None, None) == -2
    # truncated
    bad.write_bytes(struct.pack("<i5i", 1, 1, 1, 1, 1, 1))
    assert L.vr_parse_span_list(str(bad).encode(), 0, None, None) == -1
    # fractal entry with NE > nbins is rejected (C:816-819)
    sp = paths[0].encode()
    bad.write_bytes(struct.pack("<ii", 1, 1) + struct.pack("<iiiBi", 0, 0, 0, 0, 17))
    n = L.vr_parse_span_list(sp, 0, None, None)
    sl = np.zeros((n, 4), np.int32)
    assert L.vr_parse_fractal_histogram(str(bad).encode(), sl.ctypes.data, sl.ctypes.data, n, 16,
                                        0, None, None, None, None) == -2
    # spanId past the span list
    bad.write_bytes(struct.pack("<ii", 1, 1) + struct.pack("<iiiBi", 1, 0, 0, 0, 0))
    assert L.vr_parse_fractal_histogram(str(bad).encode(), sl.ctypes.data, sl.ctypes.data, 1, 16,
                                        0, None, None, None, None) == -3
    # simple frequency > 1 (checkHistogram, C:701-707)
    c, i, f = (tmp_path / n for n in ("c.bin", "i.bin", "f.bin"))
    c.write_bytes(struct.pack("<i7i", 1, 0, 0, 0, 0, 0, 0, 1))
    i.write_bytes(struct.pack("<i", 3))
    f.write_bytes(struct.pack("<d", 1.5))
    assert L.vr_parse_simple_histogram(str(c).encode(), str(i).encode(), str(f).encode(), 16, 0,
                                       None, None, None, None) == -2
    # the one-call loader reports a missing file without touching the device
    with pytest.raises(pkg.VRError):
        pkg.load_flex_files(str(tmp_path / "nope.bin"), *paths[1:], dim=12, nbins=16)
