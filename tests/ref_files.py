"""Writers for the reference's on-disk input formats (test fixtures only).

Layouts as the reference's loaders read them: loadRawFile (C:538-555),
loadCodebook (C:558-642), loadTemplates (C:645-675), and the flexible-block
files: loadSpanList (C:709-771), loadFractalHistogram (C:773-875),
loadSimpleHistogram (C:877-949), loadFlexibleTemplates (C:951-997).
"""
import struct

import numpy as np


def write_histograms(path, vol):
    """raw fp32, nBlocks x nBins, block = x + X*(y + Y*z)"""
    np.ascontiguousarray(vol, dtype=np.float32).tofile(path)


def write_codebook(path, codebook, errors, nsteps=1):
    """codebook int (..., 4) = (template id, shift, flip, NE); errors (..., slots, 2)"""
    cb = np.asarray(codebook).reshape(-1, 4)
    er = np.asarray(errors).reshape(cb.shape[0], -1, 2)
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", nsteps, cb.shape[0]))
        for i, (tid, shift, flip, ne) in enumerate(cb):
            f.write(struct.pack("<iiiBi", i, int(tid), int(shift), int(flip != 0), int(ne)))
            f.write(np.asarray(er[i, :ne, 0], dtype="<i4").tobytes())
            f.write(np.asarray(er[i, :ne, 1], dtype="<f8").tobytes())


def write_templates(path, templates):
    t = np.asarray(templates, dtype=np.float64)
    with open(path, "wb") as f:
        f.write(struct.pack("<i", t.shape[0]))
        for row in t:
            f.write(np.zeros(6, "<f8").tobytes())  # the 6 limits the loader skips
            f.write(row.astype("<f8").tobytes())


def write_flex_files(d, t):
    """span tables (oracle.synth_flex layout) -> the six files of C:79-84 in
    directory d; the span list holds the fractal spans, spanId = entry index.
    Returns the paths in vr_load_flex_files order."""
    import os
    p = [os.path.join(d, n) for n in ("spanList.bin", "codebook0.bin", "nzbCounts0.bin",
                                       "nzbBinIds0.bin", "nzbFreqs0.bin", "domainList.bin")]
    fl, fh = np.asarray(t["fractal_low"]), np.asarray(t["fractal_high"])
    with open(p[0], "wb") as f:  # lowX, highX, lowY, highY, lowZ, highZ (C:728-733)
        f.write(struct.pack("<i", fl.shape[0]))
        for lo, hi in zip(fl, fh):
            f.write(struct.pack("<6i", lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]))
    code, err = np.asarray(t["fractal_code"]), np.asarray(t["fractal_err"])
    with open(p[1], "wb") as f:
        f.write(struct.pack("<ii", 1, code.shape[0]))
        for i, (tid, shift, flip, ne) in enumerate(code):
            f.write(struct.pack("<iiiBi", i, int(tid), int(shift), int(flip != 0), int(ne)))
            f.write(np.asarray(err[i, :ne, 0], dtype="<i4").tobytes())
            f.write(np.asarray(err[i, :ne, 1], dtype="<f8").tobytes())
    sl, sh = np.asarray(t["simple_low"]), np.asarray(t["simple_high"])
    cnt, hist = np.asarray(t["simple_count"]), np.asarray(t["simple_hist"])
    with open(p[2], "wb") as fc, open(p[3], "wb") as fi, open(p[4], "wb") as ff:
        fc.write(struct.pack("<i", sl.shape[0]))
        for i in range(sl.shape[0]):
            fc.write(struct.pack("<7i", *sl[i, :3], *sh[i, :3], int(cnt[i])))
            fi.write(np.asarray(hist[i, :cnt[i], 0], dtype="<i4").tobytes())
            ff.write(np.asarray(hist[i, :cnt[i], 1], dtype="<f8").tobytes())
    write_templates(p[5], t["templates"])
    return p
