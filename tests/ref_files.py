"""Writers for the reference's on-disk input formats (test fixtures only).

Layouts as the reference's loaders read them: loadRawFile (C:538-555),
loadCodebook (C:558-642), loadTemplates (C:645-675).
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
