"""The reference's camera conventions, as the 12-float matrix copyInvViewMatrix takes.

Both reference hosts build an OpenGL column-major modelView and transpose its
first three rows into ``invViewMatrix`` (C:235-246 and C:1032-1043).  d_render
then uses it as the camera-to-volume transform: ray origin = column 3, ray
direction = upper 3x3 times normalize(u, v, -2) (K:293-296).
"""
from __future__ import annotations

import math

import numpy as np


def _rows_from_gl(model_view_colmajor: np.ndarray) -> np.ndarray:
    m = np.asarray(model_view_colmajor, dtype=np.float32).reshape(16)
    # C:235-246: invViewMatrix[4r + c] = modelView[4c + r] for r < 3
    return np.array([m[0], m[4], m[8], m[12], m[1], m[5], m[9], m[13],
                     m[2], m[6], m[10], m[14]], dtype=np.float32)


def single_test_inv_view() -> np.ndarray:
    """Camera C0: the fixed view of runSingleTest (C:1024-1043), eye at (0,0,4)."""
    mv = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 4, 1], dtype=np.float32)
    return _rows_from_gl(mv)


def _rot(angle_deg: float, axis: str) -> np.ndarray:
    a = math.radians(angle_deg)
    c, s = math.cos(a), math.sin(a)
    r = np.eye(4)
    if axis == "x":
        r[1, 1], r[1, 2], r[2, 1], r[2, 2] = c, -s, s, c
    else:  # y
        r[0, 0], r[0, 2], r[2, 0], r[2, 2] = c, s, -s, c
    return r


def display_inv_view(rotation=(30.0, 45.0), translation=(0.0, 0.0, -4.0)) -> np.ndarray:
    """Camera of display() (C:225-246): glRotatef(-rx,x) glRotatef(-ry,y) glTranslatef(-t).

    Computed in float64 and rounded to float32 (the GL driver's own rounding is
    not reproducible; the matrix is an input, so only its 12 floats matter).
    """
    rx, ry = rotation
    t = np.eye(4)
    t[0, 3], t[1, 3], t[2, 3] = -translation[0], -translation[1], -translation[2]
    m = _rot(-rx, "x") @ _rot(-ry, "y") @ t
    return m[:3, :].astype(np.float32).reshape(12)


C0 = single_test_inv_view
C1 = display_inv_view
