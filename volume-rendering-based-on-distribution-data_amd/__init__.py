"""vrdd_amd -- MI355X (gfx950) ray caster for distribution volumes.

A drop-in for the d_render path of ykou/Volume-Rendering-Based-on-Distribution-Data:
the per-ray march is a hand-written HIP kernel in csrc/ behind the reference's
C entry points (include/vr.h); this package is the thin host-side mirror of the
reference's volumeRender.cpp API plus the multi-GPU tile split.

The directory name is not a Python identifier; load it with
``_load_package()`` of __graft_entry__.py (module name ``vrdd_amd``).
"""
from . import _lib, api, camera, slabs, stream, tiles  # noqa: F401
from ._lib import VRError  # noqa: F401
from .api import *  # noqa: F401,F403

LIB_PATH = _lib.LIB_PATH
