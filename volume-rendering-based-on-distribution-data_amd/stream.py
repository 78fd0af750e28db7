"""Out-of-core GMM frames on one GPU: host-pinned z-slabs streamed through HBM.

BASELINE config 5 names "host-pinned brick streaming (out-of-core)".  On a full
8-GPU node the 2048^3 x 16 volume is resident across the GPUs as z-slabs
(slabs.py); with fewer GPUs than that -- or a volume larger
than the node's HBM -- the records stay in pinned host memory and each GPU
streams them slab by slab.  The march is the slab chain of slabs.py on a single
device: every ray crosses the slabs in the same order (march_direction), so a
frame is slab 0 with the camera rays, then slab 1 with the rays slab 0 handed
on as exact 48-byte states, and so on -- bit-identical to the whole-volume
render (the same float operations in the same order).

Two HBM slab buffers form a ring: while slab i is marched on the render
stream, slab i+1's records are copied host -> device on a copy stream into
the other buffer (which slab i-1's march has released).  A frame therefore
costs max(PCIe copy, march) per slab plus the first copy; the planes the
method reads cross PCIe once per frame (method 1: the (w, mu) plane only).  The host waits once per slab for the alive count
(it sizes the next launch).

This module is host logic over the C-ABI (vr_init_gmm adopting the slab
buffer, vr_render_gmm with a vr_gmm_slab); no device code.
"""
from __future__ import annotations

from typing import List, Tuple

from . import api, slabs
from ._lib import GMM_RAY_BYTES


def stream_bounds(nz: int, slab_slices: int, direction: int) -> List[Tuple[int, int]]:
    """Slabs of `slab_slices` slices (the last one thinner) covering [0, nz), in
    march order."""
    if slab_slices < 1:
        raise ValueError("slab_slices must be >= 1")
    if direction == 0:
        raise ValueError("rays of this view cross z-slabs in both directions")
    b = [(z, min(z + slab_slices, nz)) for z in range(0, nz, slab_slices)]
    return b if direction > 0 else b[::-1]


class GmmStream:
    """Render frames of a GMM volume held in (pinned) host memory.

    wm_host: float32 (nz, ny, nx, K, 2) (w, mu) pairs, sg_host: (nz, ny, nx, K),
    torch CPU tensors (pinned for asynchronous copies; pinned here when not).
    slab_slices: slices per streamed slab (each HBM buffer holds one more, the
    halo slice the footprints of the slab's last samples read)."""

    def __init__(self, wm_host, sg_host, slab_slices: int, device=None):
        import torch
        if tuple(sg_host.shape) != tuple(wm_host.shape[:4]) or wm_host.shape[4] != 2:
            raise ValueError("wm_host must be (nz, ny, nx, K, 2) and sg_host (nz, ny, nx, K)")
        if wm_host.dtype != torch.float32 or sg_host.dtype != torch.float32:
            raise ValueError("GMM planes are float32")
        self.torch = torch
        self.wm = wm_host if wm_host.is_pinned() else wm_host.pin_memory()
        self.sg = sg_host if sg_host.is_pinned() else sg_host.pin_memory()
        nz, ny, nx, K = (int(v) for v in sg_host.shape)
        self.dims, self.K = (nx, ny, nz), K
        self.S = min(int(slab_slices), nz)
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        cap = min(self.S + 1, nz)
        self.dwm = [torch.empty((cap, ny, nx, K, 2), dtype=torch.float32, device=dev)
                    for _ in range(2)]
        self.dsg = [torch.empty((cap, ny, nx, K), dtype=torch.float32, device=dev)
                    for _ in range(2)]
        self.copy = torch.cuda.Stream(device=dev)
        self.dev = dev
        self.rays = None
        self.cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.slab_bytes = (ny * nx * K * 12) * cap

    def _issue_copy(self, b: int, zb: int, ns: int, free_event, sigma: bool) -> object:
        torch = self.torch
        with torch.cuda.stream(self.copy):
            if free_event is not None:
                self.copy.wait_event(free_event)  # the march that last read buffer b
            self.dwm[b][:ns].copy_(self.wm[zb:zb + ns], non_blocking=True)
            if sigma:
                self.dsg[b][:ns].copy_(self.sg[zb:zb + ns], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        return ev

    def render(self, desc, stream) -> dict:
        """One frame into desc's output (the caller zeroes it, C:208), marched on
        `stream` (also made the library's stream).  Returns per-frame counters."""
        torch = self.torch
        W, H = int(desc.width), int(desc.height)
        direction = slabs.march_direction(list(desc.inv_view), W, H)
        bounds = stream_bounds(self.dims[2], self.S, direction)
        if self.rays is None or self.rays[0].shape[0] < W * H:
            self.rays = [torch.empty((W * H, GMM_RAY_BYTES // 4), dtype=torch.int32,
                                     device=self.dev) for _ in range(2)]
        api.set_stream(stream)
        # work the caller queued on its current stream (zeroing the frame, C:208)
        # comes first; the copy stream starts after it too
        stream.wait_stream(torch.cuda.current_stream())
        self.copy.wait_stream(torch.cuda.current_stream())
        nz = self.dims[2]
        res = [slabs.resident_slices(lo, hi, nz) for lo, hi in bounds]
        # the mean (method 1) reads only the (w, mu) plane: sigma stays on the host
        sigma = int(desc.query_method) != 1
        free = [None, None]
        copied = [None, None]
        copied[0] = self._issue_copy(0, res[0][0], res[0][1], None, sigma)
        n_in, handed = 0, 0
        for i, (lo, hi) in enumerate(bounds):
            b = i % 2
            zb, ns = res[i]
            stream.wait_event(copied[b])
            api.init_gmm(self.dwm[b][:ns], self.dsg[b][:ns], self.dims, z_base=zb, adopt=True)
            rin, rout = self.rays[(i + 1) % 2], self.rays[i % 2]
            with torch.cuda.stream(stream):
                api.render_gmm(desc, api.gmm_slab(lo, hi, rout, self.cnt,
                                                  d_rays_in=rin if i else None,
                                                  n_rays_in=n_in if i else 0))
                done = torch.cuda.Event()
                done.record(stream)
            free[b] = done
            if i + 1 < len(bounds):  # the next slab's copy overlaps this march
                nb = (i + 1) % 2
                copied[nb] = self._issue_copy(nb, res[i + 1][0], res[i + 1][1], free[nb], sigma)
            with torch.cuda.stream(stream):  # read on the march's stream, after it
                n_in = int(self.cnt.item())  # sizes the next launch
            handed += n_in
        api.free_gmm()  # the library held an adopted view of a ring buffer
        if n_in != 0:
            raise RuntimeError("the last slab must end every ray")
        per_voxel = self.K * (12 if sigma else 8)
        return {"slabs": len(bounds), "rays_handed_on": handed,
                "bytes_streamed": sum(ns for _, ns in res) * self.dims[0] * self.dims[1] * per_voxel}
