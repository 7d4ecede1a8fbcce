"""Batched-frames front-end: extract + stereo-match many device-resident stereo pairs per enqueue.

This is the throughput path of BASELINE.json (stereo pairs/s): images (2P, H, W) uint8 already in HBM
(a torch tensor on the GPU), pair p = images (2p, 2p+1) = (left, right).  One call enqueues the whole
pipeline (7 resize launches, detect, octree, describe, stereo) on the given HIP stream; results stay on
the device until fetched.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KP_DTYPE, BatchView, call, ptr

KITTI_BF = 386.1448  # KITTI00-02.yaml Camera.bf
KITTI_FX = 718.856   # KITTI00-02.yaml Camera.fx
# EuRoC MAV rectified stereo (ORB-SLAM2 EuRoC.yaml Camera.bf, Camera.fx; the reference ships KITTI settings
# only), the EuRoC case of tests/test_gpu_stereo.py
EUROC_BF = 47.90639384423901
EUROC_FX = 435.2046959714599


def camera_constants(width: int, height: int) -> tuple[float, float]:
    """(bf, fx) of the camera whose image size this is: EuRoC for 752x480, KITTI otherwise."""
    return (EUROC_BF, EUROC_FX) if (int(width), int(height)) == (752, 480) else (KITTI_BF, KITTI_FX)


class StereoFrontEnd:
    def __init__(self, width: int = 1241, height: int = 376, max_pairs: int = 64, nfeatures: int = 2000,
                 scaleFactor: float = 1.2, nlevels: int = 8, iniThFAST: int = 20, minThFAST: int = 7,
                 resize_simd_lanes: int = 16, lanes: int = 4, graphs: bool = False):
        self.width, self.height, self.max_pairs = int(width), int(height), int(max_pairs)
        self._params = _lib.make_params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, resize_simd_lanes)
        h = C.c_void_p()
        call("orbfe_create", C.byref(self._params), C.byref(h))
        self._h = h
        call("orbfe_batch_reserve", h, self.width, self.height, 2 * self.max_pairs)
        # concurrent chunks of enqueue() on internal streams (results are independent of it)
        call("orbfe_set_lanes", h, int(lanes))
        # graphs=True: one-lane enqueues replay a captured HIP graph (orbfe_set_graphs ORBFE_GRAPH_BATCH; off by
        # default: graph launches on several streams serialise the handles' chains; results do not depend on it)
        if _lib.has("orbfe_set_graphs"):
            call("orbfe_set_graphs", h, 3 if graphs else 1)
        v = BatchView()
        call("orbfe_batch_view_get", h, C.byref(v))
        self.kp_cap = v.kp_cap
        self.scales = np.zeros(int(nlevels), np.float32)  # the level scale factors (compact records)
        call("orbfe_get_scales", h, self.scales.ctypes.data_as(C.c_void_p), None, None, None, None)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib.lib().orbfe_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def enqueue(self, images, n_pairs: int | None = None, bf: float = KITTI_BF, fx: float = KITTI_FX,
                stream_ptr: int = 0) -> None:
        """images: device tensor (>= 2*n_pairs, H, W) uint8, C-contiguous.  stream_ptr: raw hipStream_t
        (torch.cuda.current_stream().cuda_stream), 0 = the null stream."""
        n_pairs = images.shape[0] // 2 if n_pairs is None else int(n_pairs)
        if images.dtype.itemsize != 1 or tuple(images.shape[1:]) != (self.height, self.width):
            raise ValueError("images must be (2P, H, W) uint8 with the reserved H, W")
        if not images.is_contiguous() or not images.is_cuda:
            raise ValueError("images must be a contiguous GPU tensor")
        if n_pairs > self.max_pairs or 2 * n_pairs > images.shape[0]:
            raise ValueError("n_pairs exceeds the reservation or the tensor")
        call("orbfe_frontend_batch_device", self._h, C.c_void_p(images.data_ptr()), self.width * self.height,
             n_pairs, float(bf), float(np.float32(fx)), C.c_void_p(stream_ptr))

    def enqueue_extract(self, images, n_images: int | None = None, stream_ptr: int = 0) -> None:
        n = images.shape[0] if n_images is None else int(n_images)
        call("orbfe_extract_batch_device", self._h, C.c_void_p(images.data_ptr()), self.width * self.height, n,
             C.c_void_p(stream_ptr))

    def graph_stats(self) -> dict:
        """HIP-graph captures and launches of this handle so far, and the graphs cached now."""
        cap, lau, n = C.c_int64(), C.c_int64(), C.c_int32()
        if not _lib.has("orbfe_graph_stats"):
            return {"captures": 0, "launches": 0, "cached": 0}
        call("orbfe_graph_stats", self._h, C.byref(cap), C.byref(lau), C.byref(n))
        return {"captures": cap.value, "launches": lau.value, "cached": n.value}

    def overflow(self) -> int:
        """Overflow word of the last batch (0 = no on-device capacity bound was hit); synchronises."""
        v = C.c_int32()
        call("orbfe_batch_status", self._h, C.byref(v))
        return v.value

    def fetch_image(self, i: int) -> tuple[np.ndarray, np.ndarray]:
        kps = np.empty(self.kp_cap, KP_DTYPE)
        desc = np.empty((self.kp_cap, 32), np.uint8)
        n = C.c_int32()
        call("orbfe_batch_fetch", self._h, int(i), ptr(kps), ptr(desc), self.kp_cap, C.byref(n))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def fetch_stereo(self, p: int) -> dict:
        u = np.empty(self.kp_cap, np.float32)
        d = np.empty(self.kp_cap, np.float32)
        st = np.empty(self.kp_cap, np.int8)
        m = np.empty(self.kp_cap, np.int32)
        n = C.c_int32()
        call("orbfe_batch_fetch_stereo", self._h, int(p), ptr(u), ptr(d), ptr(st), ptr(m), self.kp_cap, C.byref(n))
        k = n.value
        return dict(u_right=u[:k].copy(), depth=d[:k].copy(), status=st[:k].copy(), match_r=m[:k].copy())
