"""Drop-in for the reference's pybind11 module `pyORBExtractor` (pyORBExtractor/orb_extractor.cpp:16-40).

    from pyorbslam_amd.pyORBExtractor import ORBextractor     # instead of `from pyORBExtractor import ...`

Same constructor (keyword names of orb_extractor.cpp:23), same getters and the same return types:
operator_kd(image) -> (list of (x, y, size, angle, response, octave) tuples, (N, 32) uint8 ndarray), and
GetImagePyramid() -> list of uint8 arrays reproducing the reference caster's stride-ignoring copy.
All pixel work runs in the gfx950 library (liborbfe.so); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KP_DTYPE, call, ptr


class ORBextractor:
    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 resize_simd_lanes: int = 16):
        self._params = _lib.make_params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, resize_simd_lanes)
        h = C.c_void_p()
        call("orbfe_create", C.byref(self._params), C.byref(h))
        self._h = h
        self._nlevels = int(nlevels)
        L = self._nlevels
        self._sf = np.zeros(L, np.float32)
        self._isf = np.zeros(L, np.float32)
        self._s2 = np.zeros(L, np.float32)
        self._is2 = np.zeros(L, np.float32)
        self._npl = np.zeros(L, np.int32)
        call("orbfe_get_scales", h, ptr(self._sf), ptr(self._isf), ptr(self._s2), ptr(self._is2), ptr(self._npl))
        self._kps = np.zeros(0, KP_DTYPE)
        self._desc = np.zeros((0, 32), np.uint8)
        self._extracted = False

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib.lib().orbfe_destroy(h)
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # ---- getters (ORBextractor.h:62-86) ------------------------------------------------------------
    def GetLevels(self) -> int:
        return self._nlevels

    def GetScaleFactor(self) -> float:
        return float(np.float32(self._params.scale_factor))

    def GetScaleFactors(self) -> list:
        return [float(v) for v in self._sf]

    def GetInverseScaleFactors(self) -> list:
        return [float(v) for v in self._isf]

    def GetScaleSigmaSquares(self) -> list:
        return [float(v) for v in self._s2]

    def GetInverseScaleSigmaSquares(self) -> list:
        return [float(v) for v in self._is2]

    def features_per_level(self) -> list:
        return [int(v) for v in self._npl]

    def GetImagePyramid(self, sheared: bool = True) -> list:
        """Pyramid of the last operator_kd call.  sheared=True (default) is what the reference returns
        (opencv_type_casters.h:232-239 ignores Mat::step); sheared=False gives the true levels."""
        if not self._extracted:
            return [np.zeros((0, 0), np.uint8) for _ in range(self._nlevels)]
        out = []
        for l in range(self._nlevels):
            w, h = C.c_int32(), C.c_int32()
            call("orbfe_pyramid", self._h, l, None, int(sheared), C.byref(w), C.byref(h))
            a = np.empty((h.value, w.value), np.uint8)
            call("orbfe_pyramid", self._h, l, ptr(a), int(sheared), C.byref(w), C.byref(h))
            out.append(a)
        return out

    # ---- operator_kd (orb_extractor.cpp:31-38, ORBextractor.cpp:1042-1104) -----------------------------
    def operator_kd(self, image):
        kps, desc = self.extract(image)
        tuples = [(float(k[0]), float(k[1]), float(k[2]), float(k[3]), float(k[4]), int(k[5])) for k in kps.tolist()]
        return tuples, desc

    def extract(self, image) -> tuple[np.ndarray, np.ndarray]:
        """operator_kd with structured-array output (no per-keypoint Python objects)."""
        img = np.asarray(image)
        if img.ndim not in (2, 3):
            raise RuntimeError(f"Unsupported dim {img.ndim}, only support 2d, or 3-d")
        if img.dtype != np.uint8:
            # the reference casts int32/float32 to CV_32S/CV_32F (undefined downstream) and rejects the rest
            raise RuntimeError("Unsupported type, only support uchar, int32, float")
        if img.ndim == 3:
            if img.shape[2] != 1:
                raise RuntimeError("multi-channel images are undefined behaviour in the reference (CV_8UC1 assert "
                                   "compiled out); pass a grayscale image")
            img = img[:, :, 0]
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = int(self._params.nfeatures) + 8 * self._nlevels + 64
        kps = np.empty(cap, KP_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        n = C.c_int32()
        call("orbfe_extract", self._h, ptr(img), w, h, w, ptr(kps), ptr(desc), cap, C.byref(n))
        self._extracted = w > 0 and h > 0
        n = n.value
        if n == 0:
            # _descriptors.release() / never created -> empty cv::Mat -> (0, 0) array
            self._kps, self._desc = kps[:0].copy(), np.zeros((0, 0), np.uint8)
        else:
            self._kps, self._desc = kps[:n].copy(), desc[:n].copy()
        return self._kps, self._desc

    @property
    def last_keypoints(self) -> np.ndarray:
        return self._kps

    @property
    def last_descriptors(self) -> np.ndarray:
        return self._desc
