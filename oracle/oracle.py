"""TEST INFRASTRUCTURE ONLY — ctypes access to the C++ extractor checker (oracle/build/liborboracle.so).

Mirrors the reference pyORBExtractor surface closely enough for tests: extract(image) returns the
(x, y, size, angle, response, octave) rows and the (N, 32) descriptor block of
ORBextractor::operator_kd (ORBextractor.cpp:1042-1104); pyramid() returns the unpadded levels and
sheared() rebuilds what GetImagePyramid hands to Python (opencv_type_casters.h:232-239).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liborboracle.so"
EDGE = 19


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("resize_simd_lanes", C.c_int32)]


KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            subprocess.check_call(["make", "-s", "-C", str(HERE)])
        L = C.CDLL(str(LIB_PATH))
        P = C.POINTER(Params)
        vp = C.c_void_p
        L.oracle_extract.argtypes = [P, vp, C.c_int32, C.c_int32, C.c_int32, vp, vp, C.c_int32,
                                     C.POINTER(C.c_int32), vp]
        L.oracle_tables.argtypes = [P, vp, vp, vp, vp, vp, vp]
        L.oracle_level_sizes.argtypes = [P, C.c_int32, C.c_int32, vp]
        L.oracle_resize.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32, C.c_int32, C.c_int32]
        L.oracle_blur7.argtypes = [vp, C.c_int32, C.c_int32, vp]
        L.oracle_fast.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp, C.c_int32]
        L.oracle_level_candidates.argtypes = [P, vp, C.c_int32, C.c_int32, vp, C.c_int32]
        L.oracle_octree.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, vp,
                                    C.c_int32]
        L.oracle_octree_ties.argtypes = [P, vp, C.c_int32, C.c_int32, C.c_int32, vp]
        L.oracle_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.oracle_fast_atan2.restype = C.c_float
        L.oracle_cosf.argtypes = [C.c_float]
        L.oracle_cosf.restype = C.c_float
        L.oracle_sinf.argtypes = [C.c_float]
        L.oracle_sinf.restype = C.c_float
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


class OracleExtractor:
    """Reference-semantics extractor on the CPU (one instance per camera, like ORBextractor)."""

    def __init__(self, nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7, resize_simd_lanes=16):
        self.p = Params(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST), int(minThFAST),
                        int(resize_simd_lanes))
        self.nlevels = int(nlevels)
        self._pyr: list[np.ndarray] = []

    def tables(self):
        L = self.nlevels
        sf, isf, s2, is2 = (np.zeros(L, np.float32) for _ in range(4))
        npl = np.zeros(L, np.int32)
        um = np.zeros(16, np.int32)
        rc = lib().oracle_tables(C.byref(self.p), _ptr(sf), _ptr(isf), _ptr(s2), _ptr(is2), _ptr(npl), _ptr(um))
        assert rc == 0
        return dict(scale=sf, inv_scale=isf, sigma2=s2, inv_sigma2=is2, n_per_level=npl, umax=um)

    def level_sizes(self, w: int, h: int) -> list[tuple[int, int]]:
        wh = np.zeros(2 * self.nlevels, np.int32)
        lib().oracle_level_sizes(C.byref(self.p), w, h, _ptr(wh))
        return [(int(wh[2 * l]), int(wh[2 * l + 1])) for l in range(self.nlevels)]

    def extract(self, image: np.ndarray):
        """Returns (kps structured array with KP_DTYPE fields, desc (N,32) u8)."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = image.shape
        sizes = self.level_sizes(w, h) if w and h else []
        pyr = np.zeros(sum(a * b for a, b in sizes) or 1, np.uint8)
        cap = int(self.p.nfeatures) + 4 * self.nlevels + 16
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = C.c_int32()
        rc = lib().oracle_extract(C.byref(self.p), _ptr(image), w, h, w, _ptr(kps), _ptr(desc), cap, C.byref(n),
                                  _ptr(pyr))
        if rc == -1 and w and h:
            raise ValueError("the reference's DistributeOctTree refuses this geometry (vpIniNodes.resize of a negative "
                             "nIni, ORBextractor.cpp:543-550: std::length_error)")
        if rc != 0:
            raise RuntimeError(f"oracle_extract failed: {rc}")
        self._pyr = []
        o = 0
        for (lw, lh) in sizes:
            self._pyr.append(pyr[o:o + lw * lh].reshape(lh, lw).copy())
            o += lw * lh
        return kps[:n.value].copy(), desc[:n.value].copy()

    def octree_ties(self, image: np.ndarray) -> np.ndarray:
        """SURVEY H1 per level: (straddle, tie_runs, careful_iters, run_len, run_divided) — see
        oracle_octree_ties (orb_oracle.h)."""
        image = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = image.shape
        out = np.zeros((self.nlevels, 5), np.int32)
        rc = lib().oracle_octree_ties(C.byref(self.p), _ptr(image), w, h, w, _ptr(out))
        if rc != 0:
            raise RuntimeError(f"oracle_octree_ties failed: {rc}")
        return out

    def pyramid(self) -> list[np.ndarray]:
        return [p.copy() for p in self._pyr]

    def sheared_pyramid(self) -> list[np.ndarray]:
        return [sheared(p) for p in self._pyr]


def padded(level: np.ndarray) -> np.ndarray:
    """copyMakeBorder(level, 19, 19, 19, 19, BORDER_REFLECT_101) (ORBextractor.cpp:1122-1128)."""
    return np.pad(level, EDGE, mode="reflect")


def sheared(level: np.ndarray) -> np.ndarray:
    """What the reference's Mat->ndarray caster returns for a pyramid level: the ROI's data pointer read
    with a contiguous stride w instead of Mat::step = w + 38 (opencv_type_casters.h:232-239)."""
    h, w = level.shape
    flat = padded(level).ravel()
    base = EDGE * (w + 2 * EDGE) + EDGE
    return flat[base:base + h * w].reshape(h, w).copy()


def level_candidates(params: Params, level: np.ndarray) -> np.ndarray:
    level = np.ascontiguousarray(level, np.uint8)
    h, w = level.shape
    cap = max(1024, w * h // 2)
    out = np.zeros((cap, 3), np.int32)
    n = lib().oracle_level_candidates(C.byref(params), _ptr(level), w, h, _ptr(out), cap)
    assert n >= 0, n
    return out[:n].copy()


def octree(xyr: np.ndarray, minX: int, maxX: int, minY: int, maxY: int, N: int) -> np.ndarray:
    xyr = np.ascontiguousarray(xyr, np.int32).reshape(-1, 3)
    cap = max(64, 4 * N + 64)
    out = np.zeros((cap, 3), np.int32)
    n = lib().oracle_octree(_ptr(xyr), len(xyr), minX, maxX, minY, maxY, N, _ptr(out), cap)
    assert n >= 0, n
    return out[:n].copy()


def resize(src: np.ndarray, dw: int, dh: int, simd_lanes: int = 16) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.uint8)
    assert lib().oracle_resize(_ptr(src), sw, sh, sw, _ptr(dst), dw, dh, simd_lanes) == 0
    return dst


def blur7(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    h, w = src.shape
    dst = np.zeros_like(src)
    assert lib().oracle_blur7(_ptr(src), w, h, _ptr(dst)) == 0
    return dst


def fast(img: np.ndarray, th: int) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = w * h
    out = np.zeros((cap, 3), np.int32)
    n = lib().oracle_fast(_ptr(img), w, w, h, th, _ptr(out), cap)
    assert n >= 0
    return out[:n].copy()
