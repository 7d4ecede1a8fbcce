"""ctypes binding of liborbfe.so (the gfx950 C-ABI declared in include/orbfe.h).

The library is built in-tree (make / __graft_entry__.build()) into pyorbslam_amd/_lib/.  There is no
CPU fallback: if the shared object is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

# ORBFE_LIB selects another in-tree build of the same C-ABI (same-box A/B of kernel revisions)
LIB_PATH = Path(os.environ.get("ORBFE_LIB") or Path(__file__).resolve().parent / "_lib" / "liborbfe.so")

ORBFE_OK = 0
ERRORS = {-1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ECAPACITY", -5: "ESTATE", -6: "EOVERFLOW", -7: "EFORMAT",
          -8: "EREJECT"}
ORBFE_ECAPACITY = -4
ORBFE_EFORMAT = -7
ORBFE_EREJECT = -8


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("resize_simd_lanes", C.c_int32)]


class BatchView(C.Structure):
    _fields_ = [("kp_cap", C.c_int32), ("n_images", C.c_int32), ("n_pairs", C.c_int32),
                ("kps", C.c_void_p), ("desc", C.c_void_p), ("count", C.c_void_p), ("u_right", C.c_void_p),
                ("depth", C.c_void_p), ("status", C.c_void_p), ("match_r", C.c_void_p), ("overflow", C.c_void_p)]


class VocabInfo(C.Structure):
    _fields_ = [("k", C.c_int32), ("L", C.c_int32), ("scoring", C.c_int32), ("weighting", C.c_int32),
                ("n_nodes", C.c_int64), ("n_words", C.c_int64), ("depth", C.c_int32), ("max_children", C.c_int32)]


# cv::KeyPoint tuple layout (opencv_type_casters.h:106-108)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                     ("octave", "<i4")])

# every symbol include/orbfe.h declares (tests check the export table against the header)
SIGNATURES = {
    "orbfe_create": [C.POINTER(Params), C.POINTER(C.c_void_p)],
    "orbfe_destroy": [C.c_void_p],
    "orbfe_last_error": [],
    "orbfe_version": [],
    "orbfe_build_id": [],
    "orbfe_get_scales": [C.c_void_p] + [C.c_void_p] * 5,
    "orbfe_extract": [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32,
                      C.POINTER(C.c_int32)],
    "orbfe_pyramid": [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)],
    "orbfe_stereo_match": [C.c_void_p, C.c_void_p, C.c_double, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p,
                           C.c_void_p, C.c_int32],
    "orbfe_frame_extract": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_float,
                            C.c_int32],
    "orbfe_frame_fetch": [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)],
    "orbfe_frame_fetch_stereo": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                 C.POINTER(C.c_int32)],
    "orbfe_frame_pyramid": [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)],
    "orbfe_frame_serial": [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)],
    "orbfe_frame_pyramid_fetch": [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64],
    "orbfe_undistort_points": [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32,
                               C.c_void_p],
    "orbfe_png_decode": [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.POINTER(C.c_int32), C.POINTER(C.c_int32)],
    "orbfe_png_read_batch": [C.POINTER(C.c_char_p), C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_int32],
    "orbfe_batch_reserve": [C.c_void_p, C.c_int32, C.c_int32, C.c_int32],
    "orbfe_extract_batch_device": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p],
    "orbfe_stereo_batch_device": [C.c_void_p, C.c_int32, C.c_double, C.c_float, C.c_void_p],
    "orbfe_frontend_batch_device": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_double, C.c_float, C.c_void_p],
    "orbfe_batch_view_get": [C.c_void_p, C.POINTER(BatchView)],
    "orbfe_batch_status": [C.c_void_p, C.POINTER(C.c_int32)],
    "orbfe_batch_record_bytes": [C.c_void_p, C.POINTER(C.c_int64)],
    "orbfe_batch_pack_device": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p],
    "orbfe_batch_compact_record_bytes": [C.c_void_p, C.POINTER(C.c_int64)],
    "orbfe_batch_pack_compact_device": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p],
    "orbfe_batch_fetch": [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)],
    "orbfe_batch_fetch_stereo": [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                 C.POINTER(C.c_int32)],
    "orbfe_hamming_search": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "orbfe_hamming_csr": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                          C.c_void_p],
    "orbfe_descriptor_distance": [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)],
    "orbfe_grid_query": [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                         C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_int64],
    "orbfe_select_f_f": [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_double, C.c_int32, C.c_void_p],
    "orbfe_select_f_p": [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_double, C.c_int32, C.c_void_p],
    "orbfe_hamming_matrix": [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p],
    "orbfe_profile_begin": [C.c_void_p, C.c_int32],
    "orbfe_profile_read": [C.c_void_p, C.c_void_p, C.POINTER(C.c_int32)],
    "orbfe_microbench": [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_float)],
    "orbfe_debug_candidates": [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)],
    "orbfe_debug_selected": [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32)],
    "orbfe_debug_octree_profile": [C.c_void_p, C.c_void_p, C.c_int64],
    "orbfe_debug_cascade_profile": [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p],
    "orbfe_set_lanes": [C.c_void_p, C.c_int32],
    "orbfe_abi_version": [],
    "orbfe_set_graphs": [C.c_void_p, C.c_int32],
    "orbfe_graph_stats": [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int32)],
    "orbfe_set_octree_kernel": [C.c_void_p, C.c_int32],
    "orbfe_get_octree_kernel": [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)],
    "orbfe_debug_detect_stats": [C.c_void_p, C.POINTER(C.c_int64)],
    "orbfe_vocab_load_text": [C.c_char_p, C.POINTER(C.c_void_p)],
    "orbfe_vocab_create": [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                           C.c_void_p, C.POINTER(C.c_void_p)],
    "orbfe_vocab_destroy": [C.c_void_p],
    "orbfe_vocab_get_info": [C.c_void_p, C.POINTER(VocabInfo)],
    "orbfe_vocab_get_nodes": [C.c_void_p] * 6,
    "orbfe_vocab_transform": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p],
    "orbfe_vocab_transform_device": [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p],
    "orbfe_vocab_last_ms": [C.c_void_p, C.POINTER(C.c_float)],
}

_lib: C.CDLL | None = None


class OrbfeError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed: {ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load liborbfe.so (raises OSError if it is missing: no fallback path exists)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OSError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build()) first; "
                          "pyorbslam_amd has no CPU fallback")
        L = C.CDLL(str(LIB_PATH))
        for name, argtypes in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None and os.environ.get("ORBFE_LIB"):
                continue  # an older revision under A/B may predate some entry points
            if fn is None:
                raise OSError(f"{LIB_PATH} does not export {name}")
            fn.argtypes = argtypes
            fn.restype = C.c_char_p if name in ("orbfe_last_error", "orbfe_version", "orbfe_build_id") else C.c_int
        _lib = L
    return _lib


_pyhost = None


def pyhost():
    """The host-side CPython extension `_pyhost` (csrc/orbfe_pyhost.cpp): the per-frame Python objects of the
    reference data model (KeyPoint tuples, Frame.mGrid, mvuRight / mvDepth) built in C.  Raises ImportError
    when it is not built (`make`)."""
    global _pyhost
    if _pyhost is None:
        try:
            from . import _pyhost as m
        except ImportError as e:
            raise ImportError("pyorbslam_amd/_pyhost extension not built: run `make` (or __graft_entry__.build())") from e
        _pyhost = m
    return _pyhost


class OrbfeGeometryError(OrbfeError, ValueError):
    """A level geometry the reference's DistributeOctTree cannot take (vpIniNodes.resize of a negative nIni,
    ORBextractor.cpp:543-550): the reference throws std::length_error, which pybind11 raises as ValueError."""


def check(fn: str, rc: int) -> None:
    if rc != ORBFE_OK:
        msg = lib().orbfe_last_error().decode(errors="replace")
        if rc == -1 and "DistributeOctTree" in msg:  # EINVAL
            raise OrbfeGeometryError(fn, rc, msg)
        raise OrbfeError(fn, rc, msg)


def call(name: str, *args) -> None:
    check(name, getattr(lib(), name)(*args))


def has(name: str) -> bool:
    """Whether the loaded library exports `name` (always true for the in-tree build, which must export every
    declared symbol; an older build under ORBFE_LIB A/B may predate some)."""
    return getattr(lib(), name, None) is not None


def ptr(a: np.ndarray | None) -> C.c_void_p | None:
    return None if a is None else C.c_void_p(a.ctypes.data)


def make_params(nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                resize_simd_lanes: int = 16) -> Params:
    # pybind11 narrows the scaleFactor argument to C++ float (orb_extractor.cpp:23)
    return Params(int(nfeatures), float(np.float32(scaleFactor)), int(nlevels), int(iniThFAST), int(minThFAST),
                  int(resize_simd_lanes))


def version() -> str:
    return lib().orbfe_version().decode()


def build_id() -> str:
    """SHA-256 prefix of the sources the loaded library was built from (orbfe_build_id)."""
    fn = getattr(lib(), "orbfe_build_id", None)
    return fn().decode() if fn is not None else "unknown"


def gpu_available() -> bool:
    try:
        import torch
        return bool(torch.cuda.is_available())
    except Exception:  # pragma: no cover
        return False
