"""Drop-in for Frame.compute_stereo_matches (reference Frame.py:161-279).

The reference method reads the two extractors' last outputs (keypoints, descriptors, sheared pyramids)
from the Frame and writes Frame.mvuRight / Frame.mvDepth.  Here the whole search (row bands, octave and
disparity gates, Hamming first-minimum, 11x11 SAD over 11 shifts on the sheared pyramid, parabola fit,
depth) runs in k_stereo on the data the extractors left on the GPU; only the result lists are built on
the host, with the reference's element types:

    unmatched       Python int -1
    matched         np.float32 (NumPy-2 float32 chain of the reference)
    zero disparity  Python float: uR = uL - 0.01, depth = mbf / 0.01 (Frame.py:273-277)

Use either as a function, `compute_stereo_matches(frame)`, or patch the reference class once:
`install(Frame)`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import call, ptr
from .pyORBExtractor import ORBextractor


def stereo_match_arrays(left: ORBextractor, right: ORBextractor, mbf: float, fx32) -> dict:
    """Raw result arrays of the GPU stereo matcher for the extractors' last images."""
    n = len(left.last_keypoints)
    u = np.empty(n, np.float32)
    d = np.empty(n, np.float32)
    st = np.empty(n, np.int8)
    m = np.empty(n, np.int32)
    call("orbfe_stereo_match", left.handle, right.handle, float(mbf), float(np.float32(fx32)), ptr(u), ptr(d), ptr(st),
         ptr(m), n)
    return dict(u_right=u, depth=d, status=st, match_r=m)


def to_reference_lists(res: dict, kps_left: np.ndarray, mbf: float) -> tuple[list, list]:
    uR, dep = [], []
    xs = kps_left["x"].tolist() if len(kps_left) else []
    for i, s in enumerate(res["status"].tolist()):
        if s == 0:
            uR.append(-1)
            dep.append(-1)
        elif s == 1:
            uR.append(np.float32(res["u_right"][i]))
            dep.append(np.float32(res["depth"][i]))
        else:
            uR.append(xs[i] - 0.01)
            dep.append(mbf / 0.01)
    return uR, dep


def compute_stereo_matches(frame) -> None:
    left, right = frame.mpORBextractorLeft, frame.mpORBextractorRight
    if not isinstance(left, ORBextractor) or not isinstance(right, ORBextractor):
        raise TypeError("compute_stereo_matches needs pyorbslam_amd.pyORBExtractor.ORBextractor extractors")
    if len(left.last_keypoints) != frame.N:
        raise RuntimeError("Frame.N does not match the left extractor's last extraction")
    res = stereo_match_arrays(left, right, frame.mbf, frame.mK[0][0])
    frame.mvuRight, frame.mvDepth = to_reference_lists(res, left.last_keypoints, frame.mbf)


def install(frame_cls) -> None:
    """Replace Frame.compute_stereo_matches of the reference class (Frame.py:161) in place."""
    frame_cls.compute_stereo_matches = compute_stereo_matches
