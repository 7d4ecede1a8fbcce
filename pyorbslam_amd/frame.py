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


# Frame.__init__'s attributes that come straight from its arguments (Frame.py:15-44), which Frame.copy
# passes from `self` (Frame.py:76-77)
_CTOR_ARG_ATTRS = ("frame_args", "fx", "fy", "cx", "cy", "invfx", "invfy", "mfGridElementWidthInv",
                   "mfGridElementHeightInv", "mnMinX", "mnMaxX", "mnMinY", "mnMaxY", "FRAME_GRID_ROWS",
                   "FRAME_GRID_COLS", "mpORBvocabulary", "mbf", "mK", "mDistCoef", "mleft", "mright", "mTimeStamp",
                   "mThDepth", "mpORBextractorLeft", "mpORBextractorRight")


def frame_copy(self, frame):
    """Frame.copy (Frame.py:75-112) without its re-extraction.

    The reference builds the copy with a full Frame.__init__ on self's images — ORB extraction of both
    images, compute_stereo_matches, grid assignment — and then overwrites nearly every result with
    `frame`'s.  Extraction is deterministic, so what survives of that constructor run equals self's own
    extraction outputs; this builds the same object state directly: the constructor's attributes from
    self (fresh containers where the constructor makes fresh ones), the id draw from Frame.nNextId,
    then the reference's overrides from `frame`, in its order.  It saves one stereo-pair extraction and
    stereo match per tracked frame (Tracking.py:267, 306)."""
    cls = type(self)
    new = cls.__new__(cls)
    for k in _CTOR_ARG_ATTRS:
        setattr(new, k, getattr(self, k))
    # what the constructor run leaves that the overrides below do not replace: the id draw, mb, the raw
    # keypoint tuples of ExtractORB (Frame.py:114-121) and the extractors' pyramid copies (:59-60)
    new.mb = new.mbf / new.mK[0][0]
    new.mvKeys_ = list(self.mvKeys_)
    new.mvKeysRight_ = list(self.mvKeysRight_)
    new.mvImagePyramidLeft = [p.copy() for p in self.mvImagePyramidLeft]
    new.mvImagePyramidRight = [p.copy() for p in self.mvImagePyramidRight]
    cls.nNextId += 1
    # the reference's overrides (Frame.py:78-110)
    new.mpORBvocabulary = frame.mpORBvocabulary
    new.mpORBextractorLeft = frame.mpORBextractorLeft
    new.mpORBextractorRight = frame.mpORBextractorRight
    new.mTimeStamp = frame.mTimeStamp
    new.mK = frame.mK.copy()
    new.mDistCoef = frame.mDistCoef.copy()
    new.mbf = frame.mbf
    new.mThDepth = frame.mThDepth
    new.N = frame.N
    new.mvKeys = frame.mvKeys
    new.mvKeysRight = frame.mvKeysRight
    new.mvKeysUn = frame.mvKeysUn
    new.mvuRight = frame.mvuRight
    new.mvDepth = frame.mvDepth
    new.mBowVec = frame.mBowVec
    new.mFeatVec = frame.mFeatVec
    new.mDescriptors = frame.mDescriptors.copy()
    new.mDescriptorsRight = frame.mDescriptorsRight.copy()
    new.mvpMapPoints = frame.mvpMapPoints
    new.mvbOutlier = frame.mvbOutlier
    new.mnId = frame.mnId
    new.mpReferenceKF = frame.mpReferenceKF
    new.mnScaleLevels = frame.mnScaleLevels
    new.mfScaleFactor = frame.mfScaleFactor
    new.mfLogScaleFactor = frame.mfLogScaleFactor
    new.mvScaleFactors = frame.mvScaleFactors
    new.mvInvScaleFactors = frame.mvInvScaleFactors
    new.mvLevelSigma2 = frame.mvLevelSigma2
    new.mvInvLevelSigma2 = frame.mvInvLevelSigma2
    new.mGrid = frame.mGrid
    if frame.mTcw is not None:
        new.set_pose(frame.mTcw)
    return new


def install(frame_cls, copy: bool = True) -> None:
    """Replace Frame.compute_stereo_matches (Frame.py:161) and, unless copy=False, Frame.copy
    (Frame.py:75) of the reference class in place."""
    frame_cls.compute_stereo_matches = compute_stereo_matches
    if copy:
        frame_cls.copy = frame_copy
