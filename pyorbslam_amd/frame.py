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
`install(Frame)` (also batches Frame.ExtractORB's two images into one enqueue and replaces Frame.copy).
"""
from __future__ import annotations

import ctypes as C
import sys
from itertools import starmap

import numpy as np

from ._lib import call, ptr, pyhost
from .pyORBExtractor import LazyPyramid, ORBextractor, keypoint_tuples


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
    st = res["status"]
    if type(mbf) is float:  # built in C (_pyhost.stereo_lists): the same element types as below
        return pyhost().stereo_lists(res["u_right"], res["depth"], st, np.ascontiguousarray(kps_left["x"]), mbf)
    uR = list(res["u_right"])  # np.float32 scalars, as the reference's NumPy-2 float32 chain leaves them
    dep = list(res["depth"])
    for i in np.flatnonzero(st == 0).tolist():
        uR[i] = -1
        dep[i] = -1
    zero = np.flatnonzero(st == 2).tolist()
    if zero:
        xs = kps_left["x"]
        for i in zero:  # disparity <= 0 -> 0.01 in Python double precision (Frame.py:273-277)
            uR[i] = float(xs[i]) - 0.01
            dep[i] = mbf / 0.01
    return uR, dep


def compute_stereo_matches(frame) -> None:
    """Frame.compute_stereo_matches (Frame.py:161-279).  After the pair-batched ExtractORB below the
    result is already on the host (computed in the same enqueue as the extraction); otherwise the two
    extractors' last single-image extractions are matched on the GPU now."""
    left, right = frame.mpORBextractorLeft, frame.mpORBextractorRight
    if not isinstance(left, ORBextractor) or not isinstance(right, ORBextractor):
        raise TypeError("compute_stereo_matches needs pyorbslam_amd.pyORBExtractor.ORBextractor extractors")
    if len(left.last_keypoints) != frame.N:
        raise RuntimeError("Frame.N does not match the left extractor's last extraction")
    res = left.stereo_result
    if res is None or getattr(left, "_stereo_partner", None) is not right:
        res = stereo_match_arrays(left, right, frame.mbf, frame.mK[0][0])
    frame.mvuRight, frame.mvDepth = to_reference_lists(res, left.last_keypoints, frame.mbf)
    from .matcher import prime_u_right  # the matcher's per-frame mvuRight doubles, from the arrays
    prime_u_right(frame, res, left.last_keypoints["x"])


def _keypoint_cls(frame):
    """cv2.KeyPoint as the Frame class's module sees it (Frame.py:6, 117, 121); subclasses defined
    elsewhere resolve through their bases."""
    for cls in type(frame).__mro__:
        cv2 = getattr(sys.modules.get(cls.__module__), "cv2", None)
        if cv2 is not None and hasattr(cv2, "KeyPoint"):
            return cv2.KeyPoint
    raise RuntimeError(f"no cv2.KeyPoint in the modules of {type(frame).__name__} or its bases")


def extract_orb(self, flag, image) -> None:
    """Frame.ExtractORB (Frame.py:114-121) with the stereo pair in ONE enqueue.

    Frame.__init__ sets mleft / mright, mbf and mK before ExtractORB(0, mleft) (Frame.py:33-49), so the
    left call extracts both images, matches them and builds both sheared pyramids on the GPU
    (ORBextractor.operator_kd_stereo); ExtractORB(1, mright) then takes the waiting right results,
    GetImagePyramid() returns the device-built views and compute_stereo_matches the matched arrays.  The
    attributes written are the reference's: mvKeys_ / mDescriptors / mvKeys (flag 0) and mvKeysRight_ /
    mDescriptorsRight / mvKeysRight (flag 1).  Any other call sequence extracts one image, like the
    reference."""
    left, right = self.mpORBextractorLeft, self.mpORBextractorRight
    KeyPoint = _keypoint_cls(self)
    if flag == 0:
        mright = getattr(self, "mright", None)
        if (image is getattr(self, "mleft", None) and mright is not None and isinstance(left, ORBextractor)
                and isinstance(right, ORBextractor) and right is not left):
            kl, dl, _, _ = left.operator_kd_stereo(image, mright, right, self.mbf, self.mK[0][0])
            self.mvKeys_, self.mDescriptors = keypoint_tuples(kl), dl
        else:
            self.mvKeys_, self.mDescriptors = left.operator_kd(image)
        self.mvKeys = list(starmap(KeyPoint, self.mvKeys_))  # [KeyPoint(*kp) for kp in mvKeys_], Frame.py:117
        if isinstance(left, ORBextractor) and len(left.last_keypoints) == len(self.mvKeys):
            # the keypoints' pt, octave and angle straight from the extractor's fields (the values the
            # KeyPoints were built from), for assign_features_to_grid and the matcher while mvKeys is this list
            kl = left.last_keypoints
            self._orbfe_kxy = (self.mvKeys, np.stack((kl["x"], kl["y"]), axis=1).astype(np.float64),
                               kl["octave"].astype(np.int32), kl["angle"].astype(np.float64))
    elif flag == 1:
        pend = right.take_pending(image) if isinstance(right, ORBextractor) else None
        if pend is not None:
            self.mvKeysRight_, self.mDescriptorsRight = keypoint_tuples(pend[0]), pend[1]
        else:
            self.mvKeysRight_, self.mDescriptorsRight = right.operator_kd(image)
        self.mvKeysRight = list(starmap(KeyPoint, self.mvKeysRight_))  # Frame.py:121


# Frame.__init__'s attributes that come straight from its arguments (Frame.py:15-44), which Frame.copy
# passes from `self` (Frame.py:76-77)
_CTOR_ARG_ATTRS = ("frame_args", "fx", "fy", "cx", "cy", "invfx", "invfy", "mfGridElementWidthInv",
                   "mfGridElementHeightInv", "mnMinX", "mnMaxX", "mnMinY", "mnMaxY", "FRAME_GRID_ROWS",
                   "FRAME_GRID_COLS", "mpORBvocabulary", "mbf", "mK", "mDistCoef", "mleft", "mright", "mTimeStamp",
                   "mThDepth", "mpORBextractorLeft", "mpORBextractorRight")


def _copy_pyramid(pyr):
    if isinstance(pyr, LazyPyramid):
        return pyr.copy()
    return [p.copy() for p in pyr]


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
    # (a lazy frame's lists copy lazily: LazyPyramid.copy moves nothing while the views are on the device)
    new.mvImagePyramidLeft = _copy_pyramid(self.mvImagePyramidLeft)
    new.mvImagePyramidRight = _copy_pyramid(self.mvImagePyramidRight)
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


_undistort_local = None


def undistort_points(xy, mK, mDistCoef) -> np.ndarray:
    """cv2.undistortPoints(xy, mK, mDistCoef, None, mK) on the GPU (k_undistort): (n, 2) float32 -> (n, 2)
    float32.  Used by the Frame drop-in below and usable for Tracking.compute_image_bounds
    (Tracking.py:131-133)."""
    global _undistort_local
    import threading
    if _undistort_local is None:
        _undistort_local = threading.local()
    h = getattr(_undistort_local, "h", None)
    if h is None:
        from . import _lib
        h = C.c_void_p()
        call("orbfe_create", C.byref(_lib.make_params(2000, 1.2, 8, 20, 7)), C.byref(h))
        _undistort_local.h = h
    xy = np.ascontiguousarray(np.asarray(xy, np.float32).reshape(-1, 2))
    K = np.asarray(mK, np.float32)
    K4 = np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]], np.float32)
    d = np.ascontiguousarray(np.asarray(mDistCoef, np.float32).ravel())
    out = np.empty_like(xy)
    call("orbfe_undistort_points", h, ptr(K4), ptr(d), len(d), ptr(xy), len(xy), 2, ptr(out))
    return out


def undistort_keypoints(self):
    """Frame.undistort_keypoints (Frame.py:293-322).  Zero k1: mvKeysUn is mvKeys (the reference's only
    reachable branch).  Otherwise the reference raises NameError (it reads the undefined `mvKeys` at
    Frame.py:299); the drop-in does what that code means — cv2.undistortPoints(pts, mK, mDistCoef, None,
    mK) on the keypoints, on the GPU, new KeyPoints with the other fields kept — and assigns
    self.mvKeysUn (which the reference computes and returns but never stores) as well as returning it."""
    if self.mDistCoef[0][0] == 0:
        self.mvKeysUn = self.mvKeys
        return
    KeyPoint = _keypoint_cls(self)
    pts = np.array([kp.pt for kp in self.mvKeys], np.float32).reshape(-1, 2)
    und = undistort_points(pts, self.mK, self.mDistCoef) if len(pts) else pts
    self.mvKeysUn = [KeyPoint(x=float(und[i, 0]), y=float(und[i, 1]), size=kp.size, angle=kp.angle,
                              response=kp.response, octave=kp.octave, class_id=getattr(kp, "class_id", -1))
                     for i, kp in enumerate(self.mvKeys)]
    return self.mvKeysUn


_DOUBLE_OR_INT = (float, int, np.float64)


def assign_features_to_grid(self) -> None:
    """Frame.assign_features_to_grid + pos_in_grid (Frame.py:143-159) with the per-keypoint Python loop
    replaced by array operations: the same positions (np.round of the same float64 expression), the same
    column-major mGrid of Python lists holding keypoint indices in increasing order.  The grid is also
    kept as CSR arrays (_orbfe_grid) for the matcher's batched window queries.  Frames whose keypoint
    coordinates are not Python floats, or with no keypoints (where the reference's pos_in_grid raises),
    run the reference method."""
    kps, n = self.mvKeys, self.N
    ref = getattr(type(self), "_orbfe_ref_assign", None)
    if n == 0 or len(kps) != n or type(kps[0].pt[0]) is not float:
        if ref is None:
            raise RuntimeError("install() did not record the reference assign_features_to_grid")
        return ref(self)
    kxy = getattr(self, "_orbfe_kxy", None)
    if kxy is not None and kxy[0] is kps and len(kxy[1]) == n:
        pts = kxy[1]  # extract_orb's copy of the same coordinates (mvKeys is the list it built)
    else:
        pts = np.fromiter((c for kp in kps for c in kp.pt), np.float64, count=2 * n).reshape(n, 2)
    cols, rows = self.FRAME_GRID_COLS, self.FRAME_GRID_ROWS
    f4 = (self.mnMinX, self.mnMinY, self.mfGridElementWidthInv, self.mfGridElementHeightInv)
    if all(type(v) in _DOUBLE_OR_INT for v in f4) and type(cols) is int and type(rows) is int:
        # doubles throughout: cells, CSR and the mGrid lists in one C pass (_pyhost.grid_assign)
        self.mGrid, off, flat = pyhost().grid_assign(np.ascontiguousarray(pts, np.float64), *map(float, f4), cols, rows)
        self._orbfe_grid = (id(self.mGrid), off, flat)
        self._orbfe_pts = (kps, pts)
        return
    px = np.round((pts[:, 0] - self.mnMinX) * self.mfGridElementWidthInv).astype(int)
    py = np.round((pts[:, 1] - self.mnMinY) * self.mfGridElementHeightInv).astype(int)
    valid = (px >= 0) & (px < cols) & (py >= 0) & (py < rows)
    keep = np.flatnonzero(valid)
    cell = px[keep] * rows + py[keep]
    order = np.argsort(cell, kind="stable")  # by cell, then by keypoint index (the reference's append order)
    flat = keep[order].astype(np.int32)
    off = np.zeros(cols * rows + 1, np.int32)
    np.cumsum(np.bincount(cell, minlength=cols * rows), out=off[1:])
    self.mGrid = pyhost().grid_lists(flat, off, cols, rows)  # a new list per cell, built in C
    self._orbfe_grid = (id(self.mGrid), off, flat)
    self._orbfe_pts = (kps, pts)  # the keypoint coordinates as doubles, for the matcher's grid queries


def install(frame_cls, copy: bool = True, pair: bool = True) -> None:
    """Replace Frame.compute_stereo_matches (Frame.py:161), Frame.undistort_keypoints (Frame.py:293),
    Frame.assign_features_to_grid (Frame.py:152), unless
    pair=False Frame.ExtractORB (Frame.py:114: both images in one enqueue) and unless copy=False Frame.copy
    (Frame.py:75) of the reference class in place."""
    frame_cls.compute_stereo_matches = compute_stereo_matches
    frame_cls.undistort_keypoints = undistort_keypoints
    if frame_cls.__dict__.get("assign_features_to_grid") is not assign_features_to_grid:
        frame_cls._orbfe_ref_assign = getattr(frame_cls, "assign_features_to_grid", None)
    frame_cls.assign_features_to_grid = assign_features_to_grid
    if pair:
        frame_cls.ExtractORB = extract_orb
    if copy:
        frame_cls.copy = frame_copy
