"""Drop-in for the reference's pybind11 module `pyORBExtractor` (pyORBExtractor/orb_extractor.cpp:16-40).

    from pyorbslam_amd.pyORBExtractor import ORBextractor     # instead of `from pyORBExtractor import ...`

Same constructor (keyword names of orb_extractor.cpp:23), same getters and the same return types:
operator_kd(image) -> (list of (x, y, size, angle, response, octave) tuples, (N, 32) uint8 ndarray), and
GetImagePyramid() -> list of uint8 arrays reproducing the reference caster's stride-ignoring copy.
All pixel work runs in the gfx950 library (liborbfe.so); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import weakref
from collections.abc import Sequence

import numpy as np

from . import _lib
from ._lib import KP_DTYPE, call, ptr


FRAME_RING = 8  # include/orbfe.h ORBFE_FRAME_RING: frames whose sheared views stay on the device


class LazyPyramid(Sequence):
    """GetImagePyramid() after a lazy frame (operator_kd_stereo with want_pyramid=True): the reference's list
    of sheared uint8 views (opencv_type_casters.h:232-239), fetched from the device ring the first time an
    element is read (index, iteration, comparison, copy) — Frame.__init__ stores both lists (Frame.py:59-60)
    but the tracking loop reads them only in the reference's own compute_stereo_matches, which the GPU path
    replaces.  Before ORBFE_FRAME_RING newer frames of its extractor evict the views, a list still alive is
    fetched.  Indexing and len() behave as on the list; the type is not `list` (a list subclass could be read
    by CPython's fast paths without filling)."""

    __slots__ = ("_src", "_levels", "__weakref__")

    def __init__(self, owner, side: int, serial: int):
        self._src = (owner, side, serial)
        self._levels = None
        owner._lazy.append((serial, weakref.ref(self)))

    def _fill(self) -> list:
        if self._levels is None:
            owner, side, serial = self._src
            self._levels = owner._fetch_ring(side, serial)
            self._src = None
        return self._levels

    @property
    def filled(self) -> bool:
        return self._levels is not None

    def __len__(self) -> int:
        return len(self._levels) if self._levels is not None else self._src[0]._nlevels

    def __getitem__(self, i):
        return self._fill()[i]

    def __iter__(self):
        return iter(self._fill())

    def __eq__(self, other):
        return list(self) == (list(other) if isinstance(other, (LazyPyramid, list)) else other)

    def __add__(self, other):
        return list(self) + list(other)

    def __radd__(self, other):
        return list(other) + list(self)

    def copy(self):
        """Another lazy list of the same views while they are on the device (Frame.copy keeps the pyramids
        without moving them); a list of copied arrays once fetched."""
        if self._levels is None:
            owner, side, serial = self._src
            return LazyPyramid(owner, side, serial)
        return [a.copy() for a in self._levels]

    def __repr__(self) -> str:
        return repr(self._fill())


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
        self._frame_hw, self._frame_shapes = None, None  # operator_kd_stereo's image size, its level sizes
        # after operator_kd_stereo: (left extractor, side) whose frame holds this extractor's pyramid, the
        # stereo result of the pair (left extractor), and the right image whose results wait for
        # ExtractORB(1).  The left extractor lists the extractors reading its frame (_dependents) and hands
        # them a host copy of their pyramid (_pyr_cache) before its next extraction replaces the frame, so
        # every extractor's pyramid stays its own, as in the reference.
        self._pyr_src = None
        self._pyr_cache = None
        self._dependents = []
        # lazy frames (want_pyramid=True): (serial, weakref) of every LazyPyramid handed out, and the
        # extractors whose pyramid is a frame of this handle still in the device ring
        self._lazy = []
        self._ring_dependents = []
        self.stereo_result = None
        self._pending_image = None

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
        if self._pyr_cache is not None:
            if not sheared:
                raise RuntimeError("GetImagePyramid(sheared=False) is not available after operator_kd_stereo")
            return [a.copy() for a in self._pyr_cache]
        out = []
        if self._pyr_src is not None and sheared and self._pyr_src[3]:  # a lazy frame: views in the device ring
            owner, side, serial, _ = self._pyr_src
            return LazyPyramid(owner, side, serial)
        if self._pyr_src is not None and sheared:  # the frame path: every level out of one allocation
            owner, side = self._pyr_src[:2]
            shapes = owner._level_shapes(side)
            buf = np.empty(sum(hh * ww for hh, ww in shapes), np.uint8)
            o = 0
            for l, (hh, ww) in enumerate(shapes):
                a = buf[o:o + hh * ww].reshape(hh, ww)
                o += hh * ww
                call("orbfe_frame_pyramid", owner.handle, side, l, ptr(a), None, None)
                out.append(a)
            return out
        if self._pyr_src is not None:
            raise RuntimeError("GetImagePyramid(sheared=False) is not available after operator_kd_stereo")
        for l in range(self._nlevels):
            w, h = C.c_int32(), C.c_int32()
            call("orbfe_pyramid", self._h, l, None, int(sheared), C.byref(w), C.byref(h))
            a = np.empty((h.value, w.value), np.uint8)
            call("orbfe_pyramid", self._h, l, ptr(a), int(sheared), C.byref(w), C.byref(h))
            out.append(a)
        return out

    def _level_shapes(self, side: int) -> list:
        """(h, w) of every level of this handle's frame geometry (cleared by a frame of another size)."""
        shapes = self._frame_shapes
        if shapes is None:
            shapes = []
            for l in range(self._nlevels):
                w, h = C.c_int32(), C.c_int32()
                call("orbfe_frame_pyramid", self._h, side, l, None, C.byref(w), C.byref(h))
                shapes.append((h.value, w.value))
            self._frame_shapes = shapes
        return shapes

    def _fetch_ring(self, side: int, serial: int) -> list:
        """Side `side`'s sheared views of this handle's frame `serial` from the device ring: one transfer into
        one allocation, the levels at their 4-byte aligned offsets (orbfe_frame_pyramid_fetch)."""
        shapes = self._level_shapes(side)
        offs, o = [], 0
        for hh, ww in shapes:
            offs.append(o)
            o += (hh * ww + 3) & ~3
        buf = np.empty(max(o, 1), np.uint8)
        call("orbfe_frame_pyramid_fetch", self._h, int(serial), int(side), ptr(buf), o)
        return [buf[a:a + hh * ww].reshape(hh, ww) for a, (hh, ww) in zip(offs, shapes)]

    def _evict_ring(self, next_serial: int) -> None:
        """Before frame `next_serial` replaces ring slot next_serial % FRAME_RING: fetch every lazy pyramid
        still alive and unread whose frame would leave the ring, and give the extractors still reading such a
        frame a host copy."""
        keep = []
        for serial, ref in self._lazy:
            lp = ref()
            if lp is None or lp.filled:
                continue
            if serial <= next_serial - FRAME_RING:
                lp._fill()
            else:
                keep.append((serial, ref))
        self._lazy = keep
        deps = []
        for ex in self._ring_dependents:
            src = ex._pyr_src
            if src is None or src[0] is not self or not src[3]:
                continue
            if src[2] <= next_serial - FRAME_RING:
                ex._pyr_cache = self._fetch_ring(src[1], src[2]) if ex._extracted else None
                ex._pyr_src = None
            else:
                deps.append(ex)
        self._ring_dependents = deps

    # ---- operator_kd (orb_extractor.cpp:31-38, ORBextractor.cpp:1042-1104) -----------------------------
    def operator_kd(self, image):
        kps, desc = self.extract(image)
        return keypoint_tuples(kps), desc

    def _cap(self) -> int:
        return int(self._params.nfeatures) + 8 * self._nlevels + 64

    def _set_result(self, kps: np.ndarray, desc: np.ndarray, n: int, extracted: bool, exact: bool = False) -> None:
        """exact: kps / desc are already the n records (fresh arrays), kept without a copy."""
        self._extracted = extracted
        if n == 0:
            # _descriptors.release() / never created -> empty cv::Mat -> (0, 0) array
            self._kps, self._desc = kps[:0].copy(), np.zeros((0, 0), np.uint8)
        elif exact:
            self._kps, self._desc = kps, desc
        else:
            self._kps, self._desc = kps[:n].copy(), desc[:n].copy()

    def _release_frame(self, replaced=None) -> None:
        """Before this handle's frame is replaced: the extractors still reading their pyramid from it get a
        host copy of it (the right extractor of an earlier pair must keep its own pyramid), except
        `replaced`, the right extractor of the pair about to be extracted, whose results the new frame
        replaces anyway (until then it reports no extraction, as after a failed call)."""
        for ex in self._dependents:
            if ex._pyr_src is not None and ex._pyr_src[0] is self:
                if ex is replaced:
                    ex._extracted = False
                elif ex._pyr_src[3]:  # a lazy frame: its views stay in the device ring (_evict_ring)
                    self._ring_dependents.append(ex)
                    continue
                else:
                    ex._pyr_cache = ex.GetImagePyramid() if ex._extracted else None
                ex._pyr_src = None
        self._dependents = []

    def extract(self, image) -> tuple[np.ndarray, np.ndarray]:
        """operator_kd with structured-array output (no per-keypoint Python objects)."""
        img = as_gray_u8(image)
        h, w = img.shape
        cap = self._cap()
        kps = np.empty(cap, KP_DTYPE)
        desc = np.empty((cap, 32), np.uint8)
        n = C.c_int32()
        self._release_frame()
        if self._frame_hw is not None and (h, w) != self._frame_hw and h and w:
            self._evict_ring(2 ** 62)  # another geometry clears the ring (reserve): read every lazy list first
        self._pyr_src = None
        self._pyr_cache = None
        self.stereo_result = None
        self._pending_image = None
        call("orbfe_extract", self._h, ptr(img), w, h, w, ptr(kps), ptr(desc), cap, C.byref(n))
        self._set_result(kps, desc, n.value, w > 0 and h > 0)
        return self._kps, self._desc

    # ---- one stereo frame in one enqueue ---------------------------------------------------------------
    def operator_kd_stereo(self, left, right, right_extractor: "ORBextractor", mbf: float, fx32,
                           want_pyramid: bool = True):
        """Frame.__init__'s ExtractORB(0, left) + ExtractORB(1, right) + GetImagePyramid() of both
        extractors + compute_stereo_matches (Frame.py:48-65, 161-279) as ONE enqueue on this extractor's
        handle (orbfe_frame_extract): one host->device copy per image, the 2-image pipeline, the stereo
        match and the sheared pyramids, then one synchronisation.

        Afterwards this extractor holds the left results and `right_extractor` the right ones, exactly as
        if each had run operator_kd (last_keypoints, last_descriptors, GetImagePyramid), and
        self.stereo_result holds the raw stereo arrays of the pair.  Returns
        (kps_left, desc_left, kps_right, desc_right) as structured arrays."""
        if right_extractor is self:
            raise ValueError("the right image needs its own extractor (the reference keeps one per camera)")
        L, R = as_gray_u8(left), as_gray_u8(right)
        if L.shape != R.shape:
            raise RuntimeError("left and right images differ in size")
        h, w = L.shape
        self._release_frame(replaced=right_extractor)
        if (h, w) != self._frame_hw:
            # a new geometry: the ring's frames are gone (reserve), so every lazy list still unread is read now
            self._evict_ring(2 ** 62)
            self._frame_hw, self._frame_shapes = (h, w), None
        else:
            serial = C.c_int64()
            call("orbfe_frame_serial", self._h, C.byref(serial), None)
            self._evict_ring(serial.value + 1)
        # want_pyramid: the sheared views stay on the device until read (2, lazy); False: built on request
        call("orbfe_frame_extract", self._h, ptr(L), ptr(R), w, h, w, float(mbf), float(np.float32(fx32)),
             2 if want_pyramid else 0)
        if w > 0 and h > 0 and self._frame_shapes is None:
            # the level sizes now, while orbfe_frame_pyramid answers (it needs this handle's last call to be a
            # frame): a lazy list read after a plain extract() on this handle still finds them
            self._level_shapes(0)
        serial = C.c_int64()
        call("orbfe_frame_serial", self._h, C.byref(serial), None)
        lazy = bool(want_pyramid)
        out = []
        for side, ex in ((0, self), (1, right_extractor)):
            n = C.c_int32()  # the count first (no copy), then the records straight into exact-size arrays
            call("orbfe_frame_fetch", self._h, side, None, None, 2 ** 31 - 1, C.byref(n))
            kps = np.empty(n.value, KP_DTYPE)
            desc = np.empty((n.value, 32), np.uint8)
            call("orbfe_frame_fetch", self._h, side, ptr(kps), ptr(desc), n.value, C.byref(n))
            ex._set_result(kps, desc, n.value, w > 0 and h > 0, exact=True)
            ex._pyr_src = (self, side, serial.value, lazy) if w > 0 and h > 0 else None
            ex._pyr_cache = None
            ex.stereo_result = None
            out += [ex._kps, ex._desc]
        n = len(self._kps)
        res = dict(u_right=np.empty(n, np.float32), depth=np.empty(n, np.float32), status=np.empty(n, np.int8),
                   match_r=np.empty(n, np.int32))
        nn = C.c_int32()
        call("orbfe_frame_fetch_stereo", self._h, ptr(res["u_right"]), ptr(res["depth"]), ptr(res["status"]),
             ptr(res["match_r"]), n, C.byref(nn))
        self.stereo_result = res
        self._stereo_partner = right_extractor
        self._dependents = [right_extractor]
        right_extractor._pending_image = right
        return tuple(out)

    def take_pending(self, image):
        """The right-image results of the last operator_kd_stereo if `image` is that call's right image
        (Frame.ExtractORB(1, ...) right after ExtractORB(0, ...)); None otherwise."""
        if self._pending_image is None or self._pending_image is not image:
            return None
        self._pending_image = None
        return self._kps, self._desc

    @property
    def last_keypoints(self) -> np.ndarray:
        return self._kps

    @property
    def last_descriptors(self) -> np.ndarray:
        return self._desc


def as_gray_u8(image) -> np.ndarray:
    """The reference caster's input rules (opencv_type_casters.h:163-200): 2-D uint8, or 3-D with one channel;
    int32 / float32 are undefined behaviour downstream and every other dtype raises.

    Strides: the caster builds cv::Mat(nh, nw, CV_8UC1, info.ptr) from the buffer's first element and IGNORES
    numpy's strides (opencv_type_casters.h:200), so a non-contiguous view (a sliced ROI, every other row, ...)
    is read as nh x nw consecutive bytes starting at its first element.  The same bytes are read here (a
    zero-copy (nh, nw) view over them), so such a view yields the reference's keypoints, not those of the
    pixels the view shows.  Where those bytes would run past the end of the array's buffer (e.g. a
    negative-stride view), the reference reads out of bounds; this raises RuntimeError instead."""
    img = np.asarray(image)
    if img.ndim not in (2, 3):
        raise RuntimeError(f"Unsupported dim {img.ndim}, only support 2d, or 3-d")
    if img.dtype != np.uint8:
        # the reference casts int32/float32 to CV_32S/CV_32F (undefined downstream) and rejects the rest
        raise RuntimeError("Unsupported type, only support uchar, int32, float")
    if img.ndim == 3 and img.shape[2] != 1:
        raise RuntimeError("multi-channel images are undefined behaviour in the reference (CV_8UC1 assert "
                           "compiled out); pass a grayscale image")
    nh, nw = int(img.shape[0]), int(img.shape[1])
    if img.ndim == 3:
        img = img[:, :, 0]
    if img.flags.c_contiguous or nh * nw == 0:
        return np.ascontiguousarray(img)
    return _stride_ignoring_view(img, nh, nw)


def _stride_ignoring_view(img: np.ndarray, nh: int, nw: int) -> np.ndarray:
    """nh x nw consecutive bytes from img's first element, as a (nh, nw) array sharing img's memory."""
    owner = img
    while isinstance(owner.base, np.ndarray):
        owner = owner.base
    lo, hi = np.lib.array_utils.byte_bounds(owner)
    p = img.__array_interface__["data"][0]
    if not owner.flags.c_contiguous or p < lo or p + nh * nw > hi:
        raise RuntimeError("this strided view, read as nh x nw consecutive bytes from its first element (what the "
                           "reference's caster does, opencv_type_casters.h:200), would run past its buffer")
    flat = owner.reshape(-1).view(np.uint8)
    return flat[p - lo:p - lo + nh * nw].reshape(nh, nw)


def keypoint_tuples(kps: np.ndarray) -> list:
    """cv::KeyPoint tuples (x, y, size, angle, response, octave) as the reference caster builds them
    (opencv_type_casters.h:106-108): Python floats (exact f32 values) and an int, built in C
    (`_pyhost.keypoint_tuples`; the structured array's tolist is ~3x slower)."""
    if kps.dtype != KP_DTYPE:
        raise TypeError("keypoint records must have the orbfe_keypoint dtype")
    return _lib.pyhost().keypoint_tuples(np.ascontiguousarray(kps))
