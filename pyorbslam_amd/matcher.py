"""Drop-in for the reference ORBMatcher (ORBMatcher.py): every search of the class.

descriptor_distance (ORBMatcher.py:12-14), the BoW searches search_by_BoW_kf_f / _kf_kf (:21-213), the
projection searches search_by_projection_f_p / _f_f / _ckf_scw_mp / _f_kf_f (:215-393, 850-1008), the
fusions fuse_kf_scw_mp / fuse_pkf_mp (:395-582), search_for_triangulation (:584-711) and search_by_sim3
(:713-848) keep the reference's control flow and results exactly; what changes is where the popcounts
happen.  The reference calls a per-byte Python popcount (~10 us) once per
candidate inside the search loop.  Here every (query, candidate) pair of a search is collected first —
the candidate windows depend only on the frame grid, never on matches made during the search — and
all distances come back from ONE k_hamming_search launch (orbfe_hamming_csr).  The sequential part
that genuinely depends on earlier iterations (candidates already holding a map point with
observations, the stereo gate, best / second-best bookkeeping, the rotation histogram) then runs on the
host over those precomputed distances, evaluating the same Python expressions on the same objects, so
every dtype promotion of the reference is preserved.

The split into "collect, then replay" is exact because everything the collection phase evaluates is
static during a search (keypoints, grids, poses, map-point geometry, map-point badness at collection
time — badness never reverts), while every piece of state a search mutates (matched slots, keyframe
map-point slots, observations) is read in the replay phase at the reference's point in the loop.  The one
input a search can change under itself is a map point's descriptor (fuse_pkf_mp: MapPoint.replace
recomputes the survivor's distinctive descriptor, MapPoint.py:180); the replay compares the descriptor it
reads with the collected one and re-runs that query's distances on the GPU when they differ.

The replay loops restate ORBMatcher.py statement by statement on purpose: a drop-in must reproduce the
reference's control flow, NumPy-2 dtype promotions and the order of its side effects exactly, so those
lines necessarily read like the reference's.  The two tracking searches also have a native selection
(orbfe_select_f_f / _f_p, host C) used when every compared value is a double.
"""
from __future__ import annotations

import ctypes as C
import operator
import threading
import weakref
from collections import deque
from itertools import compress, repeat

import numpy as np

from . import _lib
from ._lib import call, ptr

TH_HIGH = 100     # ORBMatcher.py:3
TH_LOW = 50       # ORBMatcher.py:4
HISTO_LENGTH = 30  # ORBMatcher.py:5


class _OwnedHandle:
    """An orbfe handle (own stream + Hamming scratch) destroyed with its owner."""

    def __init__(self):
        self.h = C.c_void_p()
        call("orbfe_create", C.byref(_lib.make_params(2000, 1.2, 8, 20, 7)), C.byref(self.h))

    def __del__(self):
        if self.h.value and _lib._lib is not None:
            _lib.lib().orbfe_destroy(self.h)
            self.h = C.c_void_p()


# One handle per calling thread: the reference runs Tracking, LocalMapping and LoopClosing as threads
# that all use ORBMatcher and MapPoint (System.py:59-64).  A thread's handle is destroyed with its
# thread-local storage; the C side also serialises the Hamming calls of one handle (orbfe_ctx::hmu).
_local = threading.local()


def _h():
    o = getattr(_local, "owned", None)
    if o is None:
        o = _local.owned = _OwnedHandle()
    return o.h


def hamming_csr(queries: np.ndarray, train: np.ndarray, cand_off: np.ndarray, cand_idx: np.ndarray) -> np.ndarray:
    """popcount(queries[q] ^ train[cand_idx[k]]) for k in [cand_off[q], cand_off[q+1]), on the GPU."""
    q = np.ascontiguousarray(queries, np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
    off = np.ascontiguousarray(cand_off, np.int32)
    idx = np.ascontiguousarray(cand_idx, np.int32)
    out = np.empty(max(int(off[-1]) if len(off) else 0, 1), np.int32)
    if len(q) == 0 or off[-1] == 0:
        return out[:0]
    call("orbfe_hamming_csr", _h(), ptr(q), len(q), ptr(t), len(t), ptr(off), ptr(idx), ptr(out))
    return out[:int(off[-1])]


def descriptor_distance(a, b) -> int:
    """popcount(a ^ b) of two 32-byte descriptors (liborbfe host popcount: one pair does not pay a device
    round trip)."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    if a.size != 32 or b.size != 32:
        raise ValueError("descriptors must be 32 bytes")
    out = C.c_int32()
    _lib.check("orbfe_descriptor_distance", _lib.lib().orbfe_descriptor_distance(a.ctypes.data, b.ctypes.data,
                                                                               C.byref(out)))
    return out.value


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
    b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
    out = np.zeros((len(a), len(b)), np.int32)
    if len(a) and len(b):
        call("orbfe_hamming_matrix", _h(), ptr(a), len(a), ptr(b), len(b), ptr(out))
    return out


# ---------------------------------------------------------------------------------------- grid queries
# Frame.get_features_in_area (Frame.py:373-416) for all the queries of a search at once (orbfe_grid_query,
# host code in liborbfe).  Used when every operand is a double (Python float, np.float64, or a 1-element
# float64 array — the types the reference's tracking loop produces); any other operand type (a float32
# projection evaluates in float32 under NumPy 2's promotion rules) goes through the frame's own method.
_grid_cache = weakref.WeakKeyDictionary()
_F64 = (float, np.float64)


def _is_f64(v) -> bool:
    return type(v) in _F64 or (type(v) is np.ndarray and v.dtype == np.float64 and v.size == 1)


_DTYPE, _SIZE, _SHAPE = operator.attrgetter("dtype"), operator.attrgetter("size"), operator.attrgetter("shape")
_F64_DT = np.dtype(np.float64)


def _f64_array(vals: list):
    """vals as a float64 array when every element is a double in _is_f64's sense (Python float, np.float64, or
    a size-1 float64 ndarray: the values are taken exactly), else None.  The type checks run as map() over
    C-level callables, not per element in Python (the tracking searches pass ~1 000 projections each)."""
    n = len(vals)
    if n == 0:
        return np.zeros(0, np.float64)
    kinds = set(map(type, vals))
    if kinds <= _F64_SET:
        return np.array(vals, np.float64)
    if kinds == _NDARRAY_SET and set(map(_DTYPE, vals)) == {_F64_DT} and set(map(_SIZE, vals)) == {1}:
        if len(set(map(_SHAPE, vals))) == 1:  # one shape: a single (n, 1[, 1]) float64 array
            return np.array(vals, np.float64).reshape(n)
        return np.fromiter((v.item() for v in vals), np.float64, count=n)
    if all(_is_f64(v) for v in vals):  # a mix of the kinds above
        return np.fromiter((v.item() if type(v) is np.ndarray else v for v in vals), np.float64, count=n)
    return None


_F64_SET = frozenset(_F64)
_NDARRAY_SET = frozenset((np.ndarray,))
_INT_SET = frozenset((int, np.int64, np.int32))
_U8_DT = np.dtype(np.uint8)
_UR_SET = frozenset((int, float, np.float32, np.float64))
_DOUBLE_OR_INT_SET = frozenset((float, int, np.float64))
_ANGLE = operator.attrgetter("angle")
_OBSERVATIONS = operator.methodcaller("observations")
_IN_VIEW = operator.attrgetter("mbTrackInView")
_IS_BAD = operator.methodcaller("is_bad")
_VIEW_COS = operator.attrgetter("mTrackViewCos")
_TRACK_LEVEL = operator.attrgetter("mnTrackScaleLevel")
_PROJ_X = operator.attrgetter("mTrackProjX")
_PROJ_Y = operator.attrgetter("mTrackProjY")
_PROJ_XR = operator.attrgetter("mTrackProjXR")
_WORLD_POS = operator.methodcaller("get_world_pos")
_DESCRIPTOR = operator.methodcaller("get_descriptor")


def _frame_grid(frame):
    """(cell_off, cell_idx, kp_x, kp_y, kp_oct, frame4) of a frame, cached while its grid / keypoints are
    the same objects; None if the frame's grid parameters are not plain doubles."""
    try:
        ent = _grid_cache.get(frame)
    except TypeError:
        return None
    key = (id(frame.mGrid), id(frame.mvKeysUn), frame.N)
    if ent is not None and ent[0] == key:
        return ent[1]
    f4 = (frame.mnMinX, frame.mnMinY, frame.mfGridElementWidthInv, frame.mfGridElementHeightInv)
    if not all(type(v) in _F64 for v in f4):
        return None
    cols, rows = frame.FRAME_GRID_COLS, frame.FRAME_GRID_ROWS
    csr = getattr(frame, "_orbfe_grid", None)  # left by frame.assign_features_to_grid for this mGrid
    if csr is not None and csr[0] == id(frame.mGrid) and len(csr[1]) == cols * rows + 1:
        off, idx = csr[1], csr[2]
    else:
        sizes = np.fromiter((len(frame.mGrid[ix][iy]) for ix in range(cols) for iy in range(rows)), np.int32,
                            count=cols * rows)
        off = np.zeros(cols * rows + 1, np.int32)
        np.cumsum(sizes, out=off[1:])
        idx = np.fromiter((g for col in frame.mGrid for cell in col for g in cell), np.int32, count=int(off[-1]))
    kps = frame.mvKeysUn
    pts = getattr(frame, "_orbfe_pts", None)  # left by frame.assign_features_to_grid: (mvKeys, (N, 2) f64)
    if pts is not None and pts[0] is kps and kps is frame.mvKeys and len(pts[1]) == len(kps):
        kx, ky = np.ascontiguousarray(pts[1][:, 0]), np.ascontiguousarray(pts[1][:, 1])
        ko = _octaves(frame)
    else:
        kx = np.fromiter((k.pt[0] for k in kps), np.float64, count=len(kps))
        ky = np.fromiter((k.pt[1] for k in kps), np.float64, count=len(kps))
        ko = np.fromiter((k.octave for k in kps), np.int32, count=len(kps))
    grid = (off, idx, kx, ky, ko, np.array(f4, np.float64), cols, rows)
    _grid_cache[frame] = (key, grid)
    return grid


_octave_cache = weakref.WeakKeyDictionary()


def _octaves(frame) -> np.ndarray:
    """frame.mvKeys[i].octave as an int32 array, cached while mvKeys is the same list of the same length."""
    kps = frame.mvKeys
    key = (id(kps), len(kps))
    try:
        ent = _octave_cache.get(frame)
    except TypeError:
        ent = None
    if ent is not None and ent[0] == key:
        return ent[1]
    kxy = getattr(frame, "_orbfe_kxy", None)  # frame.extract_orb's copy of the fields mvKeys was built from
    if kxy is not None and kxy[0] is kps and len(kxy[2]) == len(kps) and _kp_field_ok(kps, kxy[2], "octave", int):
        arr = kxy[2]
    else:
        arr = np.fromiter((k.octave for k in kps), np.int32, count=len(kps))
    try:
        _octave_cache[frame] = (key, arr)
    except TypeError:
        pass
    return arr


_angle_cache = weakref.WeakKeyDictionary()


def _kp_field_ok(kps, arr, name, typ) -> bool:
    """The KeyPoint class kept the extractor's values as given (spot check of the first and last keypoint:
    the type and the value of field `name`), so the extractor's array stands for the KeyPoints' fields."""
    if len(kps) == 0:
        return True
    a, b = getattr(kps[0], name), getattr(kps[-1], name)
    return type(a) is typ and type(b) is typ and a == arr[0] and b == arr[-1]


def _angles(frame):
    """mvKeysUn[i].angle as doubles (the rotation histogram's input), cached per keypoint list; None when
    an angle is not a double (a float32 angle would make the reference's subtraction float32)."""
    kps = frame.mvKeysUn
    key = (id(kps), len(kps))
    try:
        ent = _angle_cache.get(frame)
    except TypeError:
        ent = None
    if ent is not None and ent[0] == key:
        return ent[1]
    arr = None
    kxy = getattr(frame, "_orbfe_kxy", None)
    if kxy is not None and kxy[0] is kps and len(kxy[3]) == len(kps) and _kp_field_ok(kps, kxy[3], "angle", float):
        arr = kxy[3]  # the KeyPoints' angles are the Python floats of these float32 values
    else:
        angles = list(map(_ANGLE, kps))
        if set(map(type, angles)) <= _F64_SET:
            arr = np.array(angles, np.float64)
    try:
        _angle_cache[frame] = (key, arr)
    except TypeError:
        pass
    return arr


def _grid_csr(frame, grid, qx, qy, qr, lo, hi):
    """orbfe_grid_query over float64 / int32 query arrays: (out_off, out_idx) as int32 arrays."""
    off, idx, kx, ky, ko, f4, cols, rows = grid
    qx, qy, qr = (np.ascontiguousarray(a, np.float64) for a in (qx, qy, qr))
    lo, hi = np.ascontiguousarray(lo, np.int32), np.ascontiguousarray(hi, np.int32)
    n = len(qx)
    out_off = np.zeros(n + 1, np.int32)
    cap = max(64 * n, 1)
    while True:
        out = np.empty(cap, np.int32)
        rc = _lib.lib().orbfe_grid_query(ptr(off), ptr(idx), cols, rows, ptr(kx), ptr(ky), ptr(ko), len(kx), ptr(f4), n,
                                         ptr(qx), ptr(qy), ptr(qr), ptr(lo), ptr(hi), ptr(out_off), ptr(out), cap)
        if rc == _lib.ORBFE_ECAPACITY:
            cap = int(out_off[-1])
            continue
        _lib.check("orbfe_grid_query", rc)
        return out_off, out[:int(out_off[-1])]


def features_in_areas(frame, queries) -> list:
    """[frame.get_features_in_area(x, y, r, lo, hi) for (x, y, r, lo, hi) in queries], batched."""
    if not queries:
        return []
    grid = _frame_grid(frame)
    fast = grid is not None and all(_is_f64(x) and _is_f64(y) and _is_f64(r) for x, y, r, _, _ in queries)
    if not fast:
        return [frame.get_features_in_area(*q) for q in queries]
    n = len(queries)
    qx = np.fromiter((q[0].item() if type(q[0]) is np.ndarray else q[0] for q in queries), np.float64, count=n)
    qy = np.fromiter((q[1].item() if type(q[1]) is np.ndarray else q[1] for q in queries), np.float64, count=n)
    qr = np.fromiter((q[2].item() if type(q[2]) is np.ndarray else q[2] for q in queries), np.float64, count=n)
    lo = np.fromiter((q[3] for q in queries), np.int32, count=n)
    hi = np.fromiter((q[4] for q in queries), np.int32, count=n)
    out_off, out = _grid_csr(frame, grid, qx, qy, qr, lo, hi)
    o = out_off.tolist()
    flat = out.tolist()
    return [flat[o[i]:o[i + 1]] for i in range(n)]


# Per-frame inputs of the native candidate selection: mvuRight as doubles (set once by the Frame
# constructor), and which slots hold a map point with observations (read fresh per search).
_uright_cache = weakref.WeakKeyDictionary()


def _u_right(frame, with_kinds: bool = False):
    """frame.mvuRight widened to a float64 array (cached while the list is the same object); with_kinds
    also returns whether every entry is already a double (Python float / int or np.float64), i.e. whether
    `python_float - mvuRight[i]` evaluates in double under NumPy 2's promotion rules (NEP 50: a Python
    float meeting an np.float32 stays float32)."""
    vals = frame.mvuRight
    try:
        ent = _uright_cache.get(frame)
    except TypeError:
        ent = None
    if ent is None or ent[0] != (id(vals), len(vals)):
        kinds = set(map(type, vals))
        if kinds <= _UR_SET:  # the values the drop-in's lists hold: -1, np.float32, Python float
            arr = np.array(vals, np.float64)  # each value widened exactly, as float(v)
        else:
            arr = np.fromiter((float(v) for v in vals), np.float64, count=len(vals))
        all_double = kinds <= _DOUBLE_OR_INT_SET
        ent = ((id(vals), len(vals)), arr, all_double)
        try:
            _uright_cache[frame] = ent
        except TypeError:
            pass
    return (ent[1], ent[2]) if with_kinds else ent[1]


def prime_u_right(frame, res: dict, xs: np.ndarray) -> None:
    """Fill _u_right's cache for a frame whose mvuRight list compute_stereo_matches has just built from the
    stereo arrays (frame.to_reference_lists): the same doubles, from the arrays instead of the 2 000-entry
    list — u_right widened where status is 1, -1 where 0, float(x) - 0.01 where 2 (Frame.py:273-277)."""
    vals = frame.mvuRight
    st = np.asarray(res["status"])
    if len(vals) != len(st):
        return
    arr = np.asarray(res["u_right"], np.float32).astype(np.float64)
    arr[st == 0] = -1.0
    z = st == 2
    if z.any():
        arr[z] = np.asarray(xs, np.float32)[z].astype(np.float64) - 0.01
    # np.float32 entries (status 1) are not doubles; -1 (int) and the status-2 Python floats are
    all_double = not bool(((st != 0) & (st != 2)).any())
    try:
        _uright_cache[frame] = ((id(vals), len(vals)), arr, all_double)
    except TypeError:
        pass


def _blocked(frame):
    """Per slot of the frame: 1 if it holds a map point with observations (ORBMatcher.py's
    `if mvpMapPoints[i]: if mvpMapPoints[i].observations() > 0: continue`)."""
    mps = frame.mvpMapPoints
    n = len(mps)
    out = np.zeros(n, np.uint8)
    if mps.count(None) == n:
        return out
    held = np.flatnonzero(np.fromiter(map(operator.is_not, mps, repeat(None, n)), bool, count=n))
    hl = held.tolist()
    out[held] = _obs_flags([mps[i] for i in hl])
    return out


def _obs_flags(mps) -> np.ndarray:
    """1 per map point that is truthy and has observations() > 0."""
    if all(mps):
        obs = list(map(_OBSERVATIONS, mps))
        if set(map(type, obs)) <= _INT_SET:
            return (np.array(obs, np.int64) > 0).astype(np.uint8)
    return np.fromiter((1 if (m and m.observations() > 0) else 0 for m in mps), np.uint8, count=len(mps))


def _descriptor_rows(descs: list) -> np.ndarray:
    """(n, 32) u8 array of n map-point descriptors (one array copy when they are all 32-byte u8 arrays)."""
    if (set(map(type, descs)) == _NDARRAY_SET and set(map(_DTYPE, descs)) == {_U8_DT}
            and set(map(_SIZE, descs)) == {32} and len(set(map(_SHAPE, descs))) == 1):
        return np.concatenate(descs).reshape(len(descs), 32)
    return np.stack([np.asarray(d, np.uint8).reshape(32) for d in descs])


class ORBMatcher:
    def __init__(self, nnratio=1, checkOri=True):
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri

    # ORBMatcher.py:12-14 (one pair, on the host in liborbfe; use descriptor_distances / hamming_* for batches)
    def descriptor_distance(self, a, b):
        return descriptor_distance(a, b)

    def descriptor_distances(self, A, B):
        return hamming_matrix(A, B)

    def compute_three_maxima(self, histo, histo_length):
        histo_counts = [len(h) for h in histo]
        return np.argsort(histo_counts)[::-1][:3]

    def radius_by_viewing_cos(self, view_cos):
        return 2.5 if view_cos > 0.998 else 4.0

    @staticmethod
    def _csr(qd, train, off, idx):
        """The one device call of a search: distances of CSR (query, candidate) pairs."""
        return hamming_csr(qd, train, off, idx)

    @classmethod
    def _batched(cls, queries, train):
        """queries: list of (descriptor, candidate list) -> list of distance arrays."""
        off = np.zeros(len(queries) + 1, np.int32)
        for i, (_, c) in enumerate(queries):
            off[i + 1] = off[i] + len(c)
        if not queries or off[-1] == 0:
            return [np.zeros(0, np.int32) for _ in queries]
        qd = np.stack([np.asarray(d, np.uint8).reshape(32) for d, _ in queries])
        idx = np.concatenate([np.asarray(c, np.int32) for _, c in queries])
        dist = cls._csr(qd, train, off, idx)
        return [dist[off[i]:off[i + 1]] for i in range(len(queries))]

    def _nonempty(self, off, idx, pmps, train):
        """Restrict a CSR candidate set to its non-empty queries and get their distances: (rows, off, dist),
        rows = indices of the non-empty queries (the reference fetches a descriptor only for those)."""
        cnt = np.diff(off)
        rows = np.flatnonzero(cnt)
        off2 = np.zeros(len(rows) + 1, np.int32)
        np.cumsum(cnt[rows], out=off2[1:])
        if len(rows) == 0:
            return rows, off2, np.zeros(0, np.int32)
        qd = _descriptor_rows(list(map(_DESCRIPTOR, map(pmps.__getitem__, rows.tolist()))))
        return rows, off2, np.ascontiguousarray(self._csr(qd, train, off2, idx), np.int32)

    # ORBMatcher.py:215-283
    def _f_p_inputs(self, vp_map_points, th, b_factor):
        """The searched map points of search_by_projection_f_p (tracked in view, then not bad: the reference's
        two `continue`s in its order), their predicted levels and radii, with the per-point attribute reads
        and calls as map() over C-level getters.  The radius is ORBMatcher's own radius_by_viewing_cos
        evaluated over an array of doubles (`vc > 0.998` in double, then `r *= th`), or point by point when a
        view cosine is not a double (a float32 one compares in float32); None (run the reference loop) when
        the method is overridden or th is not a Python number."""
        if type(self).radius_by_viewing_cos is not ORBMatcher.radius_by_viewing_cos:
            return None
        if b_factor and type(th) not in (int, float):
            return None
        cand = list(compress(vp_map_points, map(_IN_VIEW, vp_map_points)))
        pmps = list(compress(cand, map(operator.not_, map(_IS_BAD, cand))))
        cos = list(map(_VIEW_COS, pmps))
        vc = _f64_array(cos)
        if vc is None:
            # not all doubles: the reference's per-point radius on the points already selected (no
            # second mbTrackInView / is_bad() pass through the reference loop)
            radius = self.radius_by_viewing_cos
            rads = []
            for c in cos:
                r = radius(c)
                if b_factor:
                    r *= th
                rads.append(r)
            return pmps, list(map(_TRACK_LEVEL, pmps)), rads
        r = np.where(vc > 0.998, 2.5, 4.0)
        if b_factor:
            r = r * th
        return pmps, list(map(_TRACK_LEVEL, pmps)), r.tolist()

    def search_by_projection_f_p(self, frame, vp_map_points, th):
        n_matches = 0
        b_factor = th != 1.0
        radius = self.radius_by_viewing_cos
        pre = self._f_p_inputs(vp_map_points, th, b_factor) if isinstance(vp_map_points, (list, tuple)) else None
        if pre is not None:
            pmps, lvls, rads = pre
        else:
            pmps, lvls, rads = [], [], []
            for pMP in vp_map_points:
                if not pMP.mbTrackInView:
                    continue
                if pMP.is_bad():
                    continue
                r = radius(pMP.mTrackViewCos)
                if b_factor:
                    r *= th
                pmps.append(pMP)
                lvls.append(pMP.mnTrackScaleLevel)
                rads.append(r)
        done = self._f_p_native(frame, pmps, lvls, rads)
        if done is not None:
            return done
        sf = frame.mvScaleFactors
        pend = list(zip(pmps, lvls, rads))
        queries = [(p.mTrackProjX, p.mTrackProjY, r * sf[lv], lv - 1, lv) for p, lv, r in pend]
        work = [(pMP, lvl, r, v_indices, pMP.get_descriptor())
                for (pMP, lvl, r), v_indices in zip(pend, features_in_areas(frame, queries)) if v_indices]
        dists = self._batched([(w[4], w[3]) for w in work], frame.mDescriptors)
        for (pMP, n_predicted_level, r, v_indices, _), dq in zip(work, dists):
            best_dist = 256
            best_level = -1
            best_dist2 = 256
            best_level2 = -1
            best_idx = -1
            for idx, dist in zip(v_indices, dq.tolist()):
                if frame.mvpMapPoints[idx]:
                    if frame.mvpMapPoints[idx].observations() > 0:
                        continue
                if frame.mvuRight[idx] > 0:
                    er = abs(pMP.mTrackProjXR - frame.mvuRight[idx])
                    if er > r * frame.mvScaleFactors[n_predicted_level]:
                        continue
                if dist < best_dist:
                    best_dist2 = best_dist
                    best_dist = dist
                    best_level2 = best_level
                    best_level = frame.mvKeysUn[idx].octave
                    best_idx = idx
                elif dist < best_dist2:
                    best_level2 = frame.mvKeysUn[idx].octave
                    best_dist2 = dist
            if best_dist <= TH_HIGH:
                if best_level == best_level2 and best_dist > self.mfNNratio * best_dist2:
                    continue
                frame.mvpMapPoints[best_idx] = pMP
                n_matches += 1
        return n_matches

    # ORBMatcher.py:291-393
    def search_by_projection_f_f(self, current_frame, last_frame, th):
        n_matches = 0
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        Rcw = current_frame.mTcw[:3, :3]
        tcw = current_frame.mTcw[:3, 3:4]
        twc = -Rcw.T @ tcw
        Rlw = last_frame.mTcw[:3, :3]
        tlw = last_frame.mTcw[:3, 3:4]
        tlc = Rlw @ twc + tlw
        b_forward = tlc[2] > current_frame.mb
        b_backward = -tlc[2] > current_frame.mb
        # projection of every usable map point of the last frame (one stacked matmul: the same per-point
        # BLAS product as `Rcw @ x3Dw`, element-wise arithmetic in the reference's order and dtypes)
        lmps, lout, n_last = last_frame.mvpMapPoints, last_frame.mvbOutlier, last_frame.N
        if len(lmps) >= n_last and len(lout) >= n_last:
            # [i for i in range(n_last) if lmps[i] and not lout[i]] with C-level iteration (bool(m): the
            # truth test `if m` makes; `not lout[i]` only where lmps[i] is true, as the reference's `and`)
            live = list(compress(range(n_last), map(bool, lmps)))
            cand = list(compress(live, map(operator.not_, map(lout.__getitem__, live))))
        else:  # the reference's indexing (and its IndexError)
            cand = [i for i in range(n_last) if lmps[i] and not lout[i]]
        pos = list(map(_WORLD_POS, map(lmps.__getitem__, cand)))
        proj = []
        if (pos and set(map(type, pos)) == _NDARRAY_SET and set(map(_SHAPE, pos)) == {(3, 1)}
                and len(set(map(_DTYPE, pos))) == 1):
            x3Dc = Rcw @ np.concatenate(pos).reshape(len(pos), 3, 1) + tcw  # np.stack(pos), 3x faster
            zc = x3Dc[:, 2, 0]
            invzc = 1.0 / zc
            u = current_frame.fx * x3Dc[:, 0, 0] * invzc + current_frame.cx
            v = current_frame.fy * x3Dc[:, 1, 0] * invzc + current_frame.cy
            keep = ~((invzc < 0) | (u < current_frame.mnMinX) | (u > current_frame.mnMaxX) |
                     (v < current_frame.mnMinY) | (v > current_frame.mnMaxY))
            sel = np.flatnonzero(keep)
            done = self._f_f_native(current_frame, last_frame, th, b_forward, b_backward, cand, sel, u, v, invzc)
            if done is not None:
                return done
            proj = [(cand[k], u[k], v[k], invzc[k]) for k in sel.tolist()]
        else:
            for i, x3Dw in zip(cand, pos):
                x3Dc = Rcw @ x3Dw + tcw
                xc, yc, zc = x3Dc[0][0], x3Dc[1][0], x3Dc[2][0]
                invzc = 1.0 / zc
                if invzc < 0:
                    continue
                u = current_frame.fx * xc * invzc + current_frame.cx
                v = current_frame.fy * yc * invzc + current_frame.cy
                if u < current_frame.mnMinX or u > current_frame.mnMaxX:
                    continue
                if v < current_frame.mnMinY or v > current_frame.mnMaxY:
                    continue
                proj.append((i, u, v, invzc))
        queries, pend = [], []
        for i, u, v, invzc in proj:
            n_last_octave = last_frame.mvKeys[i].octave
            radius = th * current_frame.mvScaleFactors[n_last_octave]
            if b_forward:
                queries.append((u, v, radius, n_last_octave, -1))
            elif b_backward:
                queries.append((u, v, radius, 0, n_last_octave))
            else:
                queries.append((u, v, radius, n_last_octave - 1, n_last_octave + 1))
            pend.append((i, u, invzc, radius))
        work = []
        for (i, u, invzc, radius), v_indices2 in zip(pend, features_in_areas(current_frame, queries)):
            if not v_indices2:
                continue
            pMP = last_frame.mvpMapPoints[i]
            work.append((i, pMP, u, invzc, radius, v_indices2, pMP.get_descriptor()))
        dists = self._batched([(w[6], w[5]) for w in work], current_frame.mDescriptors)
        for (i, pMP, u, invzc, radius, v_indices2, _), dq in zip(work, dists):
            best_dist = 256
            best_idx2 = -1
            for i2, dist in zip(v_indices2, dq.tolist()):
                if current_frame.mvpMapPoints[i2]:
                    if current_frame.mvpMapPoints[i2].observations() > 0:
                        continue
                if current_frame.mvuRight[i2] > 0:
                    ur = u - current_frame.mbf * invzc
                    er = abs(ur - current_frame.mvuRight[i2])
                    if er > radius:
                        continue
                if dist < best_dist:
                    best_dist = dist
                    best_idx2 = i2
            if best_dist <= TH_HIGH:
                current_frame.mvpMapPoints[best_idx2] = pMP
                n_matches += 1
                if self.mbCheckOrientation:
                    rot = last_frame.mvKeysUn[i].angle - current_frame.mvKeysUn[best_idx2].angle
                    if rot < 0.0:
                        rot += 360.0
                    bin_idx = round(rot * factor)
                    if bin_idx == HISTO_LENGTH:
                        bin_idx = 0
                    assert 0 <= bin_idx < HISTO_LENGTH
                    rot_hist[bin_idx].append(best_idx2)
        if self.mbCheckOrientation:
            ind1, ind2, ind3 = self.compute_three_maxima(rot_hist, HISTO_LENGTH)
            for i in range(HISTO_LENGTH):
                if i not in (ind1, ind2, ind3):
                    for idx in rot_hist[i]:
                        current_frame.mvpMapPoints[idx] = None
                        n_matches -= 1
        return n_matches

    # ------------------------------------------------------------------------------------------------
    # native selection of the two tracking searches (orbfe_select_f_p / _f_f, host code) when every value
    # the reference's loop compares is a double: grid query -> distances of the non-empty queries -> the
    # sequential selection in C -> the assignments (and f_f's rotation histogram) here, in order.  Returns
    # None, before touching anything, when an operand has another type (float32 projections promote
    # differently under NumPy 2): the caller then runs the Python loop.

    def _f_p_native(self, frame, pmps, lvls, rads):
        """pmps / lvls / rads: the searched map points (tracked in view, not bad), their predicted levels and
        radii; the window of each is (mTrackProjX, mTrackProjY, r * mvScaleFactors[level], level - 1,
        level) as in the reference loop."""
        grid = _frame_grid(frame)
        if grid is None or not pmps:
            return None
        if not (set(map(type, lvls)) <= _INT_SET and set(map(type, rads)) <= _F64_SET):
            return None
        sf = frame.mvScaleFactors
        if not set(map(type, sf)) <= _F64_SET:
            return None
        n = len(pmps)
        lo_hi = np.array(lvls, np.int64)
        if lo_hi.min() < -len(sf) or lo_hi.max() >= len(sf):
            return None
        qr = np.array(rads, np.float64) * np.array(sf, np.float64)[lo_hi]  # r * mvScaleFactors[level], doubles
        qx = _f64_array(list(map(_PROJ_X, pmps)))
        if qx is None:
            return None
        qy = _f64_array(list(map(_PROJ_Y, pmps)))
        if qy is None:
            return None
        xr_all = list(map(_PROJ_XR, pmps))
        xr_arr = _f64_array(xr_all)
        if xr_arr is None:
            return None
        n_frame = len(frame.mvpMapPoints)
        u_right, u_double = _u_right(frame, with_kinds=True)
        # ORBMatcher.py's er = abs(XR - mvuRight[idx]): a Python-float XR against an np.float32 entry
        # evaluates in float32 (NEP 50), which the double selection in C does not reproduce
        if not u_double and float in set(map(type, xr_all)):
            return None
        if len(u_right) != n_frame or len(grid[4]) != n_frame:
            return None
        lv32 = lo_hi.astype(np.int32)
        off, idx = _grid_csr(frame, grid, qx, qy, qr, lv32 - 1, lv32)
        rows, off2, dist = self._nonempty(off, idx, pmps, frame.mDescriptors)
        if len(rows) == 0:
            return 0
        rl = rows.tolist()
        xr = np.ascontiguousarray(xr_arr[rows])
        rs = np.ascontiguousarray(qr[rows])
        q_obs = _obs_flags(list(map(pmps.__getitem__, rl)))
        blocked = _blocked(frame)
        best = np.empty(len(rl), np.int32)
        call("orbfe_select_f_p", len(rl), ptr(off2), ptr(idx), ptr(dist), ptr(xr), ptr(rs), ptr(grid[4]), ptr(q_obs),
             ptr(u_right), ptr(blocked), n_frame, float(self.mfNNratio), TH_HIGH, ptr(best))
        hit = np.flatnonzero(best >= 0).tolist()
        # frame.mvpMapPoints[best[j]] = pmps[rl[j]] in query order, the list's own __setitem__ mapped in C
        deque(map(frame.mvpMapPoints.__setitem__, best[hit].tolist(), map(pmps.__getitem__, map(rl.__getitem__, hit))), 0)
        return len(hit)

    def _f_f_native(self, cur, last, th, b_forward, b_backward, cand, sel, u, v, invzc):
        grid = _frame_grid(cur)
        if grid is None or type(th) not in (int, float):
            return None
        if not (u.dtype == np.float64 and v.dtype == np.float64 and invzc.dtype == np.float64):
            return None
        sf = cur.mvScaleFactors
        if not all(type(x) in _F64 for x in sf):
            return None
        n_frame = len(cur.mvpMapPoints)
        u_right = _u_right(cur)
        if len(u_right) != n_frame:
            return None
        ci = np.asarray(cand, np.int64)[sel].tolist()
        octv = _octaves(last)[np.asarray(ci, np.int64)] if ci else np.zeros(0, np.int32)
        radius = th * np.asarray(sf, np.float64)[octv]  # th * mvScaleFactors[octave], one double product each
        if b_forward:
            lo, hi = octv, np.full(len(ci), -1, np.int32)
        elif b_backward:
            lo, hi = np.zeros(len(ci), np.int32), octv
        else:
            lo, hi = octv - 1, octv + 1
        qx, iz = np.ascontiguousarray(u[sel]), np.ascontiguousarray(invzc[sel])
        off, idx = _grid_csr(cur, grid, qx, v[sel], radius, lo, hi)
        pmps = list(map(last.mvpMapPoints.__getitem__, ci))
        rows, off2, dist = self._nonempty(off, idx, pmps, cur.mDescriptors)
        n_matches = 0
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        if len(rows):
            rl = rows.tolist()
            q_obs = _obs_flags(list(map(pmps.__getitem__, rl)))
            blocked = _blocked(cur)
            best = np.empty(len(rl), np.int32)
            qu, qz, qrad = (np.ascontiguousarray(a[rows], np.float64) for a in (qx, iz, radius))  # held across the call
            call("orbfe_select_f_f", len(rl), ptr(off2), ptr(idx), ptr(dist), ptr(qu), ptr(qz), ptr(qrad), ptr(q_obs),
                 ptr(u_right), ptr(blocked), n_frame, float(cur.mbf), TH_HIGH, ptr(best))
            hit = np.flatnonzero(best >= 0)
            bl = best[hit].tolist()
            # cur.mvpMapPoints[b] = pmps[rl[j]] in query order, the list's own __setitem__ mapped in C
            deque(map(cur.mvpMapPoints.__setitem__, bl, map(pmps.__getitem__, map(rl.__getitem__, hit.tolist()))), 0)
            n_matches += len(bl)
            if self.mbCheckOrientation and bl:  # ORBMatcher.py:374-382
                la, ca = _angles(last), _angles(cur)
                if la is not None and ca is not None:  # doubles: the same arithmetic over arrays
                    rot = la[np.asarray(ci, np.int64)[rows[hit]]] - ca[best[hit]]
                    rot = np.where(rot < 0.0, rot + 360.0, rot)
                    bins = np.round(rot * factor).astype(np.int64)  # round() of a double: half to even
                    bins[bins == HISTO_LENGTH] = 0
                    bins = bins.tolist()
                else:
                    bins = []
                    for j, b in zip(hit.tolist(), bl):
                        rot = last.mvKeysUn[ci[rl[j]]].angle - cur.mvKeysUn[b].angle
                        if rot < 0.0:
                            rot += 360.0
                        bin_idx = round(rot * factor)
                        bins.append(0 if bin_idx == HISTO_LENGTH else bin_idx)
                assert not bins or 0 <= min(bins) <= max(bins) < HISTO_LENGTH  # ORBMatcher.py's per-bin assert
                for b, k in zip(bl, bins):
                    rot_hist[k].append(b)
        if self.mbCheckOrientation:
            ind1, ind2, ind3 = self.compute_three_maxima(rot_hist, HISTO_LENGTH)
            for i in range(HISTO_LENGTH):
                if i not in (ind1, ind2, ind3):
                    for idx2 in rot_hist[i]:
                        cur.mvpMapPoints[idx2] = None
                        n_matches -= 1
        return n_matches

    # ------------------------------------------------------------------------------------------------
    # helpers shared by the keyframe-level searches

    def _reject_by_rotation(self, rot_hist, on_reject):
        """Keep the three fullest rotation bins (ORBMatcher.py:16-19 + the callers' loops)."""
        ind1, ind2, ind3 = self.compute_three_maxima(rot_hist, HISTO_LENGTH)
        n = 0
        for i in range(HISTO_LENGTH):
            if i in [ind1, ind2, ind3]:
                continue
            for idx in rot_hist[i]:
                on_reject(idx)
                n += 1
        return n

    @staticmethod
    def _bow_common_nodes(fv1, fv2):
        """Nodes present in both DBoW2 feature vectors, in the order the reference's merge walk visits
        them (ORBMatcher.py:39-103, 140-196: advance both on equal keys, else the smaller one)."""
        out = []
        it1, it2 = iter(fv1), iter(fv2)
        try:
            k1 = next(it1)
            k2 = next(it2)
            while True:
                if k1 == k2:
                    out.append(k1)
                    k1 = next(it1)
                    k2 = next(it2)
                elif k1 < k2:
                    k1 = next(it1)
                else:
                    k2 = next(it2)
        except StopIteration:
            pass
        return out

    def _query_dists(self, pMP, snap, cands, dq, train):
        """Distances of a query collected earlier; re-run on the GPU if its descriptor changed since."""
        d = pMP.get_descriptor()
        if np.array_equal(np.asarray(d).reshape(-1), np.asarray(snap).reshape(-1)):
            return dq
        return self._batched([(d, cands)], train)[0]

    # ORBMatcher.py:21-118
    def search_by_BoW_kf_f(self, kf, frame):
        vpMapPointsKF = kf.get_map_point_matches()
        vpMapPointMatches = [None] * frame.N
        fv_kf, fv_f = kf.mFeatVec, frame.mFeatVec
        n_matches = 0
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        work = []
        for node in self._bow_common_nodes(fv_kf, fv_f):
            cands = fv_f[node]
            for idx_kf in fv_kf[node]:
                pMP = vpMapPointsKF[idx_kf]
                if not pMP or pMP.is_bad():
                    continue
                work.append((idx_kf, pMP, cands, kf.mDescriptors[idx_kf]))
        dists = self._batched([(w[3], w[2]) for w in work], frame.mDescriptors)
        for (idx_kf, pMP, cands, _), dq in zip(work, dists):
            best1, best_idx, best2 = 256, -1, 256
            for idx_f, dist in zip(cands, dq.tolist()):
                if vpMapPointMatches[idx_f]:
                    continue
                if dist < best1:
                    best2 = best1
                    best1 = dist
                    best_idx = idx_f
                elif dist < best2:
                    best2 = dist
            if best1 <= TH_LOW and float(best1) < self.mfNNratio * float(best2):
                vpMapPointMatches[best_idx] = pMP
                kp = kf.mvKeysUn[idx_kf]
                if self.mbCheckOrientation:
                    rot = kp.angle - frame.mvKeys[best_idx].angle
                    if rot < 0.0:
                        rot += 360.0
                    b = round(rot * factor)
                    if b == HISTO_LENGTH:
                        b = 0
                    assert 0 <= b < HISTO_LENGTH
                    rot_hist[b].append(best_idx)
                n_matches += 1
        if self.mbCheckOrientation:
            n_matches -= self._reject_by_rotation(rot_hist, lambda i: vpMapPointMatches.__setitem__(i, None))
        return n_matches, vpMapPointMatches

    # ORBMatcher.py:120-213
    def search_by_BoW_kf_kf(self, pKF1, pKF2):
        vKeysUn1, vKeysUn2 = pKF1.mvKeysUn, pKF2.mvKeysUn
        fv1, fv2 = pKF1.mFeatVec, pKF2.mFeatVec
        vpMapPoints1 = pKF1.get_map_point_matches()
        vpMapPoints2 = pKF2.get_map_point_matches()
        vpMatches12 = [None] * len(vpMapPoints1)
        vbMatched2 = [False] * len(vpMapPoints2)
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        n_matches = 0
        work = []
        for node in self._bow_common_nodes(fv1, fv2):
            cands = []
            for idx2 in fv2[node]:
                pMP2 = vpMapPoints2[idx2]
                if not pMP2 or pMP2.is_bad():
                    continue
                cands.append(idx2)
            for idx1 in fv1[node]:
                pMP1 = vpMapPoints1[idx1]
                if not pMP1 or pMP1.is_bad():
                    continue
                work.append((idx1, cands, pKF1.mDescriptors[idx1]))
        dists = self._batched([(w[2], w[1]) for w in work], pKF2.mDescriptors)
        for (idx1, cands, _), dq in zip(work, dists):
            best1, best_idx2, best2 = 256, -1, 256
            for idx2, dist in zip(cands, dq.tolist()):
                if vbMatched2[idx2]:
                    continue
                if dist < best1:
                    best2 = best1
                    best1 = dist
                    best_idx2 = idx2
                elif dist < best2:
                    best2 = dist
            if best1 < TH_LOW and best1 < self.mfNNratio * best2:
                vpMatches12[idx1] = vpMapPoints2[best_idx2]
                vbMatched2[best_idx2] = True
                if self.mbCheckOrientation:
                    rot = vKeysUn1[idx1].angle - vKeysUn2[best_idx2].angle
                    if rot < 0.0:
                        rot += 360.0
                    b = round(rot * factor)
                    if b == HISTO_LENGTH:
                        b = 0
                    rot_hist[b].append(idx1)
                n_matches += 1
        if self.mbCheckOrientation:
            n_matches -= self._reject_by_rotation(rot_hist, lambda i: vpMatches12.__setitem__(i, None))
        return n_matches, vpMatches12

    @staticmethod
    def _sim3_to_pose(Scw):
        sRcw = Scw[:3, :3]
        scw = np.sqrt(np.dot(sRcw[0], sRcw[0]))
        Rcw = sRcw / scw
        tcw = Scw[:3, 3:4] / scw
        return Rcw, tcw, -Rcw.T @ tcw

    @staticmethod
    def _project_checked(pMP, pKF, Rcw, tcw, strict_z):
        """Camera projection of fuse_kf_scw_mp (:414-427, strict_z False) and
        search_by_projection_ckf_scw_mp (:868-878, strict_z True: `<= 0` and 1-element array
        arithmetic, as there).  Returns (u, v, invz, p3Dw) or None."""
        p3Dw = pMP.get_world_pos()
        p3Dc = Rcw @ p3Dw + tcw
        if strict_z:
            if p3Dc[2][0] <= 0.0:
                return None
            invz = 1.0 / p3Dc[2]
            x, y = p3Dc[0] * invz, p3Dc[1] * invz
        else:
            if p3Dc[2][0] < 0.0:
                return None
            invz = 1.0 / p3Dc[2][0]
            x = p3Dc[0][0] * invz
            y = p3Dc[1][0] * invz
        u = pKF.fx * x + pKF.cx
        v = pKF.fy * y + pKF.cy
        return u, v, invz, p3Dw

    @staticmethod
    def _distance_gates(pMP, pKF, p3Dw, Ow):
        """Scale-invariance distance and viewing-angle gates (:429-441); the predicted level or None."""
        maxDistance = pMP.get_max_distance_invariance()
        minDistance = pMP.get_min_distance_invariance()
        PO = p3Dw - Ow
        dist3D = np.linalg.norm(PO)
        if dist3D < minDistance or dist3D > maxDistance:
            return None
        Pn = pMP.get_normal()
        if np.dot(PO.T, Pn) < 0.5 * dist3D:
            return None
        return pMP.predict_scale(dist3D, pKF)

    # ORBMatcher.py:395-480
    def fuse_kf_scw_mp(self, pKF, Scw, vpPoints, th, vpReplacePoint):
        Rcw, tcw, Ow = self._sim3_to_pose(Scw)
        spAlreadyFound = pKF.get_map_points()
        work = []
        for iMP, pMP in enumerate(vpPoints):
            if pMP.is_bad() or pMP in spAlreadyFound:
                continue
            pr = self._project_checked(pMP, pKF, Rcw, tcw, False)
            if pr is None:
                continue
            u, v, _, p3Dw = pr
            if not pKF.is_in_image(u, v):
                continue
            lvl = self._distance_gates(pMP, pKF, p3Dw, Ow)
            if lvl is None:
                continue
            vIndices = pKF.get_features_in_area(u, v, th * pKF.mvScaleFactors[lvl])
            if not vIndices:
                continue
            cands = [i for i in vIndices if lvl - 1 <= pKF.mvKeysUn[i].octave <= lvl]
            work.append((iMP, pMP, cands, pMP.get_descriptor()))
        dists = self._batched([(w[3], w[2]) for w in work], pKF.mDescriptors)
        n_fused = 0
        for (iMP, pMP, cands, _), dq in zip(work, dists):
            best_dist, best_idx = float('inf'), -1
            for idx, dist in zip(cands, dq.tolist()):
                if dist < best_dist:
                    best_dist = dist
                    best_idx = idx
            if best_dist <= TH_LOW:
                pMPinKF = pKF.get_map_point(best_idx)
                if pMPinKF:
                    if not pMPinKF.is_bad():
                        vpReplacePoint[iMP] = pMPinKF
                else:
                    pMP.add_observation(pKF, best_idx)
                    pKF.add_map_point(pMP, best_idx)
                n_fused += 1
        return n_fused, vpReplacePoint

    # ORBMatcher.py:482-582
    def fuse_pkf_mp(self, pKF, vpMapPoints, th):
        fx, fy, cx, cy, bf = pKF.fx, pKF.fy, pKF.cx, pKF.cy, pKF.mbf
        Rcw = pKF.get_rotation()
        tcw = pKF.get_translation()
        Ow = pKF.get_camera_center()
        work = []
        for pMP in vpMapPoints:
            # badness never reverts, so a point bad now is skipped by the replay as well; whether it is in
            # the keyframe can change during the search and is checked there
            if not pMP or pMP.is_bad():
                continue
            p3Dw = pMP.get_world_pos()
            p3Dc = Rcw @ p3Dw + tcw
            if p3Dc[2][0] < 0.0:
                continue
            invz = 1.0 / p3Dc[2][0]
            x = p3Dc[0][0] * invz
            y = p3Dc[1][0] * invz
            u = fx * x + cx
            v = fy * y + cy
            ur = u - bf * invz
            if not pKF.is_in_image(u, v):
                continue
            lvl = self._distance_gates(pMP, pKF, p3Dw, Ow)
            if lvl is None:
                continue
            vIndices = pKF.get_features_in_area(u, v, th * pKF.mvScaleFactors[lvl])
            if not vIndices:
                continue
            cands = []
            for idx in vIndices:
                kp = pKF.mvKeysUn[idx]
                kpLevel = kp.octave
                if kpLevel < lvl - 1 or kpLevel > lvl:
                    continue
                if pKF.mvuRight[idx] >= 0:
                    ex, ey, er = u - kp.pt[0], v - kp.pt[1], ur - pKF.mvuRight[idx]
                    if (ex ** 2 + ey ** 2 + er ** 2) * pKF.mvInvLevelSigma2[kpLevel] > 7.8:
                        continue
                else:
                    ex, ey = u - kp.pt[0], v - kp.pt[1]
                    if (ex ** 2 + ey ** 2) * pKF.mvInvLevelSigma2[kpLevel] > 5.99:
                        continue
                cands.append(idx)
            work.append((pMP, cands, pMP.get_descriptor()))
        dists = self._batched([(w[2], w[1]) for w in work], pKF.mDescriptors)
        n_fused = 0
        for (pMP, cands, snap), dq in zip(work, dists):
            if pMP.is_bad() or pMP.is_in_key_frame(pKF):
                continue
            dq = self._query_dists(pMP, snap, cands, dq, pKF.mDescriptors)
            best_dist, best_idx = float('inf'), -1
            for idx, dist in zip(cands, dq.tolist()):
                if dist < best_dist:
                    best_dist = dist
                    best_idx = idx
            if best_dist <= TH_LOW:
                pMPinKF = pKF.get_map_point(best_idx)
                if pMPinKF:
                    if not pMPinKF.is_bad():
                        if pMPinKF.observations() > pMP.observations():
                            pMP.replace(pMPinKF)
                        else:
                            pMPinKF.replace(pMP)
                else:
                    pMP.add_observation(pKF, best_idx)
                    pKF.add_map_point(pMP, best_idx)
                n_fused += 1
        return n_fused

    @staticmethod
    def _triangulation_nodes(fv1, fv2):
        """The node pairs search_for_triangulation visits (ORBMatcher.py:606-675).  Its walk draws a
        fresh item from both vectors every round and, on unequal keys, discards one more item of the
        smaller side — outside the try block, so an exhausted vector there raises StopIteration out of
        the search.  Reproduced as is (the search has no side effects before that point)."""
        out = []
        it1, it2 = iter(fv1.items()), iter(fv2.items())
        while True:
            try:
                k1, v1 = next(it1)
                k2, v2 = next(it2)
            except StopIteration:
                break
            if k1 == k2:
                out.append((v1, v2))
            elif k1 < k2:
                next(it1)
            else:
                next(it2)
        return out

    # ORBMatcher.py:584-696
    def search_for_triangulation(self, pKF1, pKF2, F12, bOnlyStereo=False):
        Cw = pKF1.get_camera_center()
        R2w = pKF2.get_rotation()
        t2w = pKF2.get_translation()
        C2 = R2w @ Cw + t2w
        invz = 1.0 / C2[2]
        ex = pKF2.fx * C2[0] * invz + pKF2.cx
        ey = pKF2.fy * C2[1] * invz + pKF2.cy
        vbMatched2 = [False] * pKF2.N
        vMatches12 = [-1] * pKF1.N
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        n_matches = 0
        work = []
        for f1val, f2val in self._triangulation_nodes(pKF1.mFeatVec, pKF2.mFeatVec):
            cands = []
            for idx2 in f2val:
                if pKF2.get_map_point(idx2):
                    continue
                bStereo2 = pKF2.mvuRight[idx2] >= 0
                if bOnlyStereo and not bStereo2:
                    continue
                cands.append((idx2, bStereo2))
            for idx1 in f1val:
                if pKF1.get_map_point(idx1):
                    continue
                bStereo1 = pKF1.mvuRight[idx1] >= 0
                if bOnlyStereo and not bStereo1:
                    continue
                work.append((idx1, bStereo1, cands, pKF1.mDescriptors[idx1]))
        dists = self._batched([(w[3], [c[0] for c in w[2]]) for w in work], pKF2.mDescriptors)
        for (idx1, bStereo1, cands, _), dq in zip(work, dists):
            kp1 = pKF1.mvKeysUn[idx1]
            best_dist, best_idx2 = TH_LOW, -1
            for (idx2, bStereo2), dist in zip(cands, dq.tolist()):
                if vbMatched2[idx2]:
                    continue
                if dist > TH_LOW or dist > best_dist:
                    continue
                kp2 = pKF2.mvKeysUn[idx2]
                if not bStereo1 and not bStereo2:
                    distex = ex - kp2.pt[0]
                    distey = ey - kp2.pt[1]
                    if distex ** 2 + distey ** 2 < 100 * pKF2.mvScaleFactors[kp2.octave]:
                        continue
                if self.check_dist_epipolar_line(kp1, kp2, F12, pKF2):
                    best_idx2 = idx2
                    best_dist = dist
            if best_idx2 >= 0:
                kp2 = pKF2.mvKeysUn[best_idx2]
                vMatches12[idx1] = best_idx2
                n_matches += 1
                vbMatched2[best_idx2] = True
                if self.mbCheckOrientation:
                    rot = kp1.angle - kp2.angle
                    if rot < 0:
                        rot += 360.0
                    b = round(rot * factor)
                    if b == HISTO_LENGTH:
                        b = 0
                    rot_hist[b].append(idx1)
        if self.mbCheckOrientation:
            n_matches -= self._reject_by_rotation(rot_hist, lambda i: vMatches12.__setitem__(i, -1))
        return [(i, m) for i, m in enumerate(vMatches12) if m >= 0]

    # ORBMatcher.py:698-711
    def check_dist_epipolar_line(self, kp1, kp2, F12, pKF2):
        a = kp1.pt[0] * F12[0, 0] + kp1.pt[1] * F12[1, 0] + F12[2, 0]
        b = kp1.pt[0] * F12[0, 1] + kp1.pt[1] * F12[1, 1] + F12[2, 1]
        c = kp1.pt[0] * F12[0, 2] + kp1.pt[1] * F12[1, 2] + F12[2, 2]
        num = a * kp2.pt[0] + b * kp2.pt[1] + c
        den = a ** 2 + b ** 2
        if den == 0:
            return False
        return (num ** 2) / den < 3.84 * pKF2.mvLevelSigma2[kp2.octave]

    def _sim3_side(self, vpMapPoints, already, Rw, tw, sR, t, pKFo, th, K):
        """One direction of search_by_sim3 (ORBMatcher.py:744-783 / 785-825): best index in pKFo per point.
        K = (fx, fy, cx, cy): the reference projects both directions with pKF1's intrinsics."""
        fx, fy, cx, cy = K
        work = []
        for i, pMP in enumerate(vpMapPoints):
            if not pMP or already[i] or pMP.is_bad():
                continue
            p3Dw = pMP.get_world_pos()
            p3Dc = sR @ (Rw @ p3Dw + tw) + t
            if p3Dc[2] < 0.0:
                continue
            invz = 1.0 / p3Dc[2]
            x, y = p3Dc[0] * invz, p3Dc[1] * invz
            u, v = fx * x + cx, fy * y + cy
            if not pKFo.is_in_image(u, v):
                continue
            maxDistance = pMP.get_max_distance_invariance()
            minDistance = pMP.get_min_distance_invariance()
            dist3D = np.linalg.norm(p3Dc)
            if not (minDistance <= dist3D <= maxDistance):
                continue
            lvl = pMP.predict_scale(dist3D, pKFo)
            vIndices = pKFo.get_features_in_area(u, v, th * pKFo.mvScaleFactors[lvl])
            if not vIndices:
                continue
            cands = [idx for idx in vIndices if lvl - 1 <= pKFo.mvKeysUn[idx].octave <= lvl]
            work.append((i, cands, pMP.get_descriptor()))
        best = [-1] * len(vpMapPoints)
        for (i, cands, _), dq in zip(work, self._batched([(w[2], w[1]) for w in work], pKFo.mDescriptors)):
            best_dist, best_idx = np.inf, -1
            for idx, dist in zip(cands, dq.tolist()):
                if dist < best_dist:
                    best_dist, best_idx = dist, idx
            if best_dist <= TH_HIGH:
                best[i] = best_idx
        return best

    # ORBMatcher.py:713-848
    def search_by_sim3(self, pKF1, pKF2, vpMatches12, s12, R12, t12, th):
        R1w, t1w = pKF1.get_rotation(), pKF1.get_translation()
        R2w, t2w = pKF2.get_rotation(), pKF2.get_translation()
        sR12 = s12 * R12
        sR21 = (1.0 / s12) * R12.T
        t21 = -sR21 @ t12
        vpMapPoints1 = pKF1.get_map_point_matches()
        vpMapPoints2 = pKF2.get_map_point_matches()
        N1, N2 = len(vpMapPoints1), len(vpMapPoints2)
        vbAlreadyMatched1 = [False] * N1
        vbAlreadyMatched2 = [False] * N2
        for i, pMP in enumerate(vpMatches12):
            if pMP:
                vbAlreadyMatched1[i] = True
                idx2 = pMP.get_index_in_keyframe(pKF2)
                if 0 <= idx2 < N2:
                    vbAlreadyMatched2[idx2] = True
        K = (pKF1.fx, pKF1.fy, pKF1.cx, pKF1.cy)
        vnMatch1 = self._sim3_side(vpMapPoints1, vbAlreadyMatched1, R1w, t1w, sR21, t21, pKF2, th, K)
        vnMatch2 = self._sim3_side(vpMapPoints2, vbAlreadyMatched2, R2w, t2w, sR12, t12, pKF1, th, K)
        n_found = 0
        for i1, idx2 in enumerate(vnMatch1):
            if idx2 >= 0 and vnMatch2[idx2] == i1:
                vpMatches12[i1] = vpMapPoints2[idx2]
                n_found += 1
        return n_found, vpMatches12

    # ORBMatcher.py:850-922
    def search_by_projection_ckf_scw_mp(self, pKF, Scw, vpPoints, vpMatched, th):
        sRcw = Scw[:3, :3]
        scw = np.linalg.norm(sRcw[0])
        Rcw = sRcw / scw
        tcw = Scw[:3, 3:4] / scw
        Ow = -Rcw.T @ tcw
        spAlreadyFound = set(vpMatched) - {None}
        work = []
        for pMP in vpPoints:
            if pMP.is_bad() or pMP in spAlreadyFound:
                continue
            pr = self._project_checked(pMP, pKF, Rcw, tcw, True)
            if pr is None:
                continue
            u, v, _, p3Dw = pr
            if not pKF.is_in_image(u, v):
                continue
            lvl = self._distance_gates(pMP, pKF, p3Dw, Ow)
            if lvl is None:
                continue
            vIndices = pKF.get_features_in_area(u, v, th * pKF.mvScaleFactors[lvl])
            if not vIndices:
                continue
            cands = [i for i in vIndices if lvl - 1 <= pKF.mvKeysUn[i].octave <= lvl]
            work.append((pMP, cands, pMP.get_descriptor()))
        n_matches = 0
        for (pMP, cands, _), dq in zip(work, self._batched([(w[2], w[1]) for w in work], pKF.mDescriptors)):
            best_dist, best_idx = 256, -1
            for idx, dist in zip(cands, dq.tolist()):
                if vpMatched[idx] is not None:
                    continue
                if dist < best_dist:
                    best_dist = dist
                    best_idx = idx
            if best_dist <= TH_LOW:
                vpMatched[best_idx] = pMP
                n_matches += 1
        return n_matches, vpMatched

    # ORBMatcher.py:924-1008
    def search_by_projection_f_kf_f(self, CurrentFrame, pKF, sAlreadyFound, th, ORBdist):
        Rcw = CurrentFrame.mTcw[:3, :3]
        tcw = CurrentFrame.mTcw[:3, 3:4]
        Ow = -np.dot(Rcw.T, tcw)
        rot_hist = [[] for _ in range(HISTO_LENGTH)]
        factor = 1.0 / HISTO_LENGTH
        work = []
        for i, pMP in enumerate(pKF.get_map_point_matches()):
            if not (pMP and not pMP.is_bad() and pMP not in sAlreadyFound):
                continue
            x3Dw = pMP.get_world_pos()
            x3Dc = np.dot(Rcw, x3Dw) + tcw
            invzc = 1.0 / x3Dc[2]
            u = CurrentFrame.fx * x3Dc[0] * invzc + CurrentFrame.cx
            v = CurrentFrame.fy * x3Dc[1] * invzc + CurrentFrame.cy
            if u < CurrentFrame.mnMinX or u > CurrentFrame.mnMaxX or v < CurrentFrame.mnMinY or v > CurrentFrame.mnMaxY:
                continue
            PO = x3Dw - Ow
            dist3D = np.linalg.norm(PO)
            maxDistance = pMP.get_max_distance_invariance()
            minDistance = pMP.get_min_distance_invariance()
            if dist3D < minDistance or dist3D > maxDistance:
                continue
            lvl = pMP.predict_scale(dist3D, CurrentFrame)
            vIndices2 = CurrentFrame.get_features_in_area(u, v, th * CurrentFrame.mvScaleFactors[lvl], lvl - 1, lvl + 1)
            if not vIndices2:
                continue
            work.append((i, pMP, vIndices2, pMP.get_descriptor()))
        n_matches = 0
        for (i, pMP, cands, _), dq in zip(work, self._batched([(w[3], w[2]) for w in work],
                                                             CurrentFrame.mDescriptors)):
            best_dist, best_idx2 = 256, -1
            for i2, dist in zip(cands, dq.tolist()):
                if CurrentFrame.mvpMapPoints[i2]:
                    continue
                if dist < best_dist:
                    best_dist = dist
                    best_idx2 = i2
            if best_dist <= ORBdist:
                CurrentFrame.mvpMapPoints[best_idx2] = pMP
                n_matches += 1
                if self.mbCheckOrientation:
                    rot = pKF.mvKeysUn[i].angle - CurrentFrame.mvKeysUn[best_idx2].angle
                    if rot < 0.0:
                        rot += 360.0
                    b = round(rot * factor)
                    if b == HISTO_LENGTH:
                        b = 0
                    assert 0 <= b < HISTO_LENGTH
                    rot_hist[b].append(best_idx2)
        if self.mbCheckOrientation:
            n_matches -= self._reject_by_rotation(rot_hist,
                                                  lambda i: CurrentFrame.mvpMapPoints.__setitem__(i, None))
        return n_matches
