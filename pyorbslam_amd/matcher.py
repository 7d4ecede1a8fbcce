"""Drop-in for the reference ORBMatcher's Hamming searches (ORBMatcher.py).

descriptor_distance (ORBMatcher.py:12-14), search_by_projection_f_p (:215-283) and
search_by_projection_f_f (:291-393) keep the reference's control flow and results exactly; what changes
is where the popcounts happen.  The reference calls a per-byte Python popcount (~10 us) once per
candidate inside the search loop.  Here every (query, candidate) pair of a search is collected first —
the candidate windows depend only on the frame grid, never on matches made during the search — and
all distances come back from ONE k_hamming_search launch (orbfe_hamming_csr).  The sequential part
that genuinely depends on earlier iterations (candidates already holding a map point with
observations, the stereo gate, best / second-best bookkeeping, the rotation histogram) then runs on the
host over those precomputed distances, evaluating the same Python expressions on the same objects, so
every dtype promotion of the reference is preserved.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import call, ptr

TH_HIGH = 100     # ORBMatcher.py:3
TH_LOW = 50       # ORBMatcher.py:4
HISTO_LENGTH = 30  # ORBMatcher.py:5

_handle = None


def _h():
    global _handle
    if _handle is None:
        h = C.c_void_p()
        call("orbfe_create", C.byref(_lib.make_params(2000, 1.2, 8, 20, 7)), C.byref(h))
        _handle = h
    return _handle


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


def hamming_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
    b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
    out = np.zeros((len(a), len(b)), np.int32)
    if len(a) and len(b):
        call("orbfe_hamming_matrix", _h(), ptr(a), len(a), ptr(b), len(b), ptr(out))
    return out


class ORBMatcher:
    def __init__(self, nnratio=1, checkOri=True):
        self.mfNNratio = nnratio
        self.mbCheckOrientation = checkOri

    # ORBMatcher.py:12-14 (one pair; use descriptor_distances / hamming_* for batches)
    def descriptor_distance(self, a, b):
        return int(hamming_matrix(np.asarray(a).reshape(1, 32), np.asarray(b).reshape(1, 32))[0, 0])

    def descriptor_distances(self, A, B):
        return hamming_matrix(A, B)

    def compute_three_maxima(self, histo, histo_length):
        histo_counts = [len(h) for h in histo]
        return np.argsort(histo_counts)[::-1][:3]

    def radius_by_viewing_cos(self, view_cos):
        return 2.5 if view_cos > 0.998 else 4.0

    @staticmethod
    def _batched(queries, train):
        """queries: list of (descriptor, candidate list) -> list of distance arrays."""
        off = np.zeros(len(queries) + 1, np.int32)
        for i, (_, c) in enumerate(queries):
            off[i + 1] = off[i] + len(c)
        if not queries or off[-1] == 0:
            return [np.zeros(0, np.int32) for _ in queries]
        qd = np.stack([np.asarray(d, np.uint8).reshape(32) for d, _ in queries])
        idx = np.concatenate([np.asarray(c, np.int32) for _, c in queries])
        dist = hamming_csr(qd, train, off, idx)
        return [dist[off[i]:off[i + 1]] for i in range(len(queries))]

    # ORBMatcher.py:215-283
    def search_by_projection_f_p(self, frame, vp_map_points, th):
        n_matches = 0
        b_factor = th != 1.0
        work = []
        for pMP in vp_map_points:
            if not pMP.mbTrackInView:
                continue
            if pMP.is_bad():
                continue
            n_predicted_level = pMP.mnTrackScaleLevel
            r = self.radius_by_viewing_cos(pMP.mTrackViewCos)
            if b_factor:
                r *= th
            v_indices = frame.get_features_in_area(pMP.mTrackProjX, pMP.mTrackProjY,
                                                   r * frame.mvScaleFactors[n_predicted_level],
                                                   n_predicted_level - 1, n_predicted_level)
            if not v_indices:
                continue
            work.append((pMP, n_predicted_level, r, v_indices, pMP.get_descriptor()))
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
        work = []
        for i in range(last_frame.N):
            pMP = last_frame.mvpMapPoints[i]
            if not pMP or last_frame.mvbOutlier[i]:
                continue
            x3Dw = pMP.get_world_pos()
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
            n_last_octave = last_frame.mvKeys[i].octave
            radius = th * current_frame.mvScaleFactors[n_last_octave]
            if b_forward:
                v_indices2 = current_frame.get_features_in_area(u, v, radius, n_last_octave, -1)
            elif b_backward:
                v_indices2 = current_frame.get_features_in_area(u, v, radius, 0, n_last_octave)
            else:
                v_indices2 = current_frame.get_features_in_area(u, v, radius, n_last_octave - 1, n_last_octave + 1)
            if not v_indices2:
                continue
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
