"""TEST / BASELINE INFRASTRUCTURE ONLY — Frame.compute_stereo_matches (reference Frame.py:161-279) restated
with the reference's own per-keypoint loop structure, for bench.py's cpu_baseline ("the reference's CPU
path timed on the GPU box's host cores"; the reference itself cannot travel there).

oracle/stereo_oracle.py is the fast checker (vectorised candidate scan, popcount table); this module is
deliberately NOT vectorised where the reference is not:
  * the row buckets are Python lists filled per right keypoint and row (Frame.py:170-179);
  * every candidate's Hamming distance is a Python popcount over the 32 XOR bytes, like
    Frame.descriptor_distance (Frame.py:324-326), called per candidate that passes the gates (:207-220);
  * the refinement builds 11 float32 patches per match and takes 11 numpy SAD sums (:224-255).
Keypoints are read from per-keypoint Python objects, as the reference reads cv2.KeyPoint attributes.
Outputs equal the reference's (tests/test_oracle_cpu.py checks them against the reference goldens), so
the time it takes is the reference algorithm's time under this interpreter.
"""
from __future__ import annotations

import math

import numpy as np

TH_HIGH, TH_LOW = 100, 50   # ORBMatcher.py:3-4 (imported by Frame.py:8)
_W, _L = 5, 5               # SAD half window, shift range (Frame.py:230, 237)


class _Kp:
    __slots__ = ("pt", "octave")

    def __init__(self, x, y, octave):
        self.pt = (x, y)
        self.octave = octave


def _keypoints(kps) -> list:
    return [_Kp(float(k["x"]), float(k["y"]), int(k["octave"])) for k in kps]


def _hamming(a, b) -> int:  # Frame.descriptor_distance (Frame.py:324-326)
    return sum(bin(v).count("1") for v in np.bitwise_xor(a, b))


def compute_stereo_matches_loop(kps_l, kps_r, desc_l, desc_r, pyr_l, pyr_r, scale_factors, inv_scale_factors, mbf,
                                fx32):
    """Returns (mvuRight, mvDepth) lists with the reference's element types."""
    left, right = _keypoints(kps_l), _keypoints(kps_r)
    sf = [float(v) for v in scale_factors]
    isf = [float(v) for v in inv_scale_factors]
    n = len(left)
    u_right, depth = [-1] * n, [-1] * n
    th_orb = (TH_HIGH + TH_LOW) / 2
    rows = [[] for _ in range(pyr_l[0].shape[0])]
    for ir, kp in enumerate(right):
        r = 2.0 * sf[kp.octave]
        for yi in range(math.floor(kp.pt[1] - r), math.ceil(kp.pt[1] + r) + 1):
            rows[yi].append(ir)
    mb = mbf / fx32                 # Frame.py:43 (mK is float32)
    max_d, min_d = mbf / mb, 0      # Frame.py:181-183
    for il, kp in enumerate(left):
        lvl = kp.octave
        ul, vl = kp.pt
        cands = rows[int(vl)]
        if not cands:
            continue
        min_u, max_u = ul - max_d, ul - min_d
        if max_u < 0:
            continue
        best, best_r = TH_HIGH, 0
        dl = desc_l[il][:]
        for ic in cands:
            kr = right[ic]
            if kr.octave < lvl - 1 or kr.octave > lvl + 1:
                continue
            if min_u <= kr.pt[0] <= max_u:
                d = _hamming(dl, desc_r[ic])
                if d < best:
                    best, best_r = d, ic
        if not best < th_orb:
            continue
        inv = isf[lvl]
        su_l, sv_l, su_r = round(ul * inv), round(vl * inv), round(right[best_r].pt[0] * inv)
        pl, pr = pyr_l[lvl], pyr_r[lvl]
        patch_l = pl[sv_l - _W:sv_l + _W + 1, su_l - _W:su_l + _W + 1].astype(np.float32)
        patch_l = patch_l - patch_l[_W, _W] * np.ones_like(patch_l, dtype=np.float32)
        best_sad, best_inc = float("inf"), 0
        sads = [0] * (2 * _L + 1)
        if su_r + _L - _W < 0 or su_r + _L + _W + 1 >= pr.shape[1]:
            continue
        for inc in range(-_L, _L + 1):
            patch_r = pr[sv_l - _W:sv_l + _W + 1, su_r + inc - _W:su_r + inc + _W + 1].astype(np.float32)
            patch_r = patch_r - patch_r[_W, _W] * np.ones_like(patch_r, dtype=np.float32)
            sad = np.sum(np.abs(patch_l - patch_r))
            if sad < best_sad:
                best_sad, best_inc = sad, inc
            sads[_L + inc] = sad
        if best_inc in (-_L, _L):
            continue
        d1, d2, d3 = sads[_L + best_inc - 1], sads[_L + best_inc], sads[_L + best_inc + 1]
        delta = (d1 - d3) / (2.0 * (d1 + d3 - 2.0 * d2))
        if delta < -1 or delta > 1:
            continue
        best_ur = sf[lvl] * (su_r + best_inc + delta)
        disparity = ul - best_ur
        if min_d <= disparity < max_d:
            if disparity <= 0:
                disparity = 0.01
                best_ur = ul - 0.01
            depth[il] = mbf / disparity
            u_right[il] = best_ur
    return u_right, depth
