"""Generate reference golden vectors for the stereo matcher and ORBMatcher (build container only).

This script imports the REFERENCE Python code read-only from /root/reference and records its outputs
as small fixtures under tests/golden/.  Nothing in this file travels to the GPU box at run time and no
reference source is copied: only inputs (seeds, image digests) and outputs are stored.

  * Frame.compute_stereo_matches (Frame.py:161-279) is called as an unbound method on a bare Frame
    instance whose attributes are set from an oracle extraction (kps, descriptors, sheared pyramids,
    scale tables, mb/mbf exactly as Frame.__init__ derives them at Frame.py:43-60).  Frame.py imports
    cv2 at module level (Frame.py:6) but this method never uses it, so an EMPTY module object named
    cv2 is registered only to let the import statement succeed - it implements nothing.
  * ORBMatcher.descriptor_distance / search_by_projection_f_p / search_by_projection_f_f
    (ORBMatcher.py:12-14, 215-283, 291-393) are driven with minimal stand-in Frame / MapPoint objects
    exposing only the attributes those methods read.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys
import types
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))

from oracle.oracle import OracleExtractor  # noqa: E402
from oracle import stereo_oracle  # noqa: E402
from pyorbslam_amd import synth  # noqa: E402

BF = 386.1448        # KITTI00-02.yaml:37 Camera.bf (Python float, like the YAML loader yields)
FX = 718.856         # KITTI00-02.yaml:7 Camera.fx (stored into a float32 mK, Tracking.py:49-50)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def import_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, str(REF))
    import Frame as RFrame  # noqa: E402
    import ORBMatcher as RMatcher  # noqa: E402
    return RFrame, RMatcher


class KP:
    """Stand-in exposing what compute_stereo_matches / the matcher read from cv2.KeyPoint."""
    __slots__ = ("pt", "octave", "angle")

    def __init__(self, x, y, octave, angle=0.0):
        self.pt = (float(np.float32(x)), float(np.float32(y)))
        self.octave = int(octave)
        self.angle = float(np.float32(angle))


def reference_stereo(RFrame, kl, dl, kr, dr, pyr_l, pyr_r, tables, bf=BF, fx=FX):
    f = RFrame.Frame.__new__(RFrame.Frame)
    f.mvKeys = [KP(k["x"], k["y"], k["octave"]) for k in kl]
    f.mvKeysRight = [KP(k["x"], k["y"], k["octave"]) for k in kr]
    f.mDescriptors = dl
    f.mDescriptorsRight = dr
    f.mvImagePyramidLeft = pyr_l
    f.mvImagePyramidRight = pyr_r
    f.mvScaleFactors = [float(v) for v in tables["scale"]]
    f.mvInvScaleFactors = [float(v) for v in tables["inv_scale"]]
    mK = np.eye(3, dtype=np.float32)
    mK[0, 0] = fx
    f.mK = mK
    f.mbf = bf
    f.mb = f.mbf / f.mK[0][0]
    f.N = len(f.mvKeys)
    f.compute_stereo_matches()
    return f.mvuRight, f.mvDepth


def stereo_case(RFrame, name, left, right, params, meta):
    exL = OracleExtractor(**params)
    exR = OracleExtractor(**params)
    kl, dl = exL.extract(left)
    kr, dr = exR.extract(right)
    pl, pr = exL.sheared_pyramid(), exR.sheared_pyramid()
    tables = exL.tables()
    uR, dep = reference_stereo(RFrame, kl, dl, kr, dr, pl, pr, tables)
    st_u, val_u = stereo_oracle.encode(uR)
    st_d, val_d = stereo_oracle.encode(dep)
    assert (st_u == st_d).all()
    # the oracle restatement must agree with the reference bit for bit
    ou, od, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, pl, pr, tables["scale"], tables["inv_scale"],
                                                     BF, np.float32(FX))
    s2u, v2u = stereo_oracle.encode(ou)
    s2d, v2d = stereo_oracle.encode(od)
    assert (s2u == st_u).all() and (v2u == val_u).all() and (v2d == val_d).all(), name
    np.savez_compressed(GOLD / f"stereo_{name}.npz", status=st_u, u_right=val_u, depth=val_d,
                        kps_left_sha=np.array(sha(kl)), desc_left_sha=np.array(sha(dl)),
                        kps_right_sha=np.array(sha(kr)), desc_right_sha=np.array(sha(dr)),
                        left_sha=np.array(sha(left)), right_sha=np.array(sha(right)),
                        meta=np.array(json.dumps(meta)))
    print(f"stereo_{name}: N={len(kl)} Nr={len(kr)} matched={int((st_u == 1).sum())} zero-disp={int((st_u == 2).sum())}")


def gen_stereo(RFrame):
    kitti = dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    for seed in (0, 1, 2):
        L, R = synth.make_pair(seed)
        stereo_case(RFrame, f"kitti_synth_s{seed}", L, R, kitti,
                    dict(kind="synth", seed=seed, w=1241, h=376, params=kitti))
    from PIL import Image
    png = GOLD / "kitti06-436.png"
    if not png.exists():
        shutil.copyfile(REF / "pyORBExtractor" / "kitti06-436.png", png)
    L = np.array(Image.open(png).convert("L"))
    R = synth.shifted_right(L, seed=7)
    stereo_case(RFrame, "kitti06_436", L, R, kitti, dict(kind="kitti06-436.png", right_seed=7, params=kitti))
    euroc = dict(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    L, R = synth.make_pair(100, 752, 480)
    stereo_case(RFrame, "euroc_synth_s100", L, R, euroc, dict(kind="synth", seed=100, w=752, h=480, params=euroc))
    # identical views: exercises the zero-disparity substitution (Frame.py:273-275)
    L, _ = synth.make_pair(3)
    stereo_case(RFrame, "identical_s3", L, L.copy(), kitti, dict(kind="identical", seed=3, params=kitti))


# ------------------------------------------------------------------------------------ ORBMatcher
class MP:
    """Stand-in MapPoint exposing only what search_by_projection_f_p / _f_f read."""

    def __init__(self, desc, pos=None, in_view=True, proj=(0.0, 0.0, 0.0), level=0, view_cos=1.0, bad=False, obs=2):
        self._d = desc
        self._p = pos
        self.mbTrackInView = in_view
        self.mTrackProjX, self.mTrackProjY, self.mTrackProjXR = proj
        self.mnTrackScaleLevel = level
        self.mTrackViewCos = view_cos
        self._bad = bad
        self._obs = obs

    def is_bad(self):
        return self._bad

    def get_descriptor(self):
        return self._d.copy()

    def get_world_pos(self):
        return self._p.copy()

    def observations(self):
        return self._obs


def make_frame_arrays(rng, n, w=1241, h=376):
    return dict(x=rng.uniform(20, w - 20, n).astype(np.float32), y=rng.uniform(20, h - 20, n).astype(np.float32),
                octave=rng.integers(0, 8, n).astype(np.int32), angle=rng.uniform(0, 360, n).astype(np.float32),
                desc=rng.integers(0, 256, (n, 32), dtype=np.uint8),
                uR=np.where(rng.random(n) < 0.3, -1.0, 0.0).astype(np.float32))


class GridFrame:
    """Stand-in Frame built from arrays; grid bookkeeping and get_features_in_area are the REFERENCE's
    methods (Frame.py:143-159, 373-416) bound to this object."""

    def __init__(self, RFrame, a, w=1241, h=376):
        n = len(a["x"])
        self.N = n
        self.mvKeys = [KP(a["x"][i], a["y"][i], a["octave"][i], a["angle"][i]) for i in range(n)]
        self.mvKeysUn = self.mvKeys
        self.mDescriptors = a["desc"]
        self.mvuRight = [(-1 if a["uR"][i] < 0 else np.float32(a["uR"][i])) for i in range(n)]
        self.mvpMapPoints = [None] * n
        self.mvbOutlier = [False] * n
        self.mvScaleFactors = [float(np.float32(1.2) ** 0)] + [float(v) for v in np.cumprod([np.float32(1.2)] * 7)]
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = 0.0, float(w), 0.0, float(h)
        self.FRAME_GRID_COLS, self.FRAME_GRID_ROWS = 64, 48
        self.mfGridElementWidthInv = 64.0 / w
        self.mfGridElementHeightInv = 48.0 / h
        self.fx = self.fy = FX
        self.cx, self.cy = 607.1928, 185.2157
        self.mbf = BF
        mK = np.eye(3, dtype=np.float32)
        mK[0, 0] = FX
        self.mb = self.mbf / mK[0][0]
        self._ref = RFrame.Frame
        RFrame.Frame.assign_features_to_grid(self)

    def pos_in_grid(self, kps):
        return self._ref.pos_in_grid(self, kps)

    def get_features_in_area(self, x, y, r, min_level, max_level):
        return self._ref.get_features_in_area(self, x, y, r, min_level, max_level)


def pose(rng, t_scale=0.3, rot_scale=0.02):
    a = rng.normal(0, rot_scale, 3)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) + K + K @ K / 2
    U, _, Vt = np.linalg.svd(R)
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = (U @ Vt).astype(np.float32)
    T[:3, 3] = rng.normal(0, t_scale, 3).astype(np.float32)
    return T


def noisy(rng, d):
    d = d.copy()
    if rng.random() < 0.8:
        flip = rng.integers(0, 256, 32, dtype=np.uint8) & rng.integers(0, 256, 32, dtype=np.uint8)
        flip &= rng.integers(0, 256, 32, dtype=np.uint8)
        return d ^ flip
    return rng.integers(0, 256, 32, dtype=np.uint8)


def gen_matcher(RFrame, RMatcher):
    rng = np.random.Generator(np.random.PCG64(20251015))
    m = RMatcher.ORBMatcher(0.8, True)
    a = rng.integers(0, 256, (256, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (256, 32), dtype=np.uint8)
    b[:8] = a[:8]
    b[8:16] = 255 - a[8:16]
    dd = [int(m.descriptor_distance(a[i], b[i])) for i in range(256)]
    np.savez_compressed(GOLD / "matcher_distance.npz", a=a, b=b, dist=np.array(dd, np.int32))
    counts = []
    # ---- search_by_projection_f_p (ORBMatcher.py:215-283)
    for case in range(6):
        fa = make_frame_arrays(rng, 1500)
        fa["uR"] = np.where(fa["uR"] < 0, -1.0, fa["x"] - rng.uniform(1, 60, 1500)).astype(np.float32)
        fr = GridFrame(RFrame, fa)
        nmp = 600
        q = dict(desc=np.zeros((nmp, 32), np.uint8), proj=np.zeros((nmp, 3), np.float64),
                 level=np.zeros(nmp, np.int32), view_cos=np.zeros(nmp), in_view=np.zeros(nmp, bool),
                 bad=np.zeros(nmp, bool), obs=np.zeros(nmp, np.int32))
        mps = []
        for j in range(nmp):
            i = int(rng.integers(0, fr.N))
            k = fr.mvKeys[i]
            q["desc"][j] = noisy(rng, fr.mDescriptors[i])
            px, py = float(k.pt[0] + rng.normal(0, 2)), float(k.pt[1] + rng.normal(0, 2))
            q["proj"][j] = (px, py, px - float(rng.uniform(0, 40)))
            q["level"][j] = int(np.clip(k.octave + rng.integers(-1, 2), 0, 7))
            q["view_cos"][j] = float(rng.choice([0.999, 0.5]))
            q["in_view"][j] = bool(rng.random() < 0.95)
            q["bad"][j] = bool(rng.random() < 0.03)
            q["obs"][j] = int(rng.choice([0, 1, 3]))
            mps.append(MP(q["desc"][j], in_view=bool(q["in_view"][j]), proj=tuple(float(v) for v in q["proj"][j]),
                          level=int(q["level"][j]), view_cos=float(q["view_cos"][j]), bad=bool(q["bad"][j]),
                          obs=int(q["obs"][j])))
        th = [1.0, 3.0, 5.0][case % 3]
        n = m.search_by_projection_f_p(fr, mps, th)
        assigned = np.array([(-1 if p is None else mps.index(p)) for p in fr.mvpMapPoints], np.int32)
        np.savez_compressed(GOLD / f"matcher_fp_{case}.npz", th=th, n_matches=n, assigned=assigned,
                            **{f"frame_{k}": v for k, v in fa.items()}, **{f"mp_{k}": v for k, v in q.items()})
        counts.append(n)
    # ---- search_by_projection_f_f (ORBMatcher.py:291-393)
    for case in range(6):
        ca = make_frame_arrays(rng, 1500)
        cur = GridFrame(RFrame, ca)
        Tc = pose(rng)
        # forward / backward / sideways motion relative to the last frame (b_forward / b_backward)
        dz = [0.0, 0.9, -0.9][case % 3]
        Tl = Tc.copy()
        Tl[2, 3] += np.float32(dz)
        cur.mTcw = Tc
        nl = 1200
        la = make_frame_arrays(rng, nl)
        last = GridFrame(RFrame, la)
        last.mTcw = Tl
        Rcw, tcw = Tc[:3, :3].astype(np.float64), Tc[:3, 3].astype(np.float64)
        mpos = np.zeros((nl, 3), np.float32)
        mdesc = np.zeros((nl, 32), np.uint8)
        has = np.zeros(nl, bool)
        outl = np.zeros(nl, bool)
        obs = np.zeros(nl, np.int32)
        for i in range(nl):
            if rng.random() < 0.15:
                continue
            j = int(rng.integers(0, cur.N))
            k = cur.mvKeys[j]
            z = float(rng.uniform(3, 40))
            u, v = k.pt[0] + rng.normal(0, 3), k.pt[1] + rng.normal(0, 3)
            pc = np.array([(u - cur.cx) * z / FX, (v - cur.cy) * z / FX, z])
            mpos[i] = (Rcw.T @ (pc - tcw)).astype(np.float32)
            mdesc[i] = noisy(rng, cur.mDescriptors[j])
            has[i] = True
            outl[i] = rng.random() < 0.05
            obs[i] = int(rng.choice([1, 2, 3]))
        mps = [MP(mdesc[i], pos=mpos[i].reshape(3, 1), obs=int(obs[i])) if has[i] else None for i in range(nl)]
        last.mvpMapPoints = mps
        last.mvbOutlier = [bool(v) for v in outl]
        # some current keypoints already hold map points (with and without observations)
        pre = np.full(cur.N, -1, np.int32)
        pre_obs = np.zeros(cur.N, np.int32)
        extra = []
        for j in rng.choice(cur.N, 60, replace=False):
            pre_obs[j] = int(rng.choice([0, 2]))
            extra.append(MP(cur.mDescriptors[j], pos=np.zeros((3, 1), np.float32), obs=int(pre_obs[j])))
            pre[j] = len(extra) - 1
            cur.mvpMapPoints[j] = extra[-1]
        th = [7.0, 15.0][case % 2]
        n = m.search_by_projection_f_f(cur, last, th)
        assigned = []
        for p in cur.mvpMapPoints:
            if p is None:
                assigned.append(-1)
            elif p in extra:
                assigned.append(-2 - extra.index(p))
            else:
                assigned.append(mps.index(p))
        np.savez_compressed(GOLD / f"matcher_ff_{case}.npz", th=th, n_matches=n, assigned=np.array(assigned, np.int32),
                            Tc=Tc, Tl=Tl, mp_pos=mpos, mp_desc=mdesc, mp_has=has, mp_outlier=outl, mp_obs=obs,
                            pre=pre, pre_obs=pre_obs, **{f"cur_{k}": v for k, v in ca.items()},
                            **{f"last_{k}": v for k, v in la.items()})
        counts.append(n)
    print("matcher goldens:", counts)


def main():
    GOLD.mkdir(parents=True, exist_ok=True)
    RFrame, RMatcher = import_reference()
    gen_stereo(RFrame)
    gen_matcher(RFrame, RMatcher)


if __name__ == "__main__":
    main()
