"""Stand-in KeyFrame / Frame / MapPoint world for the keyframe-level ORBMatcher goldens
(tests/golden/matcher_kf_*.npz, made by tests/golden/gen_golden_matcher_kf.py).

The searches under test (ORBMatcher.py:21-213, 395-1008 and MapPoint.py:204-240) only read a small
surface of their arguments.  These classes provide exactly that surface, built from plain arrays so the
same world can be rebuilt on the GPU box without the reference.  The methods follow the reference's
semantics (KeyFrame.py:258-310, 432-463; MapPoint.py:98-302; Frame.py:373-416) closely enough to give
realistic inputs; parity is about the matcher, which sees identical objects on both sides.  Every
mutating call is appended to World.log as an integer tuple so the side effects can be compared too.
"""
from __future__ import annotations

import threading

import numpy as np

W, H = 1241, 376
FX, FY, CX, CY = 718.856, 718.856, 607.1928, 185.2157
BF = 386.1448
NLEV = 8
SF = [float(np.float32(1.2) ** 0)] + [float(v) for v in np.cumprod([np.float32(1.2)] * 7)]
SIG2 = [s * s for s in SF]
INV_SIG2 = [1.0 / s for s in SIG2]
GRID_COLS, GRID_ROWS = 64, 48

# event codes of World.log
EV_ADD_OBS, EV_ADD_MP, EV_REPLACE, EV_REPLACE_MATCH, EV_ERASE_MATCH = range(5)


class KP:
    __slots__ = ("pt", "octave", "angle")

    def __init__(self, x, y, octave, angle):
        self.pt = (float(np.float32(x)), float(np.float32(y)))
        self.octave = int(octave)
        self.angle = float(np.float32(angle))


def _popcount_rows(a, b):
    return np.unpackbits(np.bitwise_xor(a, b), axis=-1).sum(-1)


class World:
    def __init__(self):
        self.log = []
        self.kfs = []
        self.mps = []

    def kf_id(self, kf):
        return next(i for i, k in enumerate(self.kfs) if k is kf)

    def mp_id(self, mp):
        if mp is None:
            return -1
        return next(i for i, m in enumerate(self.mps) if m is mp)


class KeyFrame:
    """KeyFrame surface: pose getters, grid search (KeyFrame.py:432-460), map-point slots."""

    def __init__(self, world, kid, a, Tcw):
        self.world = world
        self.mnId = kid
        n = len(a["x"])
        self.N = n
        self.mvKeysUn = [KP(a["x"][i], a["y"][i], a["octave"][i], a["angle"][i]) for i in range(n)]
        self.mvKeys = self.mvKeysUn
        self.mDescriptors = a["desc"]
        self.mvuRight = [(-1 if a["uR"][i] < 0 else float(np.float32(a["uR"][i]))) for i in range(n)]
        self.mvpMapPoints = [None] * n
        self.fx, self.fy, self.cx, self.cy = FX, FY, CX, CY
        self.invfx, self.invfy = 1.0 / FX, 1.0 / FY
        self.mbf = BF
        self.mb = BF / FX
        self.mvScaleFactors = list(SF)
        self.mvLevelSigma2 = list(SIG2)
        self.mvInvLevelSigma2 = list(INV_SIG2)
        self.mnScaleLevels = NLEV
        self.mfLogScaleFactor = float(np.log(1.2))
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = 0.0, float(W), 0.0, float(H)
        self.mnGridCols, self.mnGridRows = GRID_COLS, GRID_ROWS
        self.mfGridElementWidthInv = GRID_COLS / W
        self.mfGridElementHeightInv = GRID_ROWS / H
        self.Tcw = Tcw.astype(np.float32)
        # DBoW2 FeatureVector: node id -> ascending keypoint indices, iterated in ascending node order
        words = a["word"]
        self.mFeatVec = {int(w): [int(i) for i in np.nonzero(words == w)[0]] for w in np.unique(words)}
        self.mGrid = [[[] for _ in range(GRID_ROWS)] for _ in range(GRID_COLS)]
        for i, k in enumerate(self.mvKeysUn):
            gx = int(round((k.pt[0] - self.mnMinX) * self.mfGridElementWidthInv))
            gy = int(round((k.pt[1] - self.mnMinY) * self.mfGridElementHeightInv))
            if 0 <= gx < GRID_COLS and 0 <= gy < GRID_ROWS:
                self.mGrid[gx][gy].append(i)

    def is_bad(self):
        return False

    def get_rotation(self):
        return self.Tcw[:3, :3].copy()

    def get_translation(self):
        return self.Tcw[:3, 3:4].copy()

    def get_camera_center(self):
        R, t = self.Tcw[:3, :3], self.Tcw[:3, 3:4]
        return -R.T @ t

    def get_map_point_matches(self):
        return self.mvpMapPoints.copy()

    def get_map_point(self, idx):
        return self.mvpMapPoints[idx]

    def get_map_points(self):
        return {p for p in self.mvpMapPoints if p and not p.is_bad()}

    def add_map_point(self, pMP, idx):
        self.world.log.append((EV_ADD_MP, self.mnId, self.world.mp_id(pMP), int(idx)))
        self.mvpMapPoints[idx] = pMP

    def replace_map_point_match(self, idx, pMP):
        self.world.log.append((EV_REPLACE_MATCH, self.mnId, self.world.mp_id(pMP), int(idx)))
        self.mvpMapPoints[idx] = pMP

    def erase_map_point_match(self, idx):
        self.world.log.append((EV_ERASE_MATCH, self.mnId, -1, int(idx)))
        if idx >= 0:
            self.mvpMapPoints[idx] = None

    def is_in_image(self, x, y):
        return self.mnMinX <= x < self.mnMaxX and self.mnMinY <= y < self.mnMaxY

    def get_features_in_area(self, x, y, r):
        out = []
        x0 = max(0, int(np.floor((x - self.mnMinX - r) * self.mfGridElementWidthInv)))
        if x0 >= self.mnGridCols:
            return out
        x1 = min(self.mnGridCols - 1, int(np.ceil((x - self.mnMinX + r) * self.mfGridElementWidthInv)))
        if x1 < 0:
            return out
        y0 = max(0, int(np.floor((y - self.mnMinY - r) * self.mfGridElementHeightInv)))
        if y0 >= self.mnGridRows:
            return out
        y1 = min(self.mnGridRows - 1, int(np.ceil((y - self.mnMinY + r) * self.mfGridElementHeightInv)))
        if y1 < 0:
            return out
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for i in self.mGrid[ix][iy]:
                    k = self.mvKeysUn[i]
                    if abs(k.pt[0] - x) < r and abs(k.pt[1] - y) < r:
                        out.append(i)
        return out


class Frame(KeyFrame):
    """Frame surface for search_by_projection_f_kf_f: mTcw, the 5-argument grid search (Frame.py:373-416)."""

    def __init__(self, world, a, Tcw):
        super().__init__(world, -1, a, Tcw)
        self.mTcw = self.Tcw

    def get_features_in_area(self, x, y, r, min_level=-1, max_level=-1):
        out = []
        x0 = max(0, int((x - self.mnMinX - r) * self.mfGridElementWidthInv))
        if x0 >= self.mnGridCols:
            return out
        x1 = min(self.mnGridCols - 1, int((x - self.mnMinX + r) * self.mfGridElementWidthInv))
        if x1 < 0:
            return out
        y0 = max(0, int((y - self.mnMinY - r) * self.mfGridElementHeightInv))
        if y0 >= self.mnGridRows:
            return out
        y1 = min(self.mnGridRows - 1, int((y - self.mnMinY + r) * self.mfGridElementHeightInv))
        if y1 < 0:
            return out
        check = (min_level > 0) or (max_level >= 0)
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for i in self.mGrid[ix][iy]:
                    k = self.mvKeysUn[i]
                    if check:
                        if k.octave < min_level:
                            continue
                        if max_level >= 0 and k.octave > max_level:
                            continue
                    if abs(k.pt[0] - x) < r and abs(k.pt[1] - y) < r:
                        out.append(i)
        return out


class MapPoint:
    """MapPoint surface (MapPoint.py:98-302).  replace() follows MapPoint.py:157-182, including the
    descriptor recomputation of the surviving point, so later iterations can see a changed descriptor."""

    def __init__(self, world, mid, pos, desc, normal, min_d, max_d, bad=False):
        self.world = world
        self.mnId = mid
        self.mMutexFeatures = threading.Lock()
        self._pos = pos.reshape(3, 1).astype(np.float32)
        self.mDescriptor = desc.copy()
        self._normal = normal.reshape(3, 1).astype(np.float32)
        self.mfMinDistance = float(min_d)
        self.mfMaxDistance = float(max_d)
        self.mbBad = bool(bad)
        self.mObservations = {}

    def is_bad(self):
        return self.mbBad

    def get_world_pos(self):
        return self._pos.copy()

    def get_normal(self):
        return self._normal.copy()

    def get_descriptor(self):
        return self.mDescriptor.copy()

    def get_min_distance_invariance(self):
        return 0.8 * self.mfMinDistance

    def get_max_distance_invariance(self):
        return 1.2 * self.mfMaxDistance

    def predict_scale(self, current_dist, pKF):
        ratio = self.mfMaxDistance / current_dist
        n = int(np.ceil(np.log(ratio) / pKF.mfLogScaleFactor))
        return max(0, min(n, pKF.mnScaleLevels - 1))

    def observations(self):
        return len(self.mObservations)

    def is_in_key_frame(self, pKF):
        return pKF in self.mObservations

    def get_index_in_keyframe(self, pKF):
        return self.mObservations.get(pKF, -1)

    def add_observation(self, pKF, idx):
        self.world.log.append((EV_ADD_OBS, pKF.mnId, self.mnId, int(idx)))
        if pKF not in self.mObservations:
            self.mObservations[pKF] = idx

    def replace(self, pMP):
        if pMP.mnId == self.mnId:
            return
        self.world.log.append((EV_REPLACE, self.mnId, pMP.mnId, -1))
        obs = dict(self.mObservations)
        self.mObservations.clear()
        self.mbBad = True
        for kf, idx in obs.items():
            if not pMP.is_in_key_frame(kf):
                kf.replace_map_point_match(idx, pMP)
                pMP.add_observation(kf, idx)
            else:
                kf.erase_map_point_match(idx)
        pMP._distinctive()

    def _distinctive(self):  # MapPoint.py:204-240 (stand-in's own restatement)
        if self.mbBad or not self.mObservations:
            return
        D = np.stack([kf.mDescriptors[i] for kf, i in self.mObservations.items() if not kf.is_bad()])
        n = len(D)
        M = np.zeros((n, n), np.float32)
        for i in range(n):
            M[i] = _popcount_rows(D[i][None, :], D)
        med = [float(np.median(M[i])) for i in range(n)]
        self.mDescriptor = D[int(np.argmin(med))].copy()


# ------------------------------------------------------------------------------------------------
# world construction from arrays (the arrays are what the golden files store)


def kf_arrays(rng, n, n_words=160):
    x = rng.uniform(20, W - 20, n).astype(np.float32)
    y = rng.uniform(20, H - 20, n).astype(np.float32)
    octave = rng.choice(NLEV, n, p=[.3, .2, .15, .1, .08, .07, .05, .05]).astype(np.int32)
    angle = rng.uniform(0, 360, n).astype(np.float32)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    uR = np.where(rng.random(n) < 0.6, x - rng.uniform(1, 60, n), -1.0).astype(np.float32)
    word = rng.integers(0, n_words, n).astype(np.int32)
    return dict(x=x, y=y, octave=octave, angle=angle, desc=desc, uR=uR, word=word)


def noisy_desc(rng, d, flips):
    d = d.copy()
    bits = rng.choice(256, flips, replace=False)
    for b in bits:
        d[b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def pose(rng, t=0.3, r=0.02):
    ax = rng.normal(0, r, 3)
    th = float(np.linalg.norm(ax))
    k = ax / max(th, 1e-12)
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    R = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R.astype(np.float32)
    T[:3, 3] = rng.normal(0, t, 3).astype(np.float32)
    return T


def flat(prefix, d):
    return {f"{prefix}{k}": v for k, v in d.items()}


def sub(z, prefix):
    return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


def build(z):
    """World from the arrays of a golden file: keyframes kf{j}_*, an optional frame fr_*, map points mp_*,
    initial keyframe slots kfmp{j} (map point index or -1), observations obs (mp, kf, idx) rows."""
    w = World()
    nkf = int(z["n_kf"])
    for j in range(nkf):
        w.kfs.append(KeyFrame(w, j, sub(z, f"kf{j}_"), z[f"kf{j}_T"]))
    if "fr_T" in z.files:
        w.frame = Frame(w, sub(z, "fr_"), z["fr_T"])
    n_mp = len(z["mp_desc"])
    for i in range(n_mp):
        w.mps.append(MapPoint(w, i, z["mp_pos"][i], z["mp_desc"][i], z["mp_normal"][i], z["mp_min"][i],
                              z["mp_max"][i], bool(z["mp_bad"][i])))
    for j in range(nkf):
        for i, m in enumerate(z[f"kfmp{j}"]):
            if m >= 0:
                w.kfs[j].mvpMapPoints[i] = w.mps[int(m)]
    for m, k, i in z["obs"]:
        w.mps[int(m)].mObservations[w.kfs[int(k)]] = int(i)
    if "fr_mp" in z.files:
        w.frame.mvpMapPoints = [w.mps[int(m)] if m >= 0 else None for m in z["fr_mp"]]
    return w


def make_world(rng, n_kf=2, n=1000, n_mp=700, with_frame=False, n_words=160):
    """Arrays of a random world: keyframe 1.. (and the frame) re-observe keyframe 0's map points with noisy
    descriptors near their projections, so every search finds matches, rejections and collisions."""
    out = {"n_kf": np.int32(n_kf)}
    T0 = pose(rng)
    kfa = [kf_arrays(rng, n, n_words)]
    poses = [T0]
    R0, t0 = T0[:3, :3].astype(np.float64), T0[:3, 3].astype(np.float64)
    # map points from keyframe 0's keypoints: depth, world position, scale range around the octave
    a0 = kfa[0]
    idx0 = rng.choice(n, n_mp, replace=False)
    pos = np.zeros((n_mp, 3), np.float32)
    normal = np.zeros((n_mp, 3), np.float32)
    min_d = np.zeros(n_mp, np.float64)
    max_d = np.zeros(n_mp, np.float64)
    desc = np.zeros((n_mp, 32), np.uint8)
    bad = rng.random(n_mp) < 0.03
    C0 = -R0.T @ t0
    for k, i in enumerate(idx0):
        z = float(rng.uniform(4, 40))
        pc = np.array([(a0["x"][i] - CX) * z / FX, (a0["y"][i] - CY) * z / FY, z])
        pw = R0.T @ (pc - t0)
        pos[k] = pw.astype(np.float32)
        d = float(np.linalg.norm(pw - C0))
        nv = (pw - C0) / d
        if rng.random() < 0.05:
            nv = -nv  # fails the viewing-angle test
        normal[k] = nv.astype(np.float32)
        lvl = float(a0["octave"][i]) + rng.uniform(-0.6, 0.6)
        max_d[k] = d * 1.2 ** (lvl + 0.5)
        min_d[k] = max_d[k] / 1.2 ** 7
        desc[k] = noisy_desc(rng, a0["desc"][i], int(rng.integers(0, 12)))
    kfmp = [np.full(n, -1, np.int32)]
    obs = []
    for k, i in enumerate(idx0):
        if rng.random() < 0.9:
            kfmp[0][i] = k
            obs.append((k, 0, int(i)))
    targets = list(range(1, n_kf)) + (["fr"] if with_frame else [])
    for tj in targets:
        T = pose(rng)
        R, t = T[:3, :3].astype(np.float64), T[:3, 3].astype(np.float64)
        a = kf_arrays(rng, n, n_words)
        slots = np.full(n, -1, np.int32)
        # re-observe a subset of the map points: keypoint at the projection (+ noise), descriptor and word
        # copied with noise, octave near the predicted level
        j = 0
        for k in rng.permutation(n_mp):
            if j >= int(0.7 * n):
                break
            pc = R @ pos[k].astype(np.float64) + t
            if pc[2] <= 0.1:
                continue
            u, v = FX * pc[0] / pc[2] + CX, FY * pc[1] / pc[2] + CY
            if not (1 <= u < W - 1 and 1 <= v < H - 1):
                continue
            a["x"][j] = np.float32(u + rng.normal(0, 1.0))
            a["y"][j] = np.float32(v + rng.normal(0, 1.0))
            i0 = idx0[k]
            a["octave"][j] = np.int32(np.clip(a0["octave"][i0] + rng.integers(-1, 2), 0, NLEV - 1))
            a["angle"][j] = np.float32((a0["angle"][i0] + rng.normal(0, 4) + (90 if rng.random() < 0.1 else 0)) % 360)
            a["desc"][j] = noisy_desc(rng, a0["desc"][i0], int(rng.integers(0, 30)))
            a["word"][j] = a0["word"][i0] if rng.random() < 0.85 else a["word"][j]
            if a["uR"][j] >= 0:
                a["uR"][j] = np.float32(a["x"][j] - BF / pc[2] + rng.normal(0, 0.5))
            if rng.random() < 0.3:
                slots[j] = k
                obs.append((k, tj if tj != "fr" else -1, j))
            j += 1
        if tj == "fr":
            out.update(flat("fr_", a))
            out["fr_T"] = T
            fr_mp = np.where(rng.random(n) < 0.5, slots, -1).astype(np.int32)
            out["fr_mp"] = fr_mp
            obs = [o for o in obs if o[1] != -1]
        else:
            kfa.append(a)
            poses.append(T)
            kfmp.append(slots)
    for jj in range(n_kf):
        out.update(flat(f"kf{jj}_", kfa[jj]))
        out[f"kf{jj}_T"] = poses[jj]
        out[f"kfmp{jj}"] = kfmp[jj]
    out.update(mp_pos=pos, mp_normal=normal, mp_min=min_d, mp_max=max_d, mp_desc=desc, mp_bad=bad,
               obs=np.array(obs, np.int32).reshape(-1, 3))
    return out


# ------------------------------------------------------------------------------------------------
# one call of every search on fresh builds of a world (shared by the generator and the tests)


def sim3(T, s):
    S = np.eye(4)
    S[:3, :3] = s * T[:3, :3].astype(np.float64)
    S[:3, 3] = s * T[:3, 3].astype(np.float64)
    return S


def fundamental(k1, k2):
    """F12 of ORB-SLAM2's LocalMapping::ComputeF12 from the two keyframes' poses."""
    R1, t1 = k1.get_rotation().astype(np.float64), k1.get_translation().astype(np.float64)
    R2, t2 = k2.get_rotation().astype(np.float64), k2.get_translation().astype(np.float64)
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2, 0], t12[1, 0]], [t12[2, 0], 0, -t12[0, 0]], [-t12[1, 0], t12[0, 0], 0]])
    K = np.array([[FX, 0, CX], [0, FY, CY], [0, 0, 1.0]])
    Ki = np.linalg.inv(K)
    return Ki.T @ tx @ R12 @ Ki


def drive(Matcher, z, case, pick):
    """Every search on a fresh build of the world; returns the result arrays to store."""
    res = {}
    nn = [1.0, 0.75, 0.6, 0.9, 0.8, 0.7, 1.0][case]
    ori = case != 3
    m = Matcher(nn, ori)
    # search_by_BoW_kf_f (ORBMatcher.py:21-118)
    w = build(z)
    n, matches = m.search_by_BoW_kf_f(w.kfs[0], w.frame)
    res["bowf_n"] = np.int32(n)
    res["bowf_matches"] = encode_mps(w, matches)
    # search_by_BoW_kf_kf (:120-213)
    w = build(z)
    n, matches = m.search_by_BoW_kf_kf(w.kfs[0], w.kfs[1])
    res["bowkk_n"] = np.int32(n)
    res["bowkk_matches"] = encode_mps(w, matches)
    # fuse_kf_scw_mp (:395-480)
    w = build(z)
    s = [1.0, 1.3, 0.8, 2.0, 1.1, 1.0, 1.0][case]
    Scw = sim3(z["kf1_T"], s)
    pts = [w.mps[i] for i in pick("fuse_scw")]
    th = [3.0, 5.0, 8.0, 4.0, 3.0, 10.0, 10.0][case]
    n, rep = m.fuse_kf_scw_mp(w.kfs[1], Scw, pts, th, [None] * len(pts))
    res["fscw_Scw"], res["fscw_th"] = Scw, np.float64(th)
    res["fscw_n"] = np.int32(n)
    res["fscw_rep"] = encode_mps(w, rep)
    res["fscw_log"] = encode_log(w)
    # fuse_pkf_mp (:482-582): duplicates and None entries in the list exercise the dynamic checks
    w = build(z)
    sel = pick("fuse_p")
    res["fp_th"] = np.float64(th)
    lst = [None if i < 0 else w.mps[i] for i in sel]
    n = m.fuse_pkf_mp(w.kfs[1], lst, th)
    res["fp_n"] = np.int32(n)
    res["fp_log"] = encode_log(w)
    res["fp_slots"] = encode_mps(w, w.kfs[1].mvpMapPoints)
    res["fp_bad"] = np.array([p.mbBad for p in w.mps], bool)
    res["fp_desc"] = np.stack([p.mDescriptor for p in w.mps])
    # search_for_triangulation (:584-696)
    for only in (False, True):
        w = build(z)
        F12 = fundamental(w.kfs[0], w.kfs[1])
        key = f"tri{int(only)}"
        res[f"{key}_F12"] = F12
        try:
            pairs = m.search_for_triangulation(w.kfs[0], w.kfs[1], F12, only)
            res[f"{key}_pairs"] = np.array(pairs, np.int32).reshape(-1, 2)
            res[f"{key}_stop"] = np.int32(0)
        except StopIteration:
            res[f"{key}_pairs"] = np.zeros((0, 2), np.int32)
            res[f"{key}_stop"] = np.int32(1)
    # search_by_sim3 (:713-848)
    w = build(z)
    k1, k2 = w.kfs[0], w.kfs[1]
    R1, t1 = k1.get_rotation().astype(np.float64), k1.get_translation().astype(np.float64)
    R2, t2 = k2.get_rotation().astype(np.float64), k2.get_translation().astype(np.float64)
    s12 = [1.0, 1.02, 0.97, 1.0, 1.0, 1.0, 1.0][case]
    R12 = R1 @ R2.T
    t12 = s12 * (t1 - R12 @ t2)
    pre = pick("sim3")
    v12 = [None] * k1.N
    for i1, i2 in pre:
        v12[i1] = k2.mvpMapPoints[i2]
    thr = [7.5, 10.0, 5.0, 15.0, 7.5, 10.0, 10.0][case]
    n, v12 = m.search_by_sim3(k1, k2, v12, s12, R12, t12, thr)
    res.update(sim3_s=np.float64(s12), sim3_R=R12, sim3_t=t12, sim3_th=np.float64(thr), sim3_pre=pre)
    res["sim3_n"] = np.int32(n)
    res["sim3_matches"] = encode_mps(w, v12)
    # search_by_projection_ckf_scw_mp (:850-922)
    w = build(z)
    Scw = sim3(z["kf1_T"], s)
    pts = [w.mps[i] for i in pick("ckf_pts")]
    vm = [None if i < 0 else w.mps[i] for i in pick("ckf_matched")]
    n, vm = m.search_by_projection_ckf_scw_mp(w.kfs[1], Scw, pts, vm, th)
    res["ckf_n"] = np.int32(n)
    res["ckf_matched"] = encode_mps(w, vm)
    # search_by_projection_f_kf_f (:924-1008)
    w = build(z)
    found = {w.mps[i] for i in pick("fkf_found")}
    dmax = [100, 64, 50, 100, 100, 100, 100][case]
    n = m.search_by_projection_f_kf_f(w.frame, w.kfs[0], found, th, dmax)
    res["fkf_orbdist"] = np.int32(dmax)
    res["fkf_n"] = np.int32(n)
    res["fkf_frame_mps"] = encode_mps(w, w.frame.mvpMapPoints)
    return res


def encode_mps(w, lst):
    return np.array([w.mp_id(p) if p else -1 for p in lst], np.int32)


def encode_log(w):
    return np.array(w.log, np.int32).reshape(-1, 4)
