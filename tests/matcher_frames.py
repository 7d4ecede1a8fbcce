"""Rebuild the Frame / MapPoint state of the ORBMatcher goldens (tests/golden/matcher_*.npz).

The grid helpers restate Frame.assign_features_to_grid / pos_in_grid / get_features_in_area
(Frame.py:143-159, 373-416) because the reference cannot be imported on the GPU box; the goldens were
made with the reference's own methods, so matching them pins this restatement too."""
import math

import numpy as np

from conftest import BF, FX, GOLDEN


class KP:
    __slots__ = ("pt", "octave", "angle")

    def __init__(self, x, y, octave, angle=0.0):
        self.pt = (float(np.float32(x)), float(np.float32(y)))
        self.octave = int(octave)
        self.angle = float(np.float32(angle))


class MP:
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


class GridFrame:
    def __init__(self, a, w=1241, h=376):
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
        self._grid()

    def _grid(self):  # Frame.py:143-159
        self.mGrid = [[[] for _ in range(self.FRAME_GRID_ROWS)] for _ in range(self.FRAME_GRID_COLS)]
        pts = np.array([[k.pt[0], k.pt[1]] for k in self.mvKeys])
        px = np.round((pts[:, 0] - self.mnMinX) * self.mfGridElementWidthInv).astype(int)
        py = np.round((pts[:, 1] - self.mnMinY) * self.mfGridElementHeightInv).astype(int)
        ok = (px >= 0) & (px < self.FRAME_GRID_COLS) & (py >= 0) & (py < self.FRAME_GRID_ROWS)
        for i in range(self.N):
            if ok[i]:
                self.mGrid[px[i]][py[i]].append(i)

    def get_features_in_area(self, x, y, r, min_level, max_level):  # Frame.py:373-416
        out = []
        x0 = max(0, int((x - self.mnMinX - r) * self.mfGridElementWidthInv))
        if x0 >= self.FRAME_GRID_COLS:
            return out
        x1 = min(self.FRAME_GRID_COLS - 1, int((x - self.mnMinX + r) * self.mfGridElementWidthInv))
        if x1 < 0:
            return out
        y0 = max(0, int((y - self.mnMinY - r) * self.mfGridElementHeightInv))
        if y0 >= self.FRAME_GRID_ROWS:
            return out
        y1 = min(self.FRAME_GRID_ROWS - 1, int((y - self.mnMinY + r) * self.mfGridElementHeightInv))
        if y1 < 0:
            return out
        check = (min_level > 0) or (max_level >= 0)
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for g in self.mGrid[ix][iy]:
                    k = self.mvKeysUn[g]
                    if check:
                        if k.octave < min_level:
                            continue
                        if max_level >= 0 and k.octave > max_level:
                            continue
                    if abs(k.pt[0] - x) < r and abs(k.pt[1] - y) < r:
                        out.append(g)
        return out


def _sub(z, prefix):
    return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


def load_fp(case):
    z = np.load(GOLDEN / f"matcher_fp_{case}.npz", allow_pickle=False)
    fr = GridFrame(_sub(z, "frame_"))
    q = _sub(z, "mp_")
    mps = [MP(q["desc"][j], in_view=bool(q["in_view"][j]), proj=tuple(float(v) for v in q["proj"][j]),
              level=int(q["level"][j]), view_cos=float(q["view_cos"][j]), bad=bool(q["bad"][j]), obs=int(q["obs"][j]))
           for j in range(len(q["desc"]))]
    return fr, mps, float(z["th"]), int(z["n_matches"]), z["assigned"]


def load_ff(case):
    z = np.load(GOLDEN / f"matcher_ff_{case}.npz", allow_pickle=False)
    cur = GridFrame(_sub(z, "cur_"))
    last = GridFrame(_sub(z, "last_"))
    cur.mTcw = z["Tc"]
    last.mTcw = z["Tl"]
    mps = [MP(z["mp_desc"][i], pos=z["mp_pos"][i].reshape(3, 1), obs=int(z["mp_obs"][i])) if z["mp_has"][i] else None
           for i in range(last.N)]
    last.mvpMapPoints = mps
    last.mvbOutlier = [bool(v) for v in z["mp_outlier"]]
    pre = z["pre"]
    extra = [None] * int((pre >= 0).sum())
    for j in np.nonzero(pre >= 0)[0]:
        extra[pre[j]] = MP(cur.mDescriptors[j], pos=np.zeros((3, 1), np.float32), obs=int(z["pre_obs"][j]))
        cur.mvpMapPoints[j] = extra[pre[j]]
    return cur, last, mps, extra, z


def encode_ff(cur, mps, extra):
    out = []
    for p in cur.mvpMapPoints:
        if p is None:
            out.append(-1)
        elif any(p is e for e in extra):
            out.append(-2 - next(k for k, e in enumerate(extra) if e is p))
        else:
            out.append(next(k for k, m in enumerate(mps) if m is p))
    return np.array(out, np.int32)


def encode_fp(fr, mps):
    ids = {id(m): j for j, m in enumerate(mps)}
    return np.array([-1 if p is None else ids[id(p)] for p in fr.mvpMapPoints], np.int32)
