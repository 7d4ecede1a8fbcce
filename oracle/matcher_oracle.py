"""TEST INFRASTRUCTURE ONLY — restatement of ORBMatcher's projection searches (ORBMatcher.py:215-393)
with a numpy popcount per candidate, pinned against tests/golden/matcher_*.npz (made by calling the
reference ORBMatcher)."""
import numpy as np

TH_HIGH, HISTO_LENGTH = 100, 30
_POP8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


def dist(a, b):
    return int(_POP8[np.bitwise_xor(np.asarray(a, np.uint8), np.asarray(b, np.uint8))].sum())


def search_f_p(frame, mps, th, nnratio):
    n = 0
    for p in mps:
        if not p.mbTrackInView or p.is_bad():
            continue
        lvl = p.mnTrackScaleLevel
        r = 2.5 if p.mTrackViewCos > 0.998 else 4.0
        if th != 1.0:
            r *= th
        cand = frame.get_features_in_area(p.mTrackProjX, p.mTrackProjY, r * frame.mvScaleFactors[lvl], lvl - 1, lvl)
        if not cand:
            continue
        d = p.get_descriptor()
        b1, l1, b2, l2, bi = 256, -1, 256, -1, -1
        for idx in cand:
            if frame.mvpMapPoints[idx] and frame.mvpMapPoints[idx].observations() > 0:
                continue
            if frame.mvuRight[idx] > 0 and abs(p.mTrackProjXR - frame.mvuRight[idx]) > r * frame.mvScaleFactors[lvl]:
                continue
            e = dist(d, frame.mDescriptors[idx])
            if e < b1:
                b2, l2, b1, l1, bi = b1, l1, e, frame.mvKeysUn[idx].octave, idx
            elif e < b2:
                b2, l2 = e, frame.mvKeysUn[idx].octave
        if b1 <= TH_HIGH:
            if l1 == l2 and b1 > nnratio * b2:
                continue
            frame.mvpMapPoints[bi] = p
            n += 1
    return n


def search_f_f(cur, last, th, check_ori=True):
    n = 0
    hist = [[] for _ in range(HISTO_LENGTH)]
    Rcw, tcw = cur.mTcw[:3, :3], cur.mTcw[:3, 3:4]
    tlc = last.mTcw[:3, :3] @ (-Rcw.T @ tcw) + last.mTcw[:3, 3:4]
    fwd, bwd = tlc[2] > cur.mb, -tlc[2] > cur.mb
    for i in range(last.N):
        p = last.mvpMapPoints[i]
        if not p or last.mvbOutlier[i]:
            continue
        X = Rcw @ p.get_world_pos() + tcw
        xc, yc, zc = X[0][0], X[1][0], X[2][0]
        iz = 1.0 / zc
        if iz < 0:
            continue
        u = cur.fx * xc * iz + cur.cx
        v = cur.fy * yc * iz + cur.cy
        if u < cur.mnMinX or u > cur.mnMaxX or v < cur.mnMinY or v > cur.mnMaxY:
            continue
        o = last.mvKeys[i].octave
        rad = th * cur.mvScaleFactors[o]
        lo, hi = (o, -1) if fwd else ((0, o) if bwd else (o - 1, o + 1))
        cand = cur.get_features_in_area(u, v, rad, lo, hi)
        if not cand:
            continue
        d = p.get_descriptor()
        b1, bi = 256, -1
        for i2 in cand:
            if cur.mvpMapPoints[i2] and cur.mvpMapPoints[i2].observations() > 0:
                continue
            if cur.mvuRight[i2] > 0 and abs((u - cur.mbf * iz) - cur.mvuRight[i2]) > rad:
                continue
            e = dist(d, cur.mDescriptors[i2])
            if e < b1:
                b1, bi = e, i2
        if b1 <= TH_HIGH:
            cur.mvpMapPoints[bi] = p
            n += 1
            if check_ori:
                rot = last.mvKeysUn[i].angle - cur.mvKeysUn[bi].angle
                if rot < 0.0:
                    rot += 360.0
                b = round(rot * (1.0 / HISTO_LENGTH))
                hist[0 if b == HISTO_LENGTH else b].append(bi)
    if check_ori:
        top = np.argsort([len(h) for h in hist])[::-1][:3]
        for k in range(HISTO_LENGTH):
            if k not in top:
                for idx in hist[k]:
                    cur.mvpMapPoints[idx] = None
                    n -= 1
    return n
