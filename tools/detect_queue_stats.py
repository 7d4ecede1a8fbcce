"""Per-cell queue sizes of k_detect's two-queue path on synthetic KITTI images (numpy restatement of the
pre-test bound, the exact FAST M and the NMS; tools only, not a test): how many 64-lane M / NMS steps each
stage runs, and what a B \\ A fallback queue would save."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle.oracle import OracleExtractor  # noqa: E402
from pyorbslam_amd import synth  # noqa: E402

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2), (-3, -1),
          (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def maps(img):
    I = img.astype(np.int32)
    h, w = I.shape
    P = np.pad(I, 3, mode="edge")
    d = np.stack([I - P[3 + dy:3 + dy + h, 3 + dx:3 + dx + w] for dx, dy in CIRCLE])  # (16, h, w)
    M = np.zeros((h, w), np.int32)
    for k in range(16):
        idx = [(k + j) % 16 for j in range(9)]
        M = np.maximum(M, d[idx].min(0))
        M = np.maximum(M, (-d[idx]).min(0))
    c = [P[3 + dy:3 + dy + h, 3 + dx:3 + dx + w] for dx, dy in ((0, 3), (3, 0), (0, -3), (-3, 0))]
    a = np.maximum(np.minimum(c[0], c[2]), np.minimum(c[1], c[3]))
    b = np.minimum(np.maximum(c[0], c[2]), np.maximum(c[1], c[3]))
    bound = np.maximum(I - a, b - I)
    return M, bound


def cells(w, h):
    minX, minY, maxX, maxY = 16, 16, w - 16, h - 16
    W, H = maxX - minX, maxY - minY
    nC, nR = int(W / 30.0), int(H / 30.0)
    if nC <= 0 or nR <= 0:
        return
    wC, hC = int(np.ceil(W / nC)), int(np.ceil(H / nR))
    for i in range(nR):
        y0 = minY + i * hC
        if y0 >= maxY - 3:
            continue
        y1 = min(y0 + hC + 6, maxY)
        for j in range(nC):
            x0 = minX + j * wC
            if x0 >= maxX - 6:
                continue
            x1 = min(x0 + wC + 6, maxX)
            yield x0, y0, x1, y1


def main(n_img=4, ini=20, mn=7):
    st = dict(cells=0, fb=0, A=0, B=0, stA=0, stB=0, stBp=0, nmsA=0, nmsB=0, nmsAmin=0, nnBp=0)
    hist = []
    for s in range(n_img):
        L, _ = synth.make_pair(10_000 + s)
        o = OracleExtractor()
        o.extract(L)
        for lvl in o.pyramid():
            M, bound = maps(lvl)
            for x0, y0, x1, y1 in cells(lvl.shape[1], lvl.shape[0]):
                wy0, wx0, ww, wh = y0 + 3, x0 + 3, x1 - x0 - 6, y1 - y0 - 6
                if ww <= 0 or wh <= 0:
                    continue
                Mw = M[wy0:wy0 + wh, wx0:wx0 + ww]
                Bw = bound[wy0:wy0 + wh, wx0:wx0 + ww]
                pw = (ww + 1) // 2
                Mp = np.zeros((wh, 2 * pw), np.int32)
                Bp = np.zeros((wh, 2 * pw), np.int32)
                Mp[:, :ww], Bp[:, :ww] = Mw, Bw
                pb = np.maximum(Bp[:, 0::2], Bp[:, 1::2])
                pm = np.maximum(Mp[:, 0::2], Mp[:, 1::2])
                A, B = pb > ini, pb > mn
                nA, nB = int(A.sum()), int(B.sum())
                # NMS at a threshold over the window (outside = 0)
                Z = np.pad(Mw, 1)
                nb = np.max([Z[1 + dy:1 + dy + wh, 1 + dx:1 + dx + ww] for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                             if dy or dx], axis=0)
                kept_ini = int(((Mw > ini) & (Mw > nb)).sum())
                fb = kept_ini == 0
                st["cells"] += 1
                st["A"] += nA
                st["stA"] += -(-nA // 64)
                nnA = int((A & (pm > ini)).sum())
                st["nmsA"] += -(-nnA // 64)
                st["nmsAmin"] += -(-int((A & (pm > mn)).sum()) // 64)
                if fb:
                    st["fb"] += 1
                    st["B"] += nB
                    st["stB"] += -(-nB // 64)
                    st["stBp"] += -(-(nB - nA) // 64)
                    nnB = int((B & (pm > mn)).sum())
                    st["nmsB"] += -(-nnB // 64)
                    st["nnBp"] += -(-int((B & ~A & (pm > mn)).sum()) // 64)
                    hist.append((nA, nB))
    c = st["cells"]
    print({k: round(v / c, 3) for k, v in st.items()}, "cells", c)
    h = np.array(hist)
    print("fallback cells: mean |A|", h[:, 0].mean(), "mean |B|", h[:, 1].mean(),
          "share with |A| = 0:", (h[:, 0] == 0).mean())


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
