"""Polarity of k_detect's queued pixel pairs on synthetic KITTI images (numpy restatement of the cardinal
pre-test bound; tools only, not a test).  The exact M runs a bright and a dark min / max chain (40 packed ops
each) for every queued pair; a pair whose pixels pass the bound in one polarity only needs one chain.  Counts,
per queue (A at iniTh, B at minTh): pairs needing the bright chain only, the dark one only, or both; 64-lane
M steps with and without polarity-split queues; pixels that need both chains and the cells holding any."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle.oracle import OracleExtractor  # noqa: E402
from pyorbslam_amd import synth  # noqa: E402
from tools.detect_queue_stats import cells  # noqa: E402


def main(n_img=3, ini=20, mn=7):
    tot = {}
    for s in range(n_img):
        L, _ = synth.make_pair(10_000 + s)
        o = OracleExtractor()
        o.extract(L)
        for lvl in o.pyramid():
            I = lvl.astype(np.int32)
            h, w = I.shape
            P = np.pad(I, 3, mode="edge")
            c = [P[3 + dy:3 + dy + h, 3 + dx:3 + dx + w] for dx, dy in ((0, 3), (3, 0), (0, -3), (-3, 0))]
            a = np.maximum(np.minimum(c[0], c[2]), np.minimum(c[1], c[3]))
            b = np.minimum(np.maximum(c[0], c[2]), np.maximum(c[1], c[3]))
            bright, dark = I - a, b - I  # the bound is max(bright, dark)
            for x0, y0, x1, y1 in cells(w, h):
                wy0, wx0, ww, wh = y0 + 3, x0 + 3, x1 - x0 - 6, y1 - y0 - 6
                if ww <= 0 or wh <= 0:
                    continue
                pw = (ww + 1) // 2
                for name, t in (("A", ini), ("B", mn)):
                    nb = np.zeros((wh, 2 * pw), bool)
                    nd = np.zeros((wh, 2 * pw), bool)
                    nb[:, :ww] = bright[wy0:wy0 + wh, wx0:wx0 + ww] > t
                    nd[:, :ww] = dark[wy0:wy0 + wh, wx0:wx0 + ww] > t
                    pb, pd = nb[:, 0::2] | nb[:, 1::2], nd[:, 0::2] | nd[:, 1::2]
                    q = pb | pd
                    qb, qd = pb[q], pd[q]
                    d = tot.setdefault(name, dict(pairs=0, only_bright=0, only_dark=0, both=0, steps=0, steps_split=0,
                                                  px=0, both_px=0, cells=0, cells_any_both_px=0))
                    d["pairs"] += int(q.sum())
                    d["only_bright"] += int((qb & ~qd).sum())
                    d["only_dark"] += int((qd & ~qb).sum())
                    d["both"] += int((qb & qd).sum())
                    d["steps"] += -(-len(qb) // 64)
                    d["steps_split"] += -(-int(qb.sum()) // 64) + -(-int(qd.sum()) // 64)
                    d["px"] += int((nb | nd).sum())
                    nbp = int((nb & nd).sum())
                    d["both_px"] += nbp
                    d["cells"] += 1
                    d["cells_any_both_px"] += nbp > 0
    for k, d in tot.items():
        p = d["pairs"]
        print(f"queue {k}: {p} pairs; bright only {d['only_bright'] / p:.3f}, dark only {d['only_dark'] / p:.3f}, "
              f"both {d['both'] / p:.3f}; 64-lane M steps {d['steps']}, with polarity-split queues "
              f"{d['steps_split']}; pixels needing both chains {d['both_px'] / d['px']:.4f}, cells holding any "
              f"{d['cells_any_both_px'] / d['cells']:.3f} ({d['both_px'] / d['cells']:.2f} per cell)")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
