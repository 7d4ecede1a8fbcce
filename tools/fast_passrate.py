"""How many pixels each FAST filter stage lets through on the synthetic workload (development aid).

For level 0 of a few synthetic images: the fraction of pixels whose cardinal upper bound (k_detect's
pre-test, 4 circle points), 8-point upper bounds (even / odd circle positions) and exact M exceed t.
usage: python tools/fast_passrate.py [--images 4] [--t 7]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def diffs(img):
    I = img.astype(np.int32)
    h, w = I.shape
    c = I[3:h - 3, 3:w - 3]
    return np.stack([c - I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])  # d_k = I(p) - I(p+o_k)


def arc_bound(d, pos, run):
    """max over windows of `run` cyclically consecutive entries of `pos` of min(d) and of min(-d)."""
    sub = d[pos]
    n = len(pos)
    lo = np.full(d.shape[1:], -999, np.int32)
    for s in range(n):
        idx = [(s + j) % n for j in range(run)]
        lo = np.maximum(lo, np.maximum(sub[idx].min(0), (-sub[idx]).min(0)))
    return lo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=4)
    ap.add_argument("--t", type=int, default=7)
    a = ap.parse_args()
    from pyorbslam_amd import synth
    tot = {"card": 0, "even8": 0, "odd8": 0, "both8": 0, "exact": 0, "px": 0}
    for s in range(a.images):
        L, _ = synth.make_pair(s)
        d = diffs(L)
        card = arc_bound(d, [0, 4, 8, 12], 2)
        even = arc_bound(d, [0, 2, 4, 6, 8, 10, 12, 14], 4)
        odd = arc_bound(d, [1, 3, 5, 7, 9, 11, 13, 15], 4)
        m = arc_bound(d, list(range(16)), 9)
        tot["px"] += m.size
        tot["card"] += int((card > a.t).sum())
        tot["even8"] += int((even > a.t).sum())
        tot["odd8"] += int((odd > a.t).sum())
        tot["both8"] += int(((even > a.t) & (odd > a.t)).sum())
        tot["exact"] += int((m > a.t).sum())
        assert np.all(card >= m) and np.all(even >= m) and np.all(odd >= m)
    px = tot.pop("px")
    for k, v in tot.items():
        print(f"{k:6s} {v / px:8.4f}")


if __name__ == "__main__":
    main()
