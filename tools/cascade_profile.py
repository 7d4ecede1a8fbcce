"""Per-level k_resize_cascade timing from orbfe_debug_cascade_profile (development aid): medians over the
(image, strip) workgroups of the wall-clock marks (us from the workgroup's start) — 1 level-0 rows staged,
2 + l level l begins (its first barrier passed), 12 + l level l done — and the spread of workgroup starts / ends.
usage: python tools/cascade_profile.py [--pairs 8] [--frame]"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=8)
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd._lib import call
    imgs = torch.from_numpy(synth.make_batch(a.pairs)).cuda()
    fe = StereoFrontEnd(max_pairs=a.pairs)
    for _ in range(3):
        fe.enqueue(imgs)
    torch.cuda.synchronize()
    n = 2 * a.pairs * 512 * 32
    buf = np.zeros(n, np.int64)
    ns = C.c_int32()
    for _ in range(3):  # warm
        call("orbfe_debug_cascade_profile", fe.handle, buf.ctypes.data_as(C.c_void_p), n, C.byref(ns))
    S = ns.value
    m = buf[:2 * a.pairs * S * 32].reshape(2 * a.pairs * S, 32).astype(np.float64) / 100.0  # us (100 MHz)
    t0 = m[:, 0:1]
    rel = m - t0
    names = {1: "staged"} | {2 + l: f"L{l} start" for l in range(1, 8)} | {12 + l: f"L{l} done" for l in range(1, 8)}
    print(f"{2 * a.pairs} images x {S} strips; medians / max (us from the workgroup start):")
    for i in sorted(names):
        if (m[:, i] > 0).all():
            print(f"  {names[i]:10s} p50 {np.median(rel[:, i]):6.2f}  max {rel[:, i].max():6.2f}")
    last = max(i for i in names if (m[:, i] > 0).all())
    print(f"start spread {m[:, 0].max() - m[:, 0].min():.2f} us, first start -> last end {m[:, last].max() - m[:, 0].min():.2f} us")


if __name__ == "__main__":
    main()
