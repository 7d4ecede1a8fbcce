"""Per-phase octree timing from orbfe_debug_octree_profile (development aid): median over images of the
wall-clock deltas (us) between marks, per level.  usage: python tools/octree_profile.py [--pairs 64] [--seq [--first F]]
(--seq: the frames of the C3 tracking sequence, synth.StereoSequence, instead of synth.make_batch)"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--seq", action="store_true")
    ap.add_argument("--first", type=int, default=0, help="--seq: first frame")
    ap.add_argument("--lanes", type=int, default=1, help="orbfe_set_lanes chunks (1: one launch of all images)")
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd._lib import call
    if a.seq:
        sq = synth.StereoSequence(0, 1241, 376, 0.6)
        imgs = torch.from_numpy(np.stack([im for k in range(a.first, a.first + a.pairs) for im in sq.frame(k)])).cuda()
    else:
        imgs = torch.from_numpy(synth.make_batch(a.pairs)).cuda()
    fe = StereoFrontEnd(max_pairs=a.pairs, lanes=a.lanes)
    fe.enqueue(imgs)
    torch.cuda.synchronize()
    n = 2 * a.pairs * 8 * 64
    buf = np.zeros(n, np.int64)
    call("orbfe_debug_octree_profile", fe.handle, buf.ctypes.data_as(C.c_void_p), n)
    m = buf.reshape(2 * a.pairs, 8, 64).astype(np.float64) / 100.0  # us
    t0 = m[:, :, 0:1]
    for l in range(8):
        raw = {i: float(np.median(buf.reshape(2 * a.pairs, 8, 64)[:, l, i])) for i in range(40, 50)
               if (buf.reshape(2 * a.pairs, 8, 64)[:, l, i] > 0).any() and (buf.reshape(2 * a.pairs, 8, 64)[:, l, i] < 10000).all()}
        if raw:
            print(f"level {l} counters: " + " ".join(f"{i}:{v:.0f}" for i, v in raw.items()))
        ids = [i for i in range(64) if (m[:, l, i] > 0).all() and not (40 <= i < 50 and i in raw)]
        rel = {i: float(np.median(m[:, l, i] - m[:, l, 0])) for i in ids}
        print(f"level {l}: " + " ".join(f"{i}:{v:.1f}" for i, v in rel.items()))
    tot = m[:, :, 63] - m[:, :, 0]
    worst = np.argsort(tot.max(axis=1))[::-1][:4]
    print("per-image octree time (us), worst images:", {int(i): [round(float(v), 1) for v in tot[i]] for i in worst})
    start = m[:, :, 0]
    end = m[:, :, 63]
    print("block start spread (us):", float(start.max() - start.min()), " last end - first start:",
          float(end.max() - start.min()))


if __name__ == "__main__":
    main()
