"""Workload for a rocprofv3 kernel trace of the small-batch front-end (one handle, one stream): `--pairs P`
pairs per step (8 = one rank's share of 8-way C4, 1 = the C3 frame pair), `--steps K` back-to-back steps
after 5 untimed ones; with --frame the per-frame drop-in path (orbfe_frame_extract) instead.
usage: rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/small_trace.py --pairs 8 --steps 50
Analyse with tools/ktrace_steps.py OUT (per-step span, kernel time, gaps)."""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--graphs", type=int, default=1)
    ap.add_argument("--frame", action="store_true")
    ap.add_argument("--handles", type=int, default=1, help="the pairs split over this many handles / streams")
    ap.add_argument("--pyramid", type=int, default=0, help="--frame: want_pyramid (the sheared views too)")
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.batch import StereoFrontEnd, KITTI_BF, KITTI_FX
    if a.frame:
        from pyorbslam_amd.pyORBExtractor import ORBextractor
        L, R = synth.make_pair(3)
        ex = ORBextractor(2000, 1.2, 8, 20, 7)
        call("orbfe_set_graphs", ex.handle, a.graphs)
        for k in range(5 + a.steps):
            call("orbfe_frame_extract", ex.handle, L.ctypes.data, R.ctypes.data, 1241, 376, 1241, KITTI_BF,
                 float(np.float32(KITTI_FX)), a.pyramid)
        return
    imgs = torch.from_numpy(synth.make_batch(a.pairs, seed0=0)).cuda()
    from pyorbslam_amd.dist import shard
    parts = [shard(a.pairs, a.handles, i) for i in range(a.handles)]
    fes = [StereoFrontEnd(max_pairs=n, lanes=1, graphs=bool(a.graphs)) for _, n in parts]
    sts = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(a.handles - 1)]
    for _ in range(5 + a.steps):
        for (p0, n), fe, st in zip(parts, fes, sts):
            fe.enqueue(imgs[2 * p0: 2 * (p0 + n)], n, stream_ptr=st.cuda_stream)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
