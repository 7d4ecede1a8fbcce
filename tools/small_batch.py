"""Small-batch latency of the front-end: one rank's share of 8-way C4 (8 pairs) and the
per-frame pair path (orbfe_frame_extract, C3), with HIP graphs on and off.  Prints one JSON line.
usage: python tools/small_batch.py [--steps 200]"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--handles", default="1,2,4", help="handle counts to try (pairs split by dist.shard)")
    ap.add_argument("--graphs", default="0,1", help="graph settings to try")
    ap.add_argument("--no-frame", action="store_true")
    ap.add_argument("--lanes", default="1", help="orbfe_set_lanes settings to try (internal fork / join chunks)")
    a = ap.parse_args()
    import os
    from pyorbslam_amd.dist import shard
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.batch import StereoFrontEnd, KITTI_BF, KITTI_FX
    from pyorbslam_amd.pyORBExtractor import ORBextractor
    dev = torch.device("cuda", 0)
    out = {}
    imgs = torch.from_numpy(synth.make_batch(8, seed0=0)).to(dev)
    out["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    for graphs, handles, lanes in [(bool(int(g)), int(h), int(ln)) for g in a.graphs.split(",")
                                   for h in a.handles.split(",") for ln in a.lanes.split(",")]:
        if True:
            parts = [shard(8, handles, i) for i in range(handles)]
            fes = [StereoFrontEnd(max_pairs=n, lanes=lanes, graphs=graphs) for _, n in parts]
            sts = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(handles - 1)]

            def step():
                for (p0, n), f, s in zip(parts, fes, sts):
                    f.enqueue(imgs[2 * p0: 2 * (p0 + n)], n, stream_ptr=s.cuda_stream)
            for _ in range(10):
                step()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) / a.steps * 1e3
            # one step alone (queue empty before and after): its latency, not the pipelined rate
            lat = []
            for _ in range(50):
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                step()
                torch.cuda.synchronize(dev)
                lat.append(time.perf_counter() - t)
            out[f"pairs8_{handles}h{'' if lanes == 1 else f'_{lanes}lanes'}_graphs{int(graphs)}"] = {"ms_per_step": round(ms, 4),
                                                             "latency_ms_p50": round(1e3 * float(np.median(lat)), 4),
                                                             "pairs_per_s": round(8 / ms * 1e3, 1)}
            del fes
    L, R = synth.make_pair(3)
    for graphs in (() if a.no_frame else (False, True)):
        ex, er = ORBextractor(2000, 1.2, 8, 20, 7), ORBextractor(2000, 1.2, 8, 20, 7)
        call("orbfe_set_graphs", ex.handle, int(graphs))
        Lc, Rc = np.ascontiguousarray(L), np.ascontiguousarray(R)
        for pyr in (False, True):
            for _ in range(10):
                call("orbfe_frame_extract", ex.handle, Lc.ctypes.data, Rc.ctypes.data, 1241, 376, 1241, KITTI_BF,
                     float(np.float32(KITTI_FX)), int(pyr))
            ts = []
            for _ in range(100):
                t = time.perf_counter()
                call("orbfe_frame_extract", ex.handle, Lc.ctypes.data, Rc.ctypes.data, 1241, 376, 1241, KITTI_BF,
                     float(np.float32(KITTI_FX)), int(pyr))
                ts.append(time.perf_counter() - t)
            out[f"frame_extract_pyr{int(pyr)}_graphs{int(graphs)}_ms_p50"] = round(1e3 * float(np.median(ts)), 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
