"""Per-kernel micro-benchmark / ablation on one resident batch (development aid).
usage: python tools/microbench.py [--pairs 64] [--rounds 3] stage:variant ...   (stage 0 resize .. 4 stereo)"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("items", nargs="*", default=["0:0", "1:0", "2:0", "3:0", "4:0"])
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd._lib import call
    imgs = torch.from_numpy(synth.make_batch(a.pairs)).cuda()
    fe = StereoFrontEnd(max_pairs=a.pairs)
    fe.enqueue(imgs)
    torch.cuda.synchronize()
    res = {it: [] for it in a.items}
    for _ in range(a.rounds):
        for it in a.items:
            st, var = map(int, it.split(":"))
            ms = C.c_float()
            call("orbfe_microbench", fe.handle, st, var, a.reps, C.byref(ms))
            res[it].append(round(ms.value * 1000, 1))
            fe.enqueue(imgs)  # restore real stage outputs for the next item
            torch.cuda.synchronize()
    names = ["resize", "detect", "octree", "describe", "stereo", "blurwrite"]
    for it, v in res.items():
        st, var = map(int, it.split(":"))
        print(f"{names[st]:9s} v{var}: us per launch {v}  (min {min(v)})")
    print(json.dumps({k: min(v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
