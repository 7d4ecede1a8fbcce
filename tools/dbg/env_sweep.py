"""Sweep of a per-handle tuning variable read when a handle is created or reserved (ORBFE_PRIO: wave
priorities r,d,o,k,b,s; ORBFE_STAGE_REPEAT: launches per stage r,d,o,k,s; ORBFE_OCT_KEYS ...) on the default
4-handle bench step, one process, configurations interleaved over several rounds.
usage: python tools/dbg/env_sweep.py [--var ORBFE_PRIO] [--rounds 3] CFG [CFG ...]
       CFG: digits joined with commas (002000 -> "0,0,2,0,0,0"), or any string after "=" (=7424)"""
import argparse
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--var", default="ORBFE_PRIO")
    ap.add_argument("--pairs", type=int, default=512)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("cfgs", nargs="+")
    a = ap.parse_args()
    import torch
    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd
    dev = torch.device("cuda", 0)
    images = torch.from_numpy(synth.make_batch(a.pairs)).to(dev)
    per = a.pairs // a.streams
    subs = [images[2 * per * i: 2 * per * (i + 1)] for i in range(a.streams)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(a.streams - 1)]
    res = {c: [] for c in a.cfgs}
    for r in range(a.rounds):
        for c in a.cfgs:
            os.environ[a.var] = c[1:] if c.startswith("=") else ",".join(c)
            fes = [StereoFrontEnd(max_pairs=per, lanes=1) for _ in range(a.streams)]

            def step():
                for f, st, sub in zip(fes, streams, subs):
                    f.enqueue(sub, per, stream_ptr=st.cuda_stream)

            for _ in range(5):
                step()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            v = a.pairs * a.steps / dt
            res[c].append(v)
            print(f"round {r} {a.var} {c}: {v:.0f} pairs/s ({1e3 * dt / a.steps:.3f} ms/step)", flush=True)
            del fes
    for c, v in res.items():
        print(f"{a.var} {c}: median {sorted(v)[len(v) // 2]:.0f} pairs/s  all {[round(x) for x in v]}")


if __name__ == "__main__":
    main()
