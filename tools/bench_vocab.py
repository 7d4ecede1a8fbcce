"""Throughput of the BoW vocabulary descent (k_vocab_descend) on an ORBvoc-shaped tree.

ORBvoc.txt is not available offline, so the tree is a seeded complete k=10, L=6 tree (1 111 111 nodes,
tests/vocab_synth.make_full_tree).  Work: `frames` frames x `feats` descriptors, one launch per batch
(the device entry point, inputs resident in HBM), timed with HIP events on the launch stream; plus the
host entry point transform_many (H2D + launch + D2H + BowVector/FeatureVector assembly) end to end.
The CPU leg times the oracle's per-node numpy descent on a bounded sample.

  python tools/bench_vocab.py [--frames 64] [--feats 2000] [--reps 20]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--feats", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--levels-up", type=int, default=4)
    ap.add_argument("--cpu-sample", type=int, default=400)
    a = ap.parse_args()

    import torch
    import vocab_synth as VS
    from oracle.vocab_oracle import VocabOracle
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.vocabulary import TemplatedVocabulary

    t = VS.make_full_tree(seed=7, k=10, L=6)
    v = TemplatedVocabulary(k=10, L=6).from_arrays(t["parent"], t["is_leaf"], t["desc"], t["weight"])
    n = a.frames * a.feats
    q = VS.query_descriptors(t, 8, n)
    dq = torch.from_numpy(q).cuda()
    word = torch.empty(n, dtype=torch.int32, device="cuda")
    node = torch.empty(n, dtype=torch.int32, device="cuda")
    w = torch.empty(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()

    def launch():
        call("orbfe_vocab_transform_device", v._handle(), C.c_void_p(dq.data_ptr()), n, 6 - a.levels_up,
             C.c_void_p(word.data_ptr()), C.c_void_p(node.data_ptr()), C.c_void_p(w.data_ptr()),
             C.c_void_p(s.cuda_stream))

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        launch()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps

    # host entry point: per-frame python dicts like the reference returns
    frames = [q[i * a.feats:(i + 1) * a.feats] for i in range(a.frames)]
    v.transform_many(frames, a.levels_up)
    t0 = time.perf_counter()
    for _ in range(3):
        v.transform_many(frames, a.levels_up)
    host_ms = (time.perf_counter() - t0) / 3 * 1e3

    o = VocabOracle(t["parent"], t["is_leaf"], t["desc"], t["weight"], 6)
    hw, hn, hwt = (x.cpu().numpy() for x in (word, node, w))
    m = min(a.cpu_sample, n)
    t0 = time.perf_counter()
    for i in range(m):
        r = o.descend(q[i], 6 - a.levels_up)
        assert r == (int(hw[i]), int(hn[i]), float(hwt[i])), i
    cpu_s = (time.perf_counter() - t0) / m

    bytes_per = 6 * 10 * 48 + 32 + 16  # per descriptor: 6 levels x 10 children x (32 B desc + 16 B slot info)
    print(json.dumps({
        "metric": "vocabulary descents/s (k=10, L=6)", "descriptors": n, "frames": a.frames,
        "kernel_ms": round(ms, 4), "descents_per_s": round(n / (ms * 1e-3)),
        "frames_per_s_kernel": round(a.frames / (ms * 1e-3), 1),
        "host_transform_many_ms": round(host_ms, 2), "frames_per_s_host_api": round(a.frames / (host_ms * 1e-3), 1),
        "algorithmic_bytes_per_descent": bytes_per,
        "achieved_GBps_algorithmic": round(n * bytes_per / (ms * 1e-3) / 1e9, 1),
        "cpu_oracle_us_per_descent": round(cpu_s * 1e6, 1), "cpu_sample": m,
    }))


if __name__ == "__main__":
    main()
