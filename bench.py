#!/usr/bin/env python3
"""Benchmark: stereo pairs/s (ORB extract L + R + Frame.compute_stereo_matches), KITTI 1241x376.

One step = one pass of the whole hot path over one batch of P synthetic stereo pairs resident in HBM
(pyramid -> FAST cells -> octree -> IC angle + blur + rBRIEF for both images -> stereo match).
N GPUs: one process per GPU (torch.distributed.run), every rank processes its own P pairs (pairs are
independent: weak scaling, no data-path collective); timing = barrier + synchronize on both sides of
exactly K steps, max over ranks; value = N * P * K / max_elapsed.

Prints ONE JSON line on rank 0 (see README / DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
STAGES = ["resize", "detect", "octree", "blur", "describe", "stereo"]


def level_sizes(W, H, nlevels=8, sf=1.2):
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(float(s[-1]) * float(np.float32(sf))))
    return [(int(np.rint(np.float32(W) * (np.float32(1) / x))), int(np.rint(np.float32(H) * (np.float32(1) / x))))
            for x in s]


def algorithmic_bytes_per_pair(W, H, N=2000, nlevels=8):
    """B = 2*(sum_l w_l h_l + sum_{l>=1} w_l h_l + 2*N*56) + N*8, split per stage."""
    ls = level_sizes(W, H, nlevels)
    px = sum(w * h for w, h in ls)
    derived = sum(w * h for w, h in ls[1:])
    per_stage = {
        # every derived level written once, its source level read once
        "resize": 2 * (derived + sum(w * h for w, h in ls[:-1])),
        # every level read once by the FAST cells
        "detect": 2 * px,
        # the selected keypoints (4 B packed) written and read back
        "octree": 2 * 2 * N * 4,
        # every level read once and its blurred copy written once
        "blur": 2 * 2 * px,
        # keypoint records + descriptors written (24 + 32 B per keypoint)
        "describe": 2 * N * 56,
        # both keypoint sets read + uR/depth written
        "stereo": 2 * N * 56 + N * 8,
    }
    total = 2 * (px + derived + 2 * N * 56) + N * 8
    return total, per_stage


def cpu_baseline(sample_pairs: int, width: int = 1241, height: int = 376, nfeatures: int = 2000):
    """Oracle extractor (C++ restatement, 1 thread) + numpy restatement of compute_stereo_matches on a
    bounded sample of the same synthetic workload, on this host."""
    from oracle.oracle import OracleExtractor
    from oracle import stereo_oracle
    from pyorbslam_amd import synth
    exL, exR = OracleExtractor(nfeatures=nfeatures), OracleExtractor(nfeatures=nfeatures)
    t = exL.tables()
    pairs = [synth.make_pair(10_000 + i, width, height) for i in range(sample_pairs)]
    t0 = time.perf_counter()
    for L, R in pairs:
        kl, dl = exL.extract(L)
        kr, dr = exR.extract(R)
        stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, exL.sheared_pyramid(), exR.sheared_pyramid(),
                                             t["scale"], t["inv_scale"], 386.1448, np.float32(718.856))
    dt = time.perf_counter() - t0
    return {"value": sample_pairs / dt, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{sample_pairs} synthetic {width}x{height} pairs, {nfeatures} features (seeds 10000..), "
                      f"oracle C++ extractor "
                      f"(orb_oracle.cpp, -O2, 1 thread) + numpy compute_stereo_matches restatement, {dt:.1f} s"}


def load_traffic(workload: str):
    f = ROOT / "profiles" / "traffic.json"
    if not f.exists():
        return None
    try:
        return json.loads(f.read_text()).get(workload)
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=256, help="stereo pairs per step per GPU")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--no-prof", action="store_true", help="no per-stage HIP events (roofline omitted)")
    ap.add_argument("--streams", type=int, default=4,
                    help="independent front-end handles per GPU, each on its own stream with P/streams pairs")
    ap.add_argument("--lanes", type=int, default=1, help="internal concurrent chunks per handle (orbfe_set_lanes)")
    ap.add_argument("--blur-fork", type=int, default=0,
                    help="k_blur on a side stream per handle (orbfe_set_blur_fork); off by default: the 4 handles "
                         "already fill the 4 hardware queues (GPU_MAX_HW_QUEUES), side streams would share them")
    ap.add_argument("--cpu-sample", type=int, default=64, help="pairs timed for cpu_baseline (0 = skip; 64 is about 15 s)")
    ap.add_argument("--check", action="store_true", help="verify the last step's pair 0 against the oracle")
    ap.add_argument("--gather", action="store_true",
                    help="after timing, gather every pair's results on rank 0 (dist.gather_results, untimed)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; the modulo only matters when rehearsing several ranks on one GPU (gloo)
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    if world > 1:
        torch.cuda.set_device(dev)
        backend = os.environ.get("ORBFE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from pyorbslam_amd import synth
    from pyorbslam_amd.batch import StereoFrontEnd, KITTI_BF, KITTI_FX
    from pyorbslam_amd._lib import call
    import ctypes as C

    P = args.pairs
    S = max(1, args.streams)
    if P % S:
        raise SystemExit("--pairs must be a multiple of --streams")
    host = synth.make_batch(P, seed0=rank * P, width=args.width, height=args.height)
    images = torch.from_numpy(host).to(dev)
    # S sub-batches of P/S pairs, each with its own handle (buffers) and stream, so that the latency-bound
    # stages of one overlap the issue-bound stages of another; every pair is still processed exactly once
    fes = [StereoFrontEnd(args.width, args.height, max_pairs=P // S, nfeatures=args.nfeatures, lanes=args.lanes,
                          blur_fork=bool(args.blur_fork))
           for _ in range(S)]
    fe = fes[0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    subs = [images[2 * (P // S) * i: 2 * (P // S) * (i + 1)] for i in range(S)]

    def step():
        for f, st, sub in zip(fes, streams, subs):
            f.enqueue(sub, P // S, KITTI_BF, KITTI_FX, stream_ptr=st.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # per-stage HIP events on handle 0's stream (its stages run concurrently with the other handles')
    prof = not args.no_prof
    if prof:
        call("orbfe_profile_begin", fe.handle, args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms = (C.c_float * len(STAGES))()
    nb = C.c_int32()
    if prof:
        call("orbfe_profile_read", fe.handle, ms, C.byref(nb))
        stage_ms = {s: ms[i] / max(nb.value, 1) for i, s in enumerate(STAGES)}
    else:
        stage_ms = {}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        t = t.to(dev) if dist.get_backend() == "nccl" else t
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    gather_s = None
    if args.gather and world > 1:
        from pyorbslam_amd import dist as D
        tg = time.perf_counter()
        recs = np.stack([D.pack(f.kp_cap, *f.fetch_image(2 * p), *f.fetch_image(2 * p + 1), f.fetch_stereo(p))
                         for f in fes for p in range(P // S)])
        allrec = D.gather_results(recs, world * P, device=dev if dist.get_backend() == "nccl" else None)
        gather_s = time.perf_counter() - tg
        if rank == 0:
            assert allrec.shape[0] == world * P

    if args.check:
        from oracle.oracle import OracleExtractor
        k, d = fe.fetch_image(0)
        ok, od = OracleExtractor(nfeatures=args.nfeatures).extract(host[0])
        assert k.tobytes() == ok.tobytes() and np.array_equal(d, od), "parity check failed"

    if rank == 0:
        pairs_per_s = world * P * args.steps / elapsed
        total_b, per_stage_b = algorithmic_bytes_per_pair(args.width, args.height, args.nfeatures)
        # handle 0 holds P/S pairs as min(lanes, P/S) concurrent chunks; its stage events bracket chunk 0
        chunk0 = (P // S) // max(1, min(args.lanes, P // S))
        dom = max(stage_ms, key=stage_ms.get) if stage_ms else "detect"
        ach = per_stage_b[dom] * chunk0 / (stage_ms[dom] * 1e-3) / 1e9 if stage_ms else 0.0
        cam = {(1241, 376): "kitti", (752, 480): "euroc"}.get((args.width, args.height), "custom")
        workload = f"{cam}{args.width}x{args.height}_synth_{args.nfeatures}f_{P}pairs"
        tr = load_traffic(workload)
        out = {
            "metric": "stereo pairs/s (ORB extract L+R + stereo match), KITTI 1241x376, 1/2/4/8 GPU",
            "value": round(pairs_per_s, 2),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded band-limited noise + rectangles, right = per-row-block disparity shift)",
            "config": {"workload": workload, "pairs_per_step_per_gpu": P, "width": args.width,
                       "height": args.height, "nfeatures": args.nfeatures, "nlevels": 8, "scaleFactor": 1.2,
                       "iniThFAST": 20, "minThFAST": 7, "parallelism": f"pairs sharded {world}-way (replicas)",
                       "handles_per_gpu": S, "lanes_per_handle": args.lanes,
                       "blur_side_stream": bool(args.blur_fork)},
            "stage_ms_per_step": {k: round(v, 4) for k, v in stage_ms.items()},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6),
                         "traffic": (tr or {}).get(dom),
                         "algorithmic_bytes_per_pair": per_stage_b[dom],
                         "pipeline_bytes_per_pair": total_b,
                         "pipeline_frac": round(pairs_per_s / world * total_b / (HBM_PEAK_GBS * 1e9), 6)},
        }
        # the same roofline figures for every stage (handle 0's events, 64-pair launches)
        out["stage_roofline"] = {
            st: {"ms": round(stage_ms[st], 4),
                 "achieved_GBs": round(per_stage_b[st] * chunk0 / (stage_ms[st] * 1e-3) / 1e9, 3),
                 "frac": round(per_stage_b[st] * chunk0 / (stage_ms[st] * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                 "traffic": (tr or {}).get(st)}
            for st in STAGES if stage_ms.get(st, 0) > 0}
        if gather_s is not None:
            out["gather_s_untimed"] = round(gather_s, 4)
        if world == 1 and args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.width, args.height, args.nfeatures)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
