#!/usr/bin/env python3
"""Benchmark: stereo pairs/s (ORB extract L + R + Frame.compute_stereo_matches), KITTI 1241x376.

Default (--mode throughput), the BASELINE.json metric:
  One step = one pass of the whole hot path over one batch of P synthetic stereo pairs resident in HBM
  (pyramid -> FAST cells -> octree -> IC angle + blur + rBRIEF for both images -> stereo match), as S
  independent handles of P/S pairs on S streams.  N GPUs: one process per GPU (torch.distributed.run),
  every rank processes its own P pairs (pairs are independent: weak scaling, no data-path collective);
  timing = barrier + synchronize on both sides of exactly K steps, max over ranks;
  value = N * P * K / max_elapsed.
  After the timed region (untimed): every handle's overflow word is read and the first and last pair of
  every handle are compared bit for bit with the oracle (parity on the bench's own workload); then a
  standalone pass runs the same P pairs as ONE handle on ONE stream with HIP events around each stage,
  which gives every stage's own duration for the roofline (no other handle's kernels overlap it).
  --gather adds a timed device-side gather of every pair's packed results to rank 0 (RCCL).

--mode frame: BASELINE config C3, the per-frame drop-in path (Tracking's calls per frame: Frame
  construction with the pair-batched ExtractORB / stereo, search_by_projection_f_f, _f_p) over the
  synthetic moving sequence of tests/golden/sequence_kitti_synth.npz, bit-exact against it, reported as
  frames/s and per-frame latency next to the reference's per-frame CPU time.

Prints ONE JSON line on rank 0 (fields: DESIGN.md §5).
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

VALU_PEAK_GIPS = 256 * 4 * 2.4 / 4  # wave64 VALU issue, all SIMDs at the 2.4 GHz peak clock
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
STAGES = ["resize", "detect", "octree", "blur", "describe", "stereo"]
STAGE_KERNELS = {"resize": "k_resize (x7 levels)", "detect": "k_detect", "octree": "k_octree", "blur": "(fused in k_orb)",
                 "describe": "k_orb (IC angle + per-keypoint 7x7 blur + steered BRIEF)",
                 "stereo": "k_stereo_bucket + k_stereo"}
CAMERAS = {(1241, 376): ("kitti", "KITTI 1241x376"), (752, 480): ("euroc", "EuRoC 752x480")}


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
        # fused into k_orb: no blurred level is written or read (kept as a 0-ms stage for the JSON layout)
        "blur": 0,
        # k_orb: each level's pixels around the keypoints (at most the level, read once) + the keypoint
        # records and descriptors written (24 + 32 B per keypoint)
        "describe": 2 * (px + N * 56),
        # both keypoint sets read + uR/depth written
        "stereo": 2 * N * 56 + N * 8,
    }
    total = 2 * (px + derived + 2 * N * 56) + N * 8
    return total, per_stage


# ------------------------------------------------------------------------------------------- cpu baseline
def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(seeds, width, height, nfeatures, barrier, queue):
    """Oracle extractor (C++ restatement, -O3) + the loop-faithful compute_stereo_matches restatement, 1
    thread: the reference's CPU path as far as it can run on this host."""
    from oracle.oracle import OracleExtractor
    from oracle.stereo_loop import compute_stereo_matches_loop
    from pyorbslam_amd import synth
    pairs = [synth.make_pair(s, width, height) for s in seeds]
    exL, exR = OracleExtractor(nfeatures=nfeatures), OracleExtractor(nfeatures=nfeatures)
    t = exL.tables()
    if barrier is not None:
        barrier.wait()
    t0 = time.perf_counter()
    t_ext = 0.0
    for L, R in pairs:
        a = time.perf_counter()
        kl, dl = exL.extract(L)
        kr, dr = exR.extract(R)
        t_ext += time.perf_counter() - a
        compute_stereo_matches_loop(kl, kr, dl, dr, exL.sheared_pyramid(), exR.sheared_pyramid(), t["scale"],
                                    t["inv_scale"], 386.1448, np.float32(718.856))
    dt = time.perf_counter() - t0
    if queue is not None:
        queue.put((len(pairs), dt, t_ext))
    return len(pairs), dt, t_ext


def cpu_baseline(sample_pairs: int, width: int, height: int, nfeatures: int, procs: int):
    """1 thread on `sample_pairs` pairs, then `procs` independent processes with 4 pairs each (all the
    host cores this job may use).  Runs BEFORE anything initialises the GPU (the pool forks)."""
    import multiprocessing as mp
    n1, t1, te1 = _cpu_worker([10_000 + i for i in range(sample_pairs)], width, height, nfeatures, None, None)
    out = {"value": None, "unit": "pairs/s", "cores": procs, "kind": "port",
           "value_1core": n1 / t1, "extract_s_per_pair_1core": te1 / n1, "stereo_s_per_pair_1core": (t1 - te1) / n1,
           "host_cpu": _cpu_model()}
    if procs > 1:
        ctx = mp.get_context("fork")
        barrier, queue = ctx.Barrier(procs), ctx.Queue()
        per = 4
        ps = [ctx.Process(target=_cpu_worker, args=([20_000 + per * i + j for j in range(per)], width, height, nfeatures,
                                                     barrier, queue)) for i in range(procs)]
        for p in ps:
            p.start()
        res = [queue.get() for _ in ps]
        for p in ps:
            p.join()
        out["value"] = sum(r[0] for r in res) / max(r[1] for r in res)
        allp = f"; {procs} processes x {per} pairs (seeds 20000..) concurrently for the all-cores value"
    else:
        out["value"] = out["value_1core"]
        allp = ""
    ratio = None
    f = ROOT / "profiles" / "cpu_ratio.json"
    if f.exists():
        ratio = json.loads(f.read_text())
        out["reference_over_port_stereo_ratio"] = round(ratio["ratio_reference_over_loop"], 4)
        out["ratio_measured_on"] = ratio["host"] + " (build container, tools/cpu_ratio.py)"
    out["sample"] = (f"{sample_pairs} synthetic {width}x{height} pairs (seeds 10000..), {nfeatures} features, 1 thread: "
                     f"oracle C++ extractor (orb_oracle.cpp, -O3 -march=x86-64-v3 -ffp-contract=off) + "
                     f"oracle/stereo_loop.py (per-candidate Python popcount and per-shift SAD like Frame.py:161-279), "
                     f"{t1:.1f} s{allp}")
    return out


# ------------------------------------------------------------------------------------------ parity check
def parity_check(fes, host, per, width, height, nfeatures):
    """First and last pair of every handle against the oracle extractor and the stereo restatement, bit for
    bit; every handle's overflow word.  Returns (pairs checked, max overflow word, failures)."""
    from oracle import stereo_oracle
    from oracle.oracle import OracleExtractor
    from pyorbslam_amd.batch import KITTI_BF, KITTI_FX
    from pyorbslam_amd.frame import to_reference_lists
    checked, ovf, bad = 0, 0, []
    oL, oR = OracleExtractor(nfeatures=nfeatures), OracleExtractor(nfeatures=nfeatures)
    t = oL.tables()
    for hi, f in enumerate(fes):
        ovf = max(ovf, f.overflow())
        for p in sorted({0, per - 1}):
            g = hi * per + p  # global pair index inside this rank's batch
            L, R = host[2 * g], host[2 * g + 1]
            kl, dl = oL.extract(L)
            kr, dr = oR.extract(R)
            gk, gd = f.fetch_image(2 * p)
            hk, hd = f.fetch_image(2 * p + 1)
            if gk.tobytes() != kl.tobytes() or not np.array_equal(gd, dl) or hk.tobytes() != kr.tobytes() \
                    or not np.array_equal(hd, dr):
                bad.append(f"handle {hi} pair {p}: extraction differs from the oracle")
                continue
            res = f.fetch_stereo(p)
            u, d = to_reference_lists(res, gk, KITTI_BF)
            ou, od, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, oL.sheared_pyramid(), oR.sheared_pyramid(),
                                                             t["scale"], t["inv_scale"], KITTI_BF, np.float32(KITTI_FX))
            for a, b in ((u, ou), (d, od)):
                sa, va = stereo_oracle.encode(a)
                sb, vb = stereo_oracle.encode(b)
                if not (np.array_equal(sa, sb) and np.array_equal(va, vb)):
                    bad.append(f"handle {hi} pair {p}: stereo differs from the restatement")
                    break
            checked += 1
    return checked, ovf, bad


# ---------------------------------------------------------------------------------------------- frame mode
def frame_mode(args):
    """C3: the per-frame drop-in path over the recorded synthetic sequence (tests/seq_harness.py)."""
    import torch
    assert torch.cuda.is_available(), "--mode frame needs a GPU"
    sys.path.insert(0, str(ROOT / "tests"))
    import seq_harness as H
    from pyorbslam_amd import frame as F
    from pyorbslam_amd import synth
    from pyorbslam_amd.matcher import ORBMatcher
    from pyorbslam_amd.pyORBExtractor import ORBextractor
    g = H.load_golden()
    meta = json.loads(str(g["meta"]))
    seq = synth.StereoSequence(meta["seq"]["seed"], meta["width"], meta["height"], meta["seq"]["speed"])
    frames = [seq.frame(k) for k in range(meta["n_frames"])]   # rendered before timing

    class Cached:
        def frame(self, k):
            return frames[k]

    class DropInFrame(H.SeqFrame):
        pass

    F.install(DropInFrame)
    ex = (ORBextractor(**H.PARAMS), ORBextractor(**H.PARAMS))
    for _ in range(max(args.warmup, 1)):
        H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, n_frames=3)
    reps = max(1, args.steps // meta["n_frames"]) if args.steps >= meta["n_frames"] else 1
    timer, bad = {}, []
    t0 = time.perf_counter()
    for _ in range(reps):
        bad += H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, timer=timer)
    wall = time.perf_counter() - t0
    if bad:
        print(json.dumps({"error": "frame-mode parity failure", "details": bad[:10]}), flush=True)
        raise SystemExit(2)
    fr, ff, fp = (np.array(timer[k]) for k in ("frame", "f_f", "f_p"))
    lat = fr + ff + fp
    nfr = len(lat)
    ref = meta["reference_seconds_per_frame"]
    ref_ext = None
    rf = ROOT / "profiles" / "cpu_ratio.json"
    if rf.exists():
        ref_ext = json.loads(rf.read_text())["oracle_extract_s_per_pair"]
    ref_frame = (ref_ext or 0.0) + ref["stereo"] + ref["grid"] + ref["f_f"] + ref["f_p"]
    out = {
        "metric": "frames/s (C3 per-frame drop-in: Frame(L,R) extract+stereo+grid, search_by_projection_f_f, _f_p)",
        "value": round(nfr / float(lat.sum()), 3), "unit": "frames/s", "n_gpus": 1, "steps": nfr, "warmup": args.warmup,
        "ms_per_step": round(1e3 * float(lat.mean()), 3), "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic moving stereo sequence (pyorbslam_amd.synth.StereoSequence seed 0), recorded map-point "
                "inputs of tests/golden/sequence_kitti_synth.npz",
        "config": {"workload": f"kitti{meta['width']}x{meta['height']}_seq{meta['n_frames']}f_2000f_tracking",
                   "frames": meta["n_frames"], "repeats": reps, "nfeatures": 2000},
        "parity": f"bit-exact vs the reference tracking-loop golden on all {nfr} frames",
        "latency_ms": {"p50": round(1e3 * float(np.median(lat)), 3), "p90": round(1e3 * float(np.percentile(lat, 90)), 3),
                       "max": round(1e3 * float(lat.max()), 3),
                       "frame_ctor_p50": round(1e3 * float(np.median(fr)), 3),
                       "f_f_p50": round(1e3 * float(np.median(ff[ff > 0])), 3) if (ff > 0).any() else 0.0,
                       "f_p_p50": round(1e3 * float(np.median(fp[fp > 0])), 3) if (fp > 0).any() else 0.0},
        "wall_s_incl_checks": round(wall, 3),
        "reference_cpu_s_per_frame": {"extract_LR_oracle_cpp": ref_ext, **{k: round(v, 5) for k, v in ref.items()},
                                      "total": round(ref_frame, 4), "host": meta["reference_timing_host"]},
        "speedup_vs_reference_frame": round(ref_frame / float(lat.mean()), 2),
    }
    print(json.dumps(out), flush=True)


# --------------------------------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["throughput", "frame"], default="throughput")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=512, help="stereo pairs per step per GPU (256: -1.7 %%, tools/dbg/pairs_sweep.sh)")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--streams", type=int, default=4,
                    help="independent front-end handles per GPU, each on its own stream with P/streams pairs")
    ap.add_argument("--lanes", type=int, default=1, help="internal concurrent chunks per handle (orbfe_set_lanes)")
    ap.add_argument("--cpu-sample", type=int, default=40,
                    help="pairs timed on 1 thread for cpu_baseline (0 = skip); the all-cores figure adds 4 per process")
    ap.add_argument("--cpu-procs", type=int, default=0, help="processes for the all-cores cpu_baseline (0 = this "
                    "job's CPU share, at most 16)")
    ap.add_argument("--no-parity", action="store_true", help="skip the untimed parity check of the bench workload")
    ap.add_argument("--roofline-steps", type=int, default=5, help="steps of the standalone per-stage pass (0 = skip)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the standalone per-stage pass (for rocprofv3 --pmc runs whose dispatches must all be "
                         "standalone)")
    ap.add_argument("--gather", action="store_true",
                    help="also time a device-side gather of every pair's packed results to rank 0 (RCCL)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.mode == "frame":
        frame_mode(args)
        return
    cpu = None
    if world == 1 and args.cpu_sample > 0 and not args.roofline_only:
        try:
            share = len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            share = os.cpu_count() or 1
        procs = args.cpu_procs or max(1, min(16, share))
        cpu = cpu_baseline(args.cpu_sample, args.width, args.height, args.nfeatures, procs)

    import torch
    import torch.distributed as dist

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
    per = P // S
    elapsed = None
    fes = []
    if not args.roofline_only:
        # S sub-batches of P/S pairs, each with its own handle (buffers) and stream, so that the latency-bound
        # stages of one overlap the issue-bound stages of another; every pair is still processed exactly once
        fes = [StereoFrontEnd(args.width, args.height, max_pairs=per, nfeatures=args.nfeatures, lanes=args.lanes) for _ in range(S)]
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
        subs = [images[2 * per * i: 2 * per * (i + 1)] for i in range(S)]

        def step():
            for f, st, sub in zip(fes, streams, subs):
                f.enqueue(sub, per, KITTI_BF, KITTI_FX, stream_ptr=st.cuda_stream)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
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
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64)
            t = t.to(dev) if dist.get_backend() == "nccl" else t
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())

    gather = None
    if args.gather and fes:
        from pyorbslam_amd import dist as D
        gather = D.timed_gather(fes, per, dev, world, rank, reps=3)

    # ---- parity of the bench's own workload (untimed)
    parity = None
    if fes and not args.no_parity:
        checked, ovf, bad = parity_check(fes, host, per, args.width, args.height, args.nfeatures)
        if world > 1:
            t = torch.tensor([len(bad), ovf, checked], dtype=torch.int64)
            t = t.to(dev) if dist.get_backend() == "nccl" else t
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            nbad, ovf, checked = (int(v) for v in t.tolist())
        else:
            nbad = len(bad)
        parity = {"parity_checked_pairs": checked, "overflow": ovf, "parity_failures": nbad}
        if nbad or ovf:
            if rank == 0:
                print(json.dumps({"error": "bench workload failed its parity check", "overflow": ovf,
                                  "details": bad[:10]}), flush=True)
            raise SystemExit(3)

    # ---- standalone per-stage pass: the same P pairs as one handle on one stream, HIP events per stage
    stage_ms = {}
    if args.roofline_steps > 0 and rank == 0:
        del fes
        torch.cuda.synchronize(dev)
        solo = StereoFrontEnd(args.width, args.height, max_pairs=P, nfeatures=args.nfeatures, lanes=1)
        st0 = torch.cuda.current_stream(dev)
        for _ in range(2):
            solo.enqueue(images, P, KITTI_BF, KITTI_FX, stream_ptr=st0.cuda_stream)
        torch.cuda.synchronize(dev)
        call("orbfe_profile_begin", solo.handle, args.roofline_steps)
        for _ in range(args.roofline_steps):
            solo.enqueue(images, P, KITTI_BF, KITTI_FX, stream_ptr=st0.cuda_stream)
        ms = (C.c_float * len(STAGES))()
        nb = C.c_int32()
        call("orbfe_profile_read", solo.handle, ms, C.byref(nb))
        stage_ms = {s: ms[i] / max(nb.value, 1) for i, s in enumerate(STAGES)}

    if rank == 0:
        total_b, per_stage_b = algorithmic_bytes_per_pair(args.width, args.height, args.nfeatures)
        cam, cam_name = CAMERAS.get((args.width, args.height), ("custom", f"{args.width}x{args.height}"))
        workload = f"{cam}{args.width}x{args.height}_synth_{args.nfeatures}f_{P}pairs"
        tr = None
        f = ROOT / "profiles" / "traffic.json"
        if f.exists():
            tr = json.loads(f.read_text()).get(workload + "_standalone")
        out = {"metric": f"stereo pairs/s (ORB extract L+R + stereo match), {cam_name}, 1/2/4/8 GPU"}
        if elapsed is not None:
            pairs_per_s = world * P * args.steps / elapsed
            out.update({"value": round(pairs_per_s, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
                        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4)})
        else:
            pairs_per_s = None
            out.update({"value": None, "unit": "pairs/s", "n_gpus": world, "steps": 0, "warmup": 0})
        out.update({
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded band-limited noise + rectangles, right = per-row-block disparity shift)",
            "config": {"workload": workload, "pairs_per_step_per_gpu": P, "width": args.width, "height": args.height,
                       "nfeatures": args.nfeatures, "nlevels": 8, "scaleFactor": 1.2, "iniThFAST": 20, "minThFAST": 7,
                       "parallelism": f"pairs sharded {world}-way (independent replicas, no data-path collective)",
                       "handles_per_gpu": S, "lanes_per_handle": args.lanes},
        })
        if parity is not None:
            out.update(parity)
        if stage_ms:
            dom = max(stage_ms, key=stage_ms.get)
            ach = {s: per_stage_b[s] * P / (stage_ms[s] * 1e-3) / 1e9 for s in STAGES
                   if stage_ms[s] > 0 and per_stage_b[s] > 0}
            out["stage_ms_standalone_step"] = {k: round(v, 4) for k, v in stage_ms.items()}
            out["roofline"] = {
                "bound": "hbm", "kernel": STAGE_KERNELS[dom], "stage": dom, "achieved": round(ach[dom], 3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach[dom] / HBM_PEAK_GBS, 6),
                "traffic": (tr or {}).get(dom),
                "measured": f"standalone pass: {P} pairs as one handle on one stream, HIP events around each stage, "
                            f"mean of {args.roofline_steps} steps (rocprof trace: the {2 * P}-image dispatches)",
                "algorithmic_bytes_per_pair": per_stage_b[dom], "pipeline_bytes_per_pair": total_b,
                "pipeline_frac": (round(pairs_per_s / world * total_b / (HBM_PEAK_GBS * 1e9), 6)
                                  if pairs_per_s else None)}
            out["stage_roofline"] = {s: {"ms": round(stage_ms[s], 4), "achieved_GBs": round(ach[s], 3),
                                         "frac": round(ach[s] / HBM_PEAK_GBS, 6), "traffic": (tr or {}).get(s)}
                                     for s in ach}
            # the bound these kernels actually meet: VALU issue (wave-instructions per step from
            # SQ_INSTS_VALU over the same standalone pass, profiles/valu.json, tools/valu.py)
            vf = ROOT / "profiles" / "valu.json"
            vi = json.loads(vf.read_text()).get(workload + "_standalone") if vf.exists() else None
            if vi:
                vst = {s: vi[s] / (stage_ms[s] * 1e-3) / 1e9 for s in vi if stage_ms.get(s, 0) > 0}
                vdom = max(vst, key=lambda s: stage_ms[s])
                out["valu_roofline"] = {
                    "bound": "valu", "unit": "G wave-instructions/s", "peak": VALU_PEAK_GIPS,
                    "peak_def": "256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 VALU instruction",
                    "kernel": STAGE_KERNELS[vdom], "achieved": round(vst[vdom], 2),
                    "frac": round(vst[vdom] / VALU_PEAK_GIPS, 4),
                    "stages": {s: {"inst_per_step": int(vi[s]), "achieved": round(v, 2),
                                   "frac": round(v / VALU_PEAK_GIPS, 4)} for s, v in vst.items()},
                    "pipeline_frac": (round(sum(vi.values()) * pairs_per_s / world / P / 1e9 / VALU_PEAK_GIPS, 4)
                                      if pairs_per_s else None),
                    "source": "profiles/valu.json " + workload + "_standalone (rocprofv3 --pmc SQ_INSTS_VALU)"}
        if gather is not None:
            out["with_gather"] = gather
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
