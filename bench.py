#!/usr/bin/env python3
"""Benchmark: stereo pairs/s (ORB extract L + R + Frame.compute_stereo_matches), KITTI 1241x376.

Default (--mode throughput), the BASELINE.json metric:
  One step = one pass of the whole hot path over one batch of P synthetic stereo pairs resident in HBM
  (pyramid -> FAST cells -> octree -> IC angle + blur + rBRIEF for both images -> stereo match), as S
  independent handles of P/S pairs on S streams.  N GPUs: one process per GPU, every rank processes its
  own P pairs (pairs are independent: weak scaling, no data-path collective); timing = barrier +
  synchronize on both sides of exactly K steps, max over ranks; value = N * P * K / max_elapsed.
  --total-pairs T: strong scaling instead (config C4 is `--gpus 8 --total-pairs 64`): the T pairs are
  sharded over the ranks (dist.shard), value = T * K / max_elapsed.

  Launch: `python bench.py --gpus N` with N > 1 and no torch.distributed environment starts N ranks as
  fresh child processes (torch.distributed.run, before this process makes any GPU call) and exits with
  their status; under torchrun, WORLD_SIZE must equal --gpus (exit 2 otherwise).

  Beside `value` (never replacing it), each untimed or separately timed:
  * parity of the bench's own workload: every handle's overflow word, 64 pairs per rank (first, last and
    evenly spaced pairs of every handle) bit for bit against the oracle extractor and the stereo
    restatement (the oracle on a thread pool);
  * with_gather (N > 1): k_pack of every pair's record + one RCCL gather to rank 0, timed like a step;
  * c4_strong: the C4 configuration (64 pairs in total, sharded over the N ranks) timed like a step, plus
    its gather when N > 1, so every N of the driver's scaling run records the C4 curve;
  * host_fed: the same P pairs streamed from pinned host memory every step (H2D on a copy stream, double
    buffered against compute; packed records D2H), the PCIe-inclusive rate (stereo_kitti.py:39-47 reads
    images on the host);
  * a standalone pass (the same P pairs as ONE handle on ONE stream, HIP events around each stage) that
    gives every stage's own duration for the roofline; PMC-derived figures (traffic, VALU instructions)
    are taken from profiles/*.json only when they were measured on the loaded library's build id;
  * c3_frame (N = 1): BASELINE config C3, the per-frame drop-in tracking loop over the recorded synthetic
    sequence, bit-exact against its golden, p50 latency per frame;
  * cpu_baseline (N = 1, before any GPU call): the reference's CPU path as restated by the oracle.

--mode frame: C3 alone as its own JSON line.

Prints ONE JSON line on rank 0 (fields: DESIGN.md §5).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# wave64 VALU issue peak of the instruction class these kernels are made of: 4 cycles per wave64
# instruction per SIMD (packed 16-bit, dot2/dot4, perm, sad, alignbyte, shifts, integer multiply, max3 —
# ~70 % of their static VALU mix), 256 CUs x 4 SIMDs at the 2.4 GHz peak clock.  Measured per instruction:
# profiles/r03/mulrate_r3b.log (tools/dbg/mulrate.hip); the add / logic / mov / f32 add-mul class issues
# at ~2.4 cycles, so a kernel made only of those could exceed this figure.
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 4
VALU_PEAK_FAST_CLASS_GIPS = 256 * 4 * 2.4 / 2.4
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
PCIE_PEAK_GBS = 63.0   # MI355X_MICROARCH.md: PCIe Gen5 x16 spec, per direction
STAGES = ["resize", "detect", "octree", "describe", "stereo"]  # orbfe_profile_read order (ORBFE_NSTAGES)
STAGE_KERNELS = {"resize": "k_resize_rows (x7 levels)", "detect": "k_detect", "octree": "k_octree_bins",
                 "describe": "k_orb (IC angle + per-keypoint 7x7 blur + steered BRIEF; its first workgroups build "
                             "the stereo row buckets)",
                 "stereo": "k_stereo"}
CAMERAS = {(1241, 376): ("kitti", "KITTI 1241x376"), (752, 480): ("euroc", "EuRoC 752x480")}
C4_TOTAL_PAIRS = 64    # BASELINE.json configs[3]


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
        # k_orb: each level's pixels around the keypoints (at most the level, read once) + the keypoint
        # records and descriptors written (24 + 32 B per keypoint); the 7x7 blur is computed per keypoint
        "describe": 2 * (px + N * 56),
        # both keypoint sets read + uR/depth written
        "stereo": 2 * N * 56 + N * 8,
    }
    total = 2 * (px + derived + 2 * N * 56) + N * 8
    return total, per_stage


def shard(n, world, rank):
    base, extra = divmod(n, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


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


def cgroup_cpu_quota():
    """CPUs' worth of time the job's cgroup may use (cgroup v2 cpu.max, v1 cfs quota), None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def job_cpus() -> dict:
    """The host cores this job has: the CPUs in its affinity mask, capped by its cgroup's
    CPU quota when there is one — on the GPU box the mask holds all 256 hardware threads of the machine but
    cpu.max grants 16 CPUs' worth of time, so more processes than that only share those 16 (measured:
    profiles/r06/cpu_baseline_procs_r6.log)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    quota = cgroup_cpu_quota()
    cores = max(1, min(aff, int(math.ceil(quota))) if quota else aff)
    return {"cores": cores, "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "cores_rule": "min(affinity CPUs, cgroup CPU quota)"}


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
def parity_check(fes, counts, host, width, height, nfeatures, pairs_total=64, camera=None):
    """About `pairs_total` pairs of the timed batch (per handle: its first and last pair and evenly spaced
    ones between) against the oracle extractor and the stereo restatement, bit for bit; every handle's
    overflow word.  The device results are fetched first; the oracle runs on a thread pool (its C calls
    release the GIL and keep their state per thread).  Returns (pairs checked, max overflow word, failures)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import stereo_oracle
    from oracle.oracle import OracleExtractor
    from pyorbslam_amd.batch import camera_constants
    from pyorbslam_amd.frame import to_reference_lists
    bf, fx = camera or camera_constants(width, height)
    ovf, jobs = 0, []
    per = max(2, -(-pairs_total // max(len(fes), 1)))
    first = 0
    for hi, (f, n) in enumerate(zip(fes, counts)):
        ovf = max(ovf, f.overflow())
        for p in (np.unique(np.linspace(0, n - 1, min(per, n)).round().astype(int)).tolist() if n else []):
            g = first + p  # pair index inside this rank's batch
            jobs.append((hi, p, host[2 * g], host[2 * g + 1], f.fetch_image(2 * p), f.fetch_image(2 * p + 1),
                         f.fetch_stereo(p)))
        first += n

    def check(job):
        hi, p, L, R, (gk, gd), (hk, hd), res = job
        oL, oR = OracleExtractor(nfeatures=nfeatures), OracleExtractor(nfeatures=nfeatures)
        t = oL.tables()
        kl, dl = oL.extract(L)
        kr, dr = oR.extract(R)
        if gk.tobytes() != kl.tobytes() or not np.array_equal(gd, dl) or hk.tobytes() != kr.tobytes() \
                or not np.array_equal(hd, dr):
            return f"handle {hi} pair {p}: extraction differs from the oracle"
        u, d = to_reference_lists(res, gk, bf)
        ou, od, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, oL.sheared_pyramid(), oR.sheared_pyramid(),
                                                         t["scale"], t["inv_scale"], bf, np.float32(fx))
        for a, b in ((u, ou), (d, od)):
            sa, va = stereo_oracle.encode(a)
            sb, vb = stereo_oracle.encode(b)
            if not (np.array_equal(sa, sb) and np.array_equal(va, vb)):
                return f"handle {hi} pair {p}: stereo differs from the restatement"
        return None

    workers = job_cpus()["cores"]  # the job's host cores (affinity capped by the cgroup CPU quota)
    with ThreadPoolExecutor(workers) as ex:
        bad = [r for r in ex.map(check, jobs) if r is not None]
    return len(jobs), ovf, bad


# ---------------------------------------------------------------------------------------------- frame mode
def run_c3(steps: int, warmup: int) -> dict:
    """C3: the per-frame drop-in path over the recorded synthetic sequence (tests/seq_harness.py), bit-exact
    against its golden while timed."""
    import torch
    assert torch.cuda.is_available(), "C3 needs a GPU"
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
    for _ in range(max(warmup, 1)):
        H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, n_frames=3)
    reps = max(1, steps // meta["n_frames"]) if steps >= meta["n_frames"] else 1
    timer, bad = {}, []
    t0 = time.perf_counter()
    for _ in range(reps):
        bad += H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, timer=timer)
    wall = time.perf_counter() - t0
    fr, ff, fp = (np.array(timer[k]) for k in ("frame", "f_f", "f_p"))
    lat = fr + ff + fp
    nfr = len(lat)
    ref = meta["reference_seconds_per_frame"]
    ref_ext = None
    rf = ROOT / "profiles" / "cpu_ratio.json"
    if rf.exists():
        ref_ext = json.loads(rf.read_text())["oracle_extract_s_per_pair"]
    ref_frame = (ref_ext or 0.0) + ref["stereo"] + ref["grid"] + ref["f_f"] + ref["f_p"]
    return {
        "frames_per_s": round(nfr / float(lat.sum()), 3), "frames": nfr, "repeats": reps,
        "mean_ms": round(1e3 * float(lat.mean()), 3),
        "workload": f"kitti{meta['width']}x{meta['height']}_seq{meta['n_frames']}f_2000f_tracking",
        "parity": (f"bit-exact vs the reference tracking-loop golden on all {nfr} frames" if not bad
                   else f"FAILED: {bad[:5]}"),
        "parity_ok": not bad,
        "latency_ms": {"p50": round(1e3 * float(np.median(lat)), 3), "p90": round(1e3 * float(np.percentile(lat, 90)), 3),
                       "max": round(1e3 * float(lat.max()), 3),
                       "frame_ctor_p50": round(1e3 * float(np.median(fr)), 3),
                       "f_f_p50": round(1e3 * float(np.median(ff[ff > 0])), 3) if (ff > 0).any() else 0.0,
                       "f_p_p50": round(1e3 * float(np.median(fp[fp > 0])), 3) if (fp > 0).any() else 0.0},
        "wall_s_incl_checks": round(wall, 3),
        "reference_cpu_s_per_frame": {"extract_LR_oracle_cpp": ref_ext, **{k: round(v, 5) for k, v in ref.items()},
                                      "total": round(ref_frame, 4), "host": meta["reference_timing_host"]},
        "speedup_vs_reference_frame": round(ref_frame / float(lat.mean()), 2),
        "what": "Frame(L,R) (pair-batched ExtractORB + stereo + grid), search_by_projection_f_f, _f_p per frame; "
                "recorded map-point inputs of tests/golden/sequence_kitti_synth.npz",
    }


def frame_mode(args):
    c3 = run_c3(args.steps, args.warmup)
    if not c3["parity_ok"]:
        print(json.dumps({"error": "frame-mode parity failure", "details": c3["parity"]}), flush=True)
        raise SystemExit(2)
    out = {
        "metric": "frames/s (C3 per-frame drop-in: Frame(L,R) extract+stereo+grid, search_by_projection_f_f, _f_p)",
        "value": c3["frames_per_s"], "unit": "frames/s", "n_gpus": 1, "steps": c3["frames"], "warmup": args.warmup,
        "ms_per_step": c3["mean_ms"], "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic moving stereo sequence (pyorbslam_amd.synth.StereoSequence seed 0), recorded map-point "
                "inputs of tests/golden/sequence_kitti_synth.npz",
        "config": {"workload": c3["workload"], "frames": c3["frames"], "repeats": c3["repeats"], "nfeatures": 2000},
        **{k: c3[k] for k in ("parity", "latency_ms", "wall_s_incl_checks", "reference_cpu_s_per_frame",
                              "speedup_vs_reference_frame")},
    }
    print(json.dumps(out), flush=True)


# --------------------------------------------------------------------------------------- launch / ranks
def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) outside torchrun: start N ranks as fresh child processes through
    torch.distributed.run and return their exit status.  This process makes no GPU call (device_count
    does not initialise the GPU on this image), so no GPU context exists when the children start."""
    import torch
    backend = os.environ.get("ORBFE_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < args.gpus:
        print(json.dumps({"error": f"--gpus {args.gpus} needs {args.gpus} GPUs for one RCCL rank each; this host "
                                   f"shows {ndev} (ORBFE_DIST_BACKEND=gloo rehearses several ranks on one GPU)"}),
              flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_world(args) -> tuple[int, int, int] | None:
    """(world, rank, local rank) of this process, or None when it must launch the ranks itself.  Exits 2
    when a torch.distributed environment disagrees with --gpus."""
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(json.dumps({"error": f"WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a "
                                       f"{world}-rank run as {args.gpus} GPUs"}), flush=True)
            raise SystemExit(2)
        return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1:
        return None
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    return 1, 0, 0


# ------------------------------------------------------------------------------------------ the workload
class Shard:
    """This rank's pairs as S handles on S streams (pairs split evenly, dist.shard), each enqueue of the
    whole front-end on its own stream so that the latency-bound stages of one overlap the issue-bound
    stages of another; every pair is processed exactly once per step."""

    def __init__(self, images, n_pairs, streams, dev, width, height, nfeatures, lanes=1, camera=None):
        import torch
        from pyorbslam_amd.batch import StereoFrontEnd, camera_constants
        self.bf, self.fx = camera or camera_constants(width, height)
        # at least 3 pairs per handle: a one-rank share of 8-way C4 (8 pairs) runs 0.136 ms per step as 3 handles,
        # 0.141 as 2 and, depending on how the 4 streams land on the hardware queues, 0.135-0.30 as 4
        # (tools/small_batch.py, round 5): tiny handles only add latency-bound launches
        S = max(1, min(streams, -(-n_pairs // 3)))
        self.counts = [shard(n_pairs, S, i)[1] for i in range(S)]
        self.fes = [StereoFrontEnd(width, height, max_pairs=max(c, 1), nfeatures=nfeatures, lanes=lanes)
                    for c in self.counts]
        self.streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
        self.subs, o = [], 0
        for c in self.counts:
            self.subs.append(images[2 * o: 2 * (o + c)])
            o += c
        self.n_pairs = n_pairs

    def step(self, subs=None):
        for f, st, sub, c in zip(self.fes, self.streams, subs or self.subs, self.counts):
            if c:
                f.enqueue(sub, c, self.bf, self.fx, stream_ptr=st.cuda_stream)


def timed(fn, steps, warmup, dev, world):
    """warmup untimed calls, then exactly `steps` calls bracketed by barrier + synchronize on both sides;
    max over ranks of the elapsed seconds."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, dev, world)


def max_over_ranks(v, dev, world):
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64)
    t = t.to(dev) if dist.get_backend() == "nccl" else t
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_fed(sh: Shard, host, dev, world, steps, warmup, zero_copy: bool = False, h2d_streams: int = 1,
             records: bool = True) -> dict:
    """The shard's pairs streamed from pinned host memory every step, per handle: its images H2D on a copy
    stream into one of two device buffers (the handle starts as soon as ITS chunk has landed, while the
    next chunks are still on the link), its batch, and its pairs' records back in pinned host memory:
    packed into device memory and copied D2H on a second copy stream (default), or with zero_copy k_pack
    writes them straight into the pinned buffer over PCIe — measured slower, 47.3 k vs 51.1 k pairs/s
    same-box (round 4): the CUs' PCIe stores slow the H2D copies more than a copy-engine transfer does.  Timed like a step
    (barrier + synchronize, max over ranks); the records of the last step are checked against the handles'
    own results."""
    import torch
    from pyorbslam_amd import dist as D
    from pyorbslam_amd._lib import call
    n = sh.n_pairs
    H = len(sh.fes)
    hin = torch.from_numpy(host).pin_memory()
    dbuf = [torch.empty(hin.shape, dtype=torch.uint8, device=dev) for _ in range(2)]
    # compact records (k_pack_compact, 8 + 91 kp_cap bytes instead of 8 + 121 kp_cap) on the copy path;
    # the zero-copy variant writes full records (k_pack accepts page-locked host memory)
    kc = sh.fes[0].kp_cap
    rb = D.record_bytes(kc) if zero_copy else D.compact_record_bytes(kc)
    pack_fn = "orbfe_batch_pack_device" if zero_copy else "orbfe_batch_pack_compact_device"
    drec = [] if zero_copy else [torch.empty((n, rb), dtype=torch.uint8, device=dev) for _ in range(2)]
    hrec = [torch.empty((n, rb), dtype=torch.uint8).pin_memory() for _ in range(2)]
    h2ds = [torch.cuda.Stream(dev) for _ in range(max(1, h2d_streams))]  # handle j's images on h2ds[j % n]
    d2h = torch.cuda.Stream(dev)
    ev = {name: [[torch.cuda.Event() for _ in range(H)] for _ in range(2)] for name in ("in", "free", "out")}
    offs = np.concatenate([[0], np.cumsum(sh.counts)]).tolist()
    it = [0]
    seen = [False, False]  # buffer b has been used once: its events were recorded

    def step():
        b = it[0] % 2
        it[0] += 1
        for j, (f, st, c) in enumerate(zip(sh.fes, sh.streams, sh.counts)):
            o0, o1 = offs[j], offs[j + 1]
            h2d = h2ds[j % len(h2ds)]
            with torch.cuda.stream(h2d):
                if seen[b]:
                    h2d.wait_event(ev["free"][b][j])   # handle j finished reading dbuf[b] two steps ago
                dbuf[b][2 * o0:2 * o1].copy_(hin[2 * o0:2 * o1], non_blocking=True)
                ev["in"][b][j].record(h2d)
            st.wait_event(ev["in"][b][j])
            if seen[b] and not zero_copy and records:
                st.wait_event(ev["out"][b][j])         # drec[b] rows of handle j have left the device
            f.enqueue(dbuf[b][2 * o0:2 * o1], c, sh.bf, sh.fx, stream_ptr=st.cuda_stream)
            if records:
                dst = hrec[b][o0] if zero_copy else drec[b][o0]
                call(pack_fn, f.handle, C.c_void_p(dst.data_ptr()), rb, 0, c, C.c_void_p(st.cuda_stream))
            ev["free"][b][j].record(st)
            if not zero_copy and records:
                with torch.cuda.stream(d2h):
                    d2h.wait_event(ev["free"][b][j])
                    hrec[b][o0:o1].copy_(drec[b][o0:o1], non_blocking=True)
                    ev["out"][b][j].record(d2h)
        seen[b] = True

    el = timed(step, steps, warmup, dev, world)
    if not records:  # the images' H2D leg and the compute only: what the link allows without the results
        return {"value": round(world * n * steps / el, 2), "unit": "pairs/s", "ms_per_step": round(el / steps * 1e3, 4),
                "h2d_GBs_per_gpu": round(host.nbytes * steps / el / 1e9, 2)}
    last = (it[0] - 1) % 2
    r0 = hrec[last][0].numpy()
    u = D.unpack(kc, r0) if zero_copy else D.unpack_compact(kc, r0, sh.fes[0].scales)
    k, d = sh.fes[0].fetch_image(0)
    kr, dr = sh.fes[0].fetch_image(1)
    s = sh.fes[0].fetch_stereo(0)
    ok = (u["kps_left"].tobytes() == k.tobytes() and np.array_equal(u["desc_left"], d)
          and u["kps_right"].tobytes() == kr.tobytes() and np.array_equal(u["desc_right"], dr)
          and np.array_equal(u["u_right"], s["u_right"]) and np.array_equal(u["depth"], s["depth"])
          and np.array_equal(u["status"], s["status"]))
    if not ok:
        raise RuntimeError("host-fed record of pair 0 differs from the handle's own results")
    in_b = host.nbytes
    out_b = n * rb
    pps = world * n * steps / el
    return {"value": round(pps, 2), "unit": "pairs/s", "ms_per_step": round(el / steps * 1e3, 4),
            "h2d_bytes_per_pair": int(in_b // n), "d2h_bytes_per_pair": int(rb),
            "h2d_GBs_per_gpu": round(in_b * steps / el / 1e9, 2), "d2h_GBs_per_gpu": round(out_b * steps / el / 1e9, 2),
            "pcie_bound_pairs_per_s_per_gpu": round(PCIE_PEAK_GBS * 1e9 / (in_b / n), 1),
            "record_check": ok,
            "records": "k_pack into pinned host memory" if zero_copy else "k_pack_compact + D2H copy (compact records)",
            "h2d_streams": len(h2ds),
            "what": "per handle: its images H2D from pinned host memory (copy stream, two device buffers), its batch, "
                    "its pairs' records packed " + ("by k_pack straight into pinned host memory (zero-copy stores over "
                                                    "PCIe)" if zero_copy else "on the device and copied D2H (second "
                                                                               "copy stream)")
                    + "; chunks of later handles stream while earlier handles compute; PCIe Gen5 x16 spec 63 GB/s per "
                      "direction bounds the H2D leg (tools/dbg/pcie_probe.py measured 57 GB/s H2D alone, 45 GB/s with "
                      "a D2H copy running)"}


# ----------------------------------------------------------------------------------- evidence lookups
def stamped(name: str, key: str, build: str):
    """profiles/<name>.json entry `key` if it was measured on library build `build`, else (None, reason)."""
    f = ROOT / "profiles" / name
    if not f.exists():
        return None, f"profiles/{name} absent"
    data = json.loads(f.read_text())
    if key not in data:
        return None, f"no {key} entry in profiles/{name}"
    meta = data.get(key + "_meta", {})
    if meta.get("build_id") != build:
        return None, (f"profiles/{name} {key} was measured on build {meta.get('build_id', 'unstamped')}, "
                      f"the loaded library is {build}: dropped")
    return data[key], f"profiles/{name} {key} (build {build}, git {meta.get('git_rev', '?')})"


# ----------------------------------------------------------------------------- standalone pass / roofline
def standalone_stages(images, P, width, height, nfeatures, steps, dev) -> dict:
    """The P pairs as ONE handle on ONE stream (stream path: profiling events between the stages), mean ms
    per stage over `steps` batches."""
    import torch
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.batch import StereoFrontEnd, camera_constants
    bf, fx = camera_constants(width, height)
    torch.cuda.synchronize(dev)
    solo = StereoFrontEnd(width, height, max_pairs=P, nfeatures=nfeatures, lanes=1)
    st0 = torch.cuda.current_stream(dev)
    for _ in range(2):
        solo.enqueue(images, P, bf, fx, stream_ptr=st0.cuda_stream)
    torch.cuda.synchronize(dev)
    call("orbfe_profile_begin", solo.handle, steps)
    for _ in range(steps):
        solo.enqueue(images, P, bf, fx, stream_ptr=st0.cuda_stream)
    ms = (C.c_float * len(STAGES))()
    nb = C.c_int32()
    call("orbfe_profile_read", solo.handle, ms, C.byref(nb))
    del solo
    return {s: ms[i] / max(nb.value, 1) for i, s in enumerate(STAGES)}


def roofline_block(stage_ms: dict, P: int, width: int, height: int, nfeatures: int, workload: str, build: str,
                   pairs_per_s_per_gpu, steps: int) -> dict:
    """roofline (the largest standalone stage against HBM), stage_roofline, valu_roofline: PMC figures only
    from profiles/*.json entries stamped with the loaded library's build id."""
    out = {}
    total_b, per_stage_b = algorithmic_bytes_per_pair(width, height, nfeatures)
    tr, tr_src = stamped("traffic.json", workload + "_standalone", build)
    dom = max(stage_ms, key=stage_ms.get)
    ach = {s: per_stage_b[s] * P / (stage_ms[s] * 1e-3) / 1e9 for s in STAGES
           if stage_ms[s] > 0 and per_stage_b[s] > 0}
    out["stage_ms_standalone_step"] = {k: round(v, 4) for k, v in stage_ms.items()}
    out["roofline"] = {
        "bound": "hbm", "kernel": STAGE_KERNELS[dom], "stage": dom, "achieved": round(ach[dom], 3),
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach[dom] / HBM_PEAK_GBS, 6),
        "traffic": (tr or {}).get(dom), "traffic_source": tr_src,
        "measured": f"standalone pass: {P} pairs as one handle on one stream, HIP events around each stage, "
                    f"mean of {steps} steps (rocprof trace: the {2 * P}-image dispatches)",
        "algorithmic_bytes_per_pair": per_stage_b[dom], "pipeline_bytes_per_pair": total_b,
        "pipeline_frac": (round(pairs_per_s_per_gpu * total_b / (HBM_PEAK_GBS * 1e9), 6)
                          if pairs_per_s_per_gpu else None)}
    out["stage_roofline"] = {s: {"ms": round(stage_ms[s], 4), "achieved_GBs": round(ach[s], 3),
                                 "frac": round(ach[s] / HBM_PEAK_GBS, 6), "traffic": (tr or {}).get(s)}
                             for s in ach}
    # the bound these kernels actually meet: VALU issue (wave-instructions per step from SQ_INSTS_VALU over
    # the same standalone pass, profiles/valu.json, tools/valu.py); busy-cycle counters beside it
    vi, vi_src = stamped("valu.json", workload + "_standalone", build)
    if vi:
        inst = {k: v for k, v in vi.items() if k in STAGES}
        vst = {s: inst[s] / (stage_ms[s] * 1e-3) / 1e9 for s in inst if stage_ms.get(s, 0) > 0}
        vdom = max(vst, key=lambda s: stage_ms[s])
        out["valu_roofline"] = {
            "bound": "valu", "unit": "G wave-instructions/s", "peak": VALU_PEAK_GIPS,
            "peak_def": "256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction of the packed-16-bit / "
                        "dot / perm / sad / shift / multiply class; the add / logic / mov class issues at ~2.4 "
                        f"cycles ({VALU_PEAK_FAST_CLASS_GIPS:.0f} G/s): a class-peak fraction, see busy",
            "kernel": STAGE_KERNELS[vdom], "achieved": round(vst[vdom], 2),
            "frac": round(vst[vdom] / VALU_PEAK_GIPS, 4),
            "stages": {s: {"inst_per_step": int(inst[s]), "achieved": round(v, 2),
                           "frac": round(v / VALU_PEAK_GIPS, 4)} for s, v in vst.items()},
            "pipeline_frac": (round(sum(inst.values()) * pairs_per_s_per_gpu / P / 1e9 / VALU_PEAK_GIPS, 4)
                              if pairs_per_s_per_gpu else None),
            "source": vi_src + " (rocprofv3 --pmc SQ_INSTS_VALU)"}
        if "busy" in vi:  # per-stage VALU-busy fraction from the busy-cycle pass (tools/valu.py)
            out["valu_roofline"]["valu_busy"] = {s: b.get("valu_busy") for s, b in vi["busy"].items()}
            out["valu_roofline"]["valu_busy_def"] = ("4 x SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): "
                                                     "share of SIMD cycles issuing VALU, same standalone pass")
    else:
        out["valu_roofline"] = {"dropped": vi_src}
    return out


def workload_name(width, height, nfeatures, P, total_pairs=0):
    cam, _ = CAMERAS.get((width, height), ("custom", f"{width}x{height}"))
    return f"{cam}{width}x{height}_synth_{nfeatures}f_" + (f"{total_pairs}pairs_total" if total_pairs else f"{P}pairs")


def c5_euroc(args, dev) -> dict:
    """BASELINE configs[4]: EuRoC 752x480, 1000 features, 512 pairs per step on this GPU (the default bench
    step's handles and streams), timed like the headline; its own parity sample (64 pairs against the
    oracle) and its standalone per-stage roofline from the build-stamped EuRoC PMC entries."""
    import torch
    from pyorbslam_amd import synth
    W, H, N, P = 752, 480, 1000, args.pairs
    host = synth.make_batch(P, seed0=0, width=W, height=H)
    images = torch.from_numpy(host).to(dev)
    sh = Shard(images, P, args.streams, dev, W, H, N, args.lanes)
    el = timed(sh.step, args.steps, args.warmup, dev, 1)
    checked, ovf, bad = parity_check(sh.fes, sh.counts, host, W, H, N, args.parity_pairs)
    pps = P * args.steps / el
    wl = workload_name(W, H, N, P)
    out = {"value": round(pps, 2), "unit": "pairs/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "steps": args.steps, "warmup": args.warmup, "workload": wl, "pairs_per_step": P, "nfeatures": N,
           "handles": len(sh.fes), "parity_checked_pairs": checked, "overflow": ovf, "parity_failures": len(bad)}
    del sh
    if args.roofline_steps > 0:
        stage_ms = standalone_stages(images, P, W, H, N, args.roofline_steps, dev)
        from pyorbslam_amd import _lib
        out.update(roofline_block(stage_ms, P, W, H, N, wl, _lib.build_id(), pps, args.roofline_steps))
    if bad or ovf:
        out["details"] = bad[:5]
    return out


def rank_share_measure(args, dev) -> dict:
    """One rank's share of 8-way C4 (BASELINE configs[3]: 64 pairs over 8 GPUs = 8 pairs per GPU), timed like a
    step: the body of the `--rank-share-only` child process (c4_rank_share)."""
    import torch
    from pyorbslam_amd import synth
    first, n = shard(C4_TOTAL_PAIRS, 8, 0)
    host = synth.make_batch(n, seed0=first, width=args.width, height=args.height)
    images = torch.from_numpy(host).to(dev)
    sh = Shard(images, n, args.streams, dev, args.width, args.height, args.nfeatures, args.lanes)
    # ~0.15 ms steps: 400 of them (60 ms) after 50 warm-up steps, clocks and queues in steady state
    steps = max(args.steps, 400)
    el = timed(sh.step, steps, max(args.warmup, 50), dev, 1)
    ms = el / steps * 1e3
    checked, ovf, bad = parity_check(sh.fes, sh.counts, host, args.width, args.height, args.nfeatures, n)
    return {"pairs": n, "handles": len(sh.fes), "steps": steps, "ms_per_step": round(ms, 4),
            "value": round(n / (ms * 1e-3), 2), "unit": "pairs/s",
            "graphs": all(f.graph_stats()["launches"] > 0 for f in sh.fes),
            "parity_checked_pairs": checked, "parity_failures": len(bad), "overflow": ovf}


def c4_rank_share(args, c4_value) -> dict:
    """One rank's share of 8-way C4 on this GPU, measured in a fresh child process (`bench.py
    --rank-share-only`): a rank of an 8-GPU C4 run holds only its own 8 pairs' handles, and in this process,
    after the headline's, C4's and the host-fed handles and streams, the same 8-pair step read 0.166-0.25 ms
    against 0.14 alone (round 5).  The projected 8-GPU C4 rate is 64 pairs per rank-share step, its efficiency
    that against 8 x this GPU's whole-C4 rate (c4_strong)."""
    cmd = [sys.executable, str(Path(__file__).resolve()), "--rank-share-only", "--width", str(args.width), "--height",
           str(args.height), "--nfeatures", str(args.nfeatures), "--streams", str(args.streams), "--lanes",
           str(args.lanes), "--steps", str(args.steps), "--warmup", str(args.warmup)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        raise RuntimeError(f"rank-share child failed (exit {r.returncode}): {r.stderr[-2000:]}")
    out = json.loads(line[-1])
    ms = out["ms_per_step"]
    proj = C4_TOTAL_PAIRS / (ms * 1e-3)
    out.update({"projected_8gpu_c4_pairs_per_s": round(proj, 1),
                "projected_8way_efficiency": round(proj / (8 * c4_value), 4) if c4_value else None,
                "process": "fresh child (bench.py --rank-share-only)",
                "what": "8 pairs (one rank's share of 64 over 8 GPUs) on this GPU, timed like a step in a process of "
                        "their own; projected 8-way C4 rate = 64 / rank-share step time, efficiency = that / "
                        "(8 x c4_strong.value)"})
    return out


# --------------------------------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["throughput", "frame"], default="throughput")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=512, help="stereo pairs per step per GPU (weak scaling)")
    ap.add_argument("--total-pairs", type=int, default=0,
                    help="strong scaling: this many pairs per step in total, sharded over the GPUs (C4: 64)")
    ap.add_argument("--width", type=int, default=1241)
    ap.add_argument("--height", type=int, default=376)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--streams", type=int, default=4,
                    help="independent front-end handles per GPU, each on its own stream with P/streams pairs")
    ap.add_argument("--lanes", type=int, default=1, help="internal concurrent chunks per handle (orbfe_set_lanes)")
    ap.add_argument("--cpu-sample", type=int, default=40,
                    help="pairs timed on 1 thread for cpu_baseline (0 = skip); the all-cores figure adds 4 per process")
    ap.add_argument("--cpu-procs", type=int, default=0, help="processes for the all-cores cpu_baseline (0 = the job's "
                    "host cores: its affinity CPUs capped by its cgroup CPU quota, job_cpus)")
    ap.add_argument("--no-parity", action="store_true", help="skip the untimed parity check of the bench workload")
    ap.add_argument("--parity-pairs", type=int, default=64,
                    help="pairs of the timed batch checked against the oracle after the timed region (per rank)")
    ap.add_argument("--roofline-steps", type=int, default=5, help="steps of the standalone per-stage pass (0 = skip)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the standalone per-stage pass (for rocprofv3 --pmc runs whose dispatches must all be "
                         "standalone)")
    ap.add_argument("--no-gather", action="store_true", help="skip the timed rank-0 gather (N > 1)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (64 pairs in total) line")
    ap.add_argument("--no-host-fed", action="store_true", help="skip the host-fed (PCIe-inclusive) line")
    ap.add_argument("--host-fed-h2d-streams", type=int, default=1, help="copy streams carrying the host-fed H2D chunks")
    ap.add_argument("--host-fed-zero-copy", action="store_true",
                    help="host-fed records written by k_pack straight into pinned host memory (default: device buffer "
                         "+ D2H copy)")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 tracking-loop latency (N = 1)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 EuRoC line (N = 1, KITTI runs only)")
    ap.add_argument("--allow-dev-env", action="store_true",
                    help="run with ORBFE_* development variables set (A/B of library builds); value is then null")
    ap.add_argument("--rank-share-only", action="store_true",
                    help="internal: measure C4's 8-pair rank share alone and print it (the c4_rank_share child)")
    args = ap.parse_args()

    # no development switch may change what is measured unnoticed: ORBFE_* variables other than the rank
    # backend choice are recorded in the line, and a run with one set prints no value
    orbfe_env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("ORBFE_")}
    dev_env = {k: v for k, v in orbfe_env.items() if k != "ORBFE_DIST_BACKEND"}
    if dev_env and not args.allow_dev_env:
        print(json.dumps({"error": f"ORBFE_* development variables set ({', '.join(dev_env)}): unset them (they select "
                                   "another library build; --allow-dev-env runs anyway and reports value null)"}),
              flush=True)
        raise SystemExit(2)
    wr = check_world(args)
    if wr is None:
        raise SystemExit(launch_ranks(args))
    world, rank, local = wr
    if args.mode == "frame":
        frame_mode(args)
        return
    if args.rank_share_only:
        import torch
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        print(json.dumps(rank_share_measure(args, dev)), flush=True)
        return
    extras = not args.roofline_only
    cpu = None
    if world == 1 and args.cpu_sample > 0 and extras:
        cpus = job_cpus()
        procs = args.cpu_procs or cpus["cores"]
        cpu = cpu_baseline(args.cpu_sample, args.width, args.height, args.nfeatures, procs)
        cpu.update({k: v for k, v in cpus.items() if k != "cores"})

    import torch
    import torch.distributed as dist

    # one process per GPU; the modulo only matters when rehearsing several ranks on one GPU (gloo)
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("ORBFE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from pyorbslam_amd import _lib, synth
    from pyorbslam_amd import dist as D

    strong = args.total_pairs > 0
    if strong:
        first, P = shard(args.total_pairs, world, rank)
        total = args.total_pairs
    else:
        first, P = rank * args.pairs, args.pairs
        total = world * args.pairs
    host = synth.make_batch(P, seed0=first, width=args.width, height=args.height)
    images = torch.from_numpy(host).to(dev)
    elapsed = None
    sh = None
    n_handles = 0
    if extras:
        sh = Shard(images, P, args.streams, dev, args.width, args.height, args.nfeatures, args.lanes)
        n_handles = len(sh.fes)
        elapsed = timed(sh.step, args.steps, args.warmup, dev, world)

    gather = None
    if extras and world > 1 and not args.no_gather:
        gather = D.timed_gather(sh.fes, sh.counts, dev, world, rank, max_local=shard(total, world, 0)[1])

    # ---- parity of the bench's own workload (untimed)
    parity = None
    if sh is not None and not args.no_parity:
        checked, ovf, bad = parity_check(sh.fes, sh.counts, host, args.width, args.height, args.nfeatures,
                                         args.parity_pairs)
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

    # ---- C4: 64 pairs in total sharded over the ranks, timed like a step (+ its gather when N > 1)
    c4 = None
    if extras and not strong and not args.no_c4:
        c4_first, c4_n = shard(C4_TOTAL_PAIRS, world, rank)
        c4_imgs = (images[: 2 * c4_n] if c4_n <= P else  # a small --pairs run: the shard needs its own pairs
                   torch.from_numpy(synth.make_batch(c4_n, seed0=c4_first, width=args.width, height=args.height)).to(dev))
        c4_sh = Shard(c4_imgs, c4_n, args.streams, dev, args.width, args.height, args.nfeatures)
        el4 = timed(c4_sh.step, args.steps, args.warmup, dev, world)
        c4 = {"total_pairs": C4_TOTAL_PAIRS, "pairs_per_gpu": c4_n, "handles_per_gpu": len(c4_sh.fes),
              "value": round(C4_TOTAL_PAIRS * args.steps / el4, 2), "unit": "pairs/s",
              "ms_per_step": round(el4 / args.steps * 1e3, 4), "scaling": "strong",
              "what": "BASELINE configs[3]: 64 synthetic pairs per step in total, sharded over the ranks (dist.shard), "
                      "barrier + synchronize around K steps, max over ranks"}
        if world > 1 and not args.no_gather:
            c4["with_gather"] = D.timed_gather(c4_sh.fes, c4_sh.counts, dev, world, rank,
                                               max_local=shard(C4_TOTAL_PAIRS, world, 0)[1])
        del c4_sh

    # ---- host-fed (PCIe-inclusive) rate of the same workload
    hf = None
    if extras and not args.no_host_fed:
        hf = host_fed(sh, host, dev, world, max(args.steps // 2, 4), 2, zero_copy=args.host_fed_zero_copy,
                      h2d_streams=args.host_fed_h2d_streams)
        hf["images_only"] = host_fed(sh, host, dev, world, max(args.steps // 2, 4), 2, records=False)

    # ---- C4's rank share (8 pairs) on this GPU, and C5 (EuRoC), N = 1
    share = None
    if extras and world == 1 and not strong and not args.no_c4:
        share = c4_rank_share(args, c4["value"] if c4 else None)
    c5 = None
    if extras and world == 1 and not strong and not args.no_c5 and (args.width, args.height) == (1241, 376):
        c5 = c5_euroc(args, dev)
        if c5["parity_failures"] or c5["overflow"]:
            print(json.dumps({"error": "C5 (EuRoC) workload failed its parity check", **c5}), flush=True)
            raise SystemExit(3)

    # ---- standalone per-stage pass: the same P pairs as one handle on one stream, HIP events per stage
    stage_ms = {}
    if args.roofline_steps > 0 and rank == 0:
        del sh
        stage_ms = standalone_stages(images, P, args.width, args.height, args.nfeatures, args.roofline_steps, dev)

    c3 = None
    if extras and world == 1 and not args.no_c3 and (ROOT / "tests" / "golden" / "sequence_kitti_synth.npz").exists():
        c3 = run_c3(0, 1)
        if not c3["parity_ok"]:
            print(json.dumps({"error": "C3 tracking-loop parity failure", "details": c3["parity"]}), flush=True)
            raise SystemExit(3)

    if rank == 0:
        build = _lib.build_id()
        cam, cam_name = CAMERAS.get((args.width, args.height), ("custom", f"{args.width}x{args.height}"))
        workload = workload_name(args.width, args.height, args.nfeatures, P, args.total_pairs if strong else 0)
        out = {"metric": f"stereo pairs/s (ORB extract L+R + stereo match), {cam_name}, 1/2/4/8 GPU"}
        if elapsed is not None and not dev_env:
            pairs_per_s = total * args.steps / elapsed
            out.update({"value": round(pairs_per_s, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
                        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4)})
        else:
            pairs_per_s = None
            out.update({"value": None, "unit": "pairs/s", "n_gpus": world, "steps": 0, "warmup": 0})
        out.update({
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded band-limited noise + rectangles, right = per-row-block disparity shift)",
            "config": {"workload": workload, "pairs_per_step_per_gpu": P, "total_pairs_per_step": total,
                       "width": args.width, "height": args.height,
                       "nfeatures": args.nfeatures, "nlevels": 8, "scaleFactor": 1.2, "iniThFAST": 20, "minThFAST": 7,
                       "parallelism": (f"{total} pairs sharded {world}-way" if strong else
                                       f"{P} pairs per GPU on {world} GPU(s)")
                       + " (independent ranks, no data-path collective)",
                       "handles_per_gpu": n_handles, "lanes_per_handle": args.lanes},
            "build_id": build, "orbfe_env": orbfe_env,
        })
        if dev_env and elapsed is not None:
            out["dev_env_ms_per_step"] = round(elapsed / args.steps * 1e3, 4)
        if parity is not None:
            out.update(parity)
        if stage_ms:
            out.update(roofline_block(stage_ms, P, args.width, args.height, args.nfeatures, workload, build,
                                      pairs_per_s / world if pairs_per_s else None, args.roofline_steps))
        if gather is not None:
            out["with_gather"] = gather
        if c4 is None and strong and args.total_pairs == C4_TOTAL_PAIRS and pairs_per_s is not None:
            # --total-pairs 64 IS C4: its line under the same key as the weak-scaling run's C4 block
            c4 = {"total_pairs": C4_TOTAL_PAIRS, "pairs_per_gpu": P, "handles_per_gpu": n_handles,
                  "value": out["value"], "unit": "pairs/s", "ms_per_step": out["ms_per_step"], "scaling": "strong",
                  "what": "BASELINE configs[3]: this run's own step (--total-pairs 64, sharded over the ranks)"}
            if gather is not None:
                c4["with_gather"] = gather
        if c4 is not None:
            out["c4_strong"] = c4
        if share is not None:
            out["c4_rank_share"] = share
        if c5 is not None:
            out["c5_euroc"] = c5
        if hf is not None:
            out["host_fed"] = hf
        if c3 is not None:
            out["c3_frame"] = {k: c3[k] for k in ("frames_per_s", "frames", "latency_ms", "parity", "workload",
                                                  "speedup_vs_reference_frame", "what")}
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
