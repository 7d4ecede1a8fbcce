"""Multi-GPU batched-frames mode: one process per GPU, stereo pairs sharded across ranks.

Pairs are independent (no cross-frame state in the front-end), so ranks exchange nothing on the data
path.  The north star's only collective — collecting every pair's keypoints, descriptors and stereo
results on rank 0 — is `gather_results`, a single gather of fixed-capacity byte records (RCCL over
xGMI with backend "nccl", gloo on CPU).  It is not part of the timed step.
"""
from __future__ import annotations

import numpy as np

from ._lib import KP_DTYPE


def shard(n_pairs: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of pairs owned by `rank`: (first pair, count).  Blocks differ by at most one."""
    base, extra = divmod(n_pairs, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def record_bytes(kp_cap: int) -> int:
    # count L, count R (i32) | kps L, R | desc L, R | uR, depth (f32) | status (i8), padded to 16 B
    raw = 8 + 2 * kp_cap * KP_DTYPE.itemsize + 2 * kp_cap * 32 + kp_cap * 8 + kp_cap
    return (raw + 15) // 16 * 16


def pack(kp_cap: int, kl, dl, kr, dr, stereo: dict) -> np.ndarray:
    rec = np.zeros(record_bytes(kp_cap), np.uint8)
    o = 0

    def put(arr):
        nonlocal o
        b = np.ascontiguousarray(arr).view(np.uint8).ravel()
        rec[o:o + b.size] = b
        return b.size

    o += put(np.array([len(kl), len(kr)], np.int32))
    for k in (kl, kr):
        put(k)
        o += kp_cap * KP_DTYPE.itemsize
    for d in (dl, dr):
        put(d.reshape(-1, 32) if d.size else np.zeros((0, 32), np.uint8))
        o += kp_cap * 32
    put(stereo["u_right"].astype(np.float32))
    o += kp_cap * 4
    put(stereo["depth"].astype(np.float32))
    o += kp_cap * 4
    put(stereo["status"].astype(np.int8))
    return rec


def unpack(kp_cap: int, rec: np.ndarray) -> dict:
    o = 0
    nl, nr = rec[0:8].view(np.int32).tolist()
    o = 8
    out = {}
    for name, n in (("kps_left", nl), ("kps_right", nr)):
        out[name] = rec[o:o + n * KP_DTYPE.itemsize].view(KP_DTYPE).copy()
        o += kp_cap * KP_DTYPE.itemsize
    for name, n in (("desc_left", nl), ("desc_right", nr)):
        out[name] = rec[o:o + n * 32].reshape(n, 32).copy()
        o += kp_cap * 32
    out["u_right"] = rec[o:o + nl * 4].view(np.float32).copy()
    o += kp_cap * 4
    out["depth"] = rec[o:o + nl * 4].view(np.float32).copy()
    o += kp_cap * 4
    out["status"] = rec[o:o + nl].view(np.int8).copy()
    return out


def gather_results(records: np.ndarray, n_pairs_total: int, device=None, dst: int = 0):
    """records: (local_pairs, record_bytes) uint8 of this rank.  Returns, on rank dst, the records of all
    pairs in global pair order (None elsewhere).  One collective: an all_gather of equal-size buffers
    (every rank pads to the largest shard), which both RCCL and gloo implement."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    rb = records.shape[1]
    maxn = shard(n_pairs_total, world, 0)[1]
    buf = np.zeros((maxn, rb), np.uint8)
    buf[:len(records)] = records
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    if rank != dst:
        return None
    full = []
    for r in range(world):
        _, n = shard(n_pairs_total, world, r)
        full.append(outs[r].cpu().numpy()[:n])
    return np.concatenate(full, axis=0)
