"""Multi-GPU batched-frames mode: one process per GPU, stereo pairs sharded across ranks.

Pairs are independent (no cross-frame state in the front-end), so ranks exchange nothing on the data
path.  The north star's only collective — collecting every pair's keypoints, descriptors and stereo
results on rank 0 — is one gather of fixed-capacity byte records (RCCL over xGMI with backend "nccl",
gloo on CPU): `pack_device` builds the records on the GPU with k_pack, `gather_records` gathers them,
`timed_gather` times both for bench.py --gather (reported next to, not inside, the timed step).
"""
from __future__ import annotations

import hashlib
import time

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


_GATHER_BUF: dict = {}


def compact_record_bytes(kp_cap: int) -> int:
    """orbfe_batch_pack_compact_device's record: 8 + 91 kp_cap bytes, padded to 16 (include/orbfe.h)."""
    return (8 + 91 * kp_cap + 15) // 16 * 16


def unpack_compact(kp_cap: int, rec: np.ndarray, scales) -> dict:
    """A compact record back to unpack()'s arrays, bit for bit: x = f32(level x) * scale[octave], size =
    (float)(int)(31 * scale[octave]) (ORBextractor.cpp:836, 1094-1099: what k_orb wrote), response = score;
    scales: the extractor's float32 scale factors (orbfe_get_scales)."""
    sc = np.asarray(scales, np.float32)
    size = np.array([float(int(np.float32(31) * v)) for v in sc], np.float32)
    nl, nr = rec[0:8].view(np.int32).tolist()
    out = {}
    o_kp, o_desc, o_st = 8, 8 + 16 * kp_cap, 8 + 80 * kp_cap
    for s, (name, n) in enumerate((("kps_left", nl), ("kps_right", nr))):
        kw = rec[o_kp + 8 * kp_cap * s:o_kp + 8 * kp_cap * s + 8 * n].view(np.uint32).reshape(n, 2)
        xyo = kw[:, 0]
        oct_ = (xyo >> 28).astype(np.int32)  # x | y << 14 | octave << 28 (kCompactXYBits)
        k = np.empty(n, KP_DTYPE)
        k["x"] = (xyo & 0x3FFF).astype(np.float32) * sc[oct_]
        k["y"] = ((xyo >> 14) & 0x3FFF).astype(np.float32) * sc[oct_]
        k["size"] = size[oct_]
        k["angle"] = kw[:, 1].view(np.float32)
        o_sc = 8 + 88 * kp_cap + s * kp_cap
        k["response"] = rec[o_sc:o_sc + n].astype(np.float32)
        k["octave"] = oct_
        out[name] = k
    for s, (name, n) in enumerate((("desc_left", nl), ("desc_right", nr))):
        out[name] = rec[o_desc + 32 * kp_cap * s:o_desc + 32 * kp_cap * s + 32 * n].reshape(n, 32).copy()
    out["u_right"] = rec[o_st:o_st + 4 * nl].view(np.float32).copy()
    out["depth"] = rec[o_st + 4 * kp_cap:o_st + 4 * kp_cap + 4 * nl].view(np.float32).copy()
    o = 8 + 90 * kp_cap
    out["status"] = rec[o:o + nl].view(np.int8).copy()
    return out


def gather_buffer(world: int, records):
    """A reusable receive buffer for gather_records(out=...): one (world * local_pairs, record_bytes) tensor per
    (shape, dtype, device), allocated on first use and returned again for every later request of that shape —
    whoever passes it as `out` gets it overwritten by the next such gather (clear_gather_buffers frees them)."""
    import torch
    key = (world, tuple(records.shape), records.dtype, str(records.device))
    buf = _GATHER_BUF.get(key)
    if buf is None:
        buf = torch.empty((world * records.shape[0],) + tuple(records.shape[1:]), dtype=records.dtype,
                          device=records.device)
        _GATHER_BUF[key] = buf
    return buf


def clear_gather_buffers() -> None:
    """Drop the buffers gather_buffer keeps for reuse."""
    _GATHER_BUF.clear()


def gather_records(records, dst: int = 0, out=None):
    """records: (local_pairs, record_bytes) uint8 torch tensor of this rank — on the GPU with backend "nccl"
    (RCCL over xGMI), on the CPU with gloo.  Every rank must pass the same shape (the batched-frames mode
    gives every rank the same pair count; pad otherwise).  One collective, a gather to `dst` straight into
    rank-major slices of one receive buffer (no per-rank tensors, no concatenation): returns that
    (world * local_pairs, record_bytes) tensor on dst — global pair order —, None elsewhere.  The buffer is
    `out` when given (e.g. gather_buffer's reusable one, which the next gather into it overwrites), else a new
    tensor that belongs to the caller (no silent aliasing across gathers)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if world == 1:
        return records
    if rank == dst:
        full = (torch.empty((world * records.shape[0],) + tuple(records.shape[1:]), dtype=records.dtype,
                            device=records.device) if out is None else out)
        if tuple(full.shape) != (world * records.shape[0],) + tuple(records.shape[1:]):
            raise ValueError("gather output buffer has the wrong shape")
        parts = list(full.view((world,) + tuple(records.shape)).unbind(0))  # contiguous rank slices
    else:
        full, parts = None, None
    dist.gather(records, gather_list=parts, dst=dst)
    return full


def gather_results(records: np.ndarray, n_pairs_total: int, device=None, dst: int = 0):
    """Host-array convenience over gather_records for uneven shards (shard()): every rank pads its
    records to the largest shard.  Returns the records of all pairs in global pair order on dst."""
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
    full = gather_records(t, dst)
    if rank != dst:
        return None
    full = full.cpu().numpy().reshape(world, maxn, rb)
    return np.concatenate([full[r, :shard(n_pairs_total, world, r)[1]] for r in range(world)], axis=0)


def pack_device(frontends, counts, out, compact: bool = False) -> None:
    """Pack every pair of the handles' last stereo batches into `out` ((sum(counts), record bytes) uint8 device
    tensor, handle-major) with k_pack (compact: k_pack_compact) on the current stream; the pack orders itself
    after the batch that produced its results, whatever stream that batch ran on."""
    import ctypes as C
    import torch
    from ._lib import call
    rb = out.shape[1]
    st = torch.cuda.current_stream(out.device).cuda_stream
    fn = "orbfe_batch_pack_compact_device" if compact else "orbfe_batch_pack_device"
    o = 0
    for f, n in zip(frontends, counts):
        if n:
            call(fn, f.handle, C.c_void_p(out[o].data_ptr()), rb, 0, n, C.c_void_p(st))
        o += n


def fields_digest(kl, dl, kr, dr, stereo: dict) -> bytes:
    """SHA-256 over one pair's result fields in record order — keypoints L, R (orbfe_keypoint records),
    descriptors L, R, u_right, depth, status — as orbfe_batch_fetch / _fetch_stereo return them and as
    unpack / unpack_compact rebuild them from a gathered record.  Equal digests = every field bit-equal."""
    h = hashlib.sha256()
    for a in (kl, kr, dl, dr, stereo["u_right"], stereo["depth"], stereo["status"]):
        a = np.ascontiguousarray(a)
        h.update(np.int64(a.size).tobytes())
        h.update(a.tobytes())
    return h.digest()


DIGEST_ROW = 33  # per sent record: valid flag (1 B) + fields_digest (32 B); padded rows send zeros


def local_digests(frontends, counts, max_local: int) -> np.ndarray:
    """(max_local, DIGEST_ROW) uint8: row j = 1 + fields_digest of this rank's local pair j (handle-major, the
    order pack_device writes), fetched through orbfe_batch_fetch / orbfe_batch_fetch_stereo — independent of
    k_pack; rows past the rank's own pairs (padding of uneven shards) stay zero."""
    out = np.zeros((int(max_local), DIGEST_ROW), np.uint8)
    j = 0
    for f, n in zip(frontends, counts):
        for p in range(int(n)):
            kl, dl = f.fetch_image(2 * p)
            kr, dr = f.fetch_image(2 * p + 1)
            out[j, 0] = 1
            out[j, 1:] = np.frombuffer(fields_digest(kl, dl, kr, dr, f.fetch_stereo(p)), np.uint8)
            j += 1
    return out


def check_gathered(full: np.ndarray, digests: np.ndarray, unpack_fn) -> dict:
    """Rank 0's check of a gather: full (world * max_local, record_bytes) records in rank-major order,
    digests (world * max_local, DIGEST_ROW) the senders' local_digests in the same order.  Every valid row is
    unpacked (unpack_fn(record) -> unpack()'s dict) and its fields' digest compared with its sender's; every
    padded row must be all zero bytes.  Returns counts and the first failing rows (rank, local index)."""
    full = np.asarray(full)
    digests = np.asarray(digests)
    if full.shape[0] != digests.shape[0]:
        raise ValueError("records and digests disagree in row count")
    verified, padded, bad = 0, 0, []
    for i in range(full.shape[0]):
        if digests[i, 0]:
            u = unpack_fn(full[i])
            d = fields_digest(u["kps_left"], u["desc_left"], u["kps_right"], u["desc_right"], u)
            if d == digests[i, 1:].tobytes():
                verified += 1
            else:
                bad.append(i)
        elif digests[i].any() or full[i].any():
            bad.append(i)
        else:
            padded += 1
    return {"ok": not bad, "records_verified": verified, "padded_rows_zero": padded, "bad_rows": bad[:8],
            "rows": int(full.shape[0])}


def timed_gather(frontends, counts, device, world: int, rank: int, max_local: int | None = None,
                 reps: int = 3, compact: bool = True) -> dict:
    """Pack (k_pack_compact: compact records, 25 % fewer bytes over xGMI) + gather to rank 0 of every pair's
    results, timed like the bench step (barrier + synchronise on both sides, max over ranks); every rank
    sends max_local records (its own pairs, padded: uneven shards of a strong-scaling run).

    Then, untimed, EVERY gathered row is checked: each rank sends, in a second gather,
    the digest of each of its pairs' fields as orbfe_batch_fetch / _fetch_stereo return them (local_digests,
    independent of k_pack); rank 0 unpacks every record and compares its fields' digest with its sender's,
    and checks that the padded rows of uneven shards are zero (check_gathered).  Rank 0's own first pair is
    also compared field by field."""
    import torch
    import torch.distributed as dist
    n_local = int(sum(counts))
    max_local = n_local if max_local is None else int(max_local)
    kc = frontends[0].kp_cap
    rb = compact_record_bytes(kc) if compact else record_bytes(kc)
    buf = torch.zeros((max_local, rb), dtype=torch.uint8, device=device)
    nccl = world > 1 and dist.get_backend() == "nccl"
    times = []
    full = None
    for _ in range(reps + 1):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        pack_device(frontends, counts, buf, compact)
        # RCCL gathers the device buffer in place; a gloo rehearsal (several ranks on one GPU) stages it
        src = buf if world == 1 or nccl else buf.cpu()
        # the one receive buffer of this shape, reused across the repetitions (allocated outside the timing
        # by the warm-up repetition)
        full = gather_records(src, 0, out=gather_buffer(world, src) if rank == 0 and world > 1 else None)
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        times.append(time.perf_counter() - t0)
    dt = float(np.mean(times[1:]))
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device if nccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # untimed: every rank's digests to rank 0 (same collective path as the records)
    dg = torch.from_numpy(local_digests(frontends, counts, max_local))
    dg_full = gather_records(dg.to(device) if nccl else dg, 0) if world > 1 else dg
    ok, chk = None, None
    if rank == 0:
        full_np = full.cpu().numpy() if world > 1 else buf.cpu().numpy()
        unpack_fn = ((lambda r: unpack_compact(kc, r, frontends[0].scales)) if compact else (lambda r: unpack(kc, r)))
        chk = check_gathered(full_np, dg_full.cpu().numpy(), unpack_fn)
        u = unpack_fn(full_np[0])
        k, d = frontends[0].fetch_image(0)
        kr, dr = frontends[0].fetch_image(1)
        s = frontends[0].fetch_stereo(0)
        first = (u["kps_left"].tobytes() == k.tobytes() and np.array_equal(u["desc_left"], d)
                 and u["kps_right"].tobytes() == kr.tobytes() and np.array_equal(u["desc_right"], dr)
                 and np.array_equal(u["u_right"], s["u_right"]) and np.array_equal(u["depth"], s["depth"])
                 and np.array_equal(u["status"], s["status"]))
        ok = bool(first and chk["ok"])
        if not ok:
            raise RuntimeError(f"gathered records differ from their senders' orbfe_batch_fetch results: {chk}")
    return {"gather_ms": round(1e3 * dt, 4), "record_bytes": rb, "records": "compact" if compact else "full",
            "pairs_gathered": world * max_local,
            "records_verified": chk["records_verified"] if chk else None,
            "padded_rows_zero": chk["padded_rows_zero"] if chk else None,
            "bytes_to_rank0": world * max_local * rb, "record_check": ok,
            "GBs_into_rank0": round(world * max_local * rb / dt / 1e9, 2),
            "what": "k_pack on every rank + one gather of the records to rank 0 (RCCL with nccl, gloo on CPU), "
                    f"mean of {reps} after 1 warm-up, barrier + synchronize around each, max over ranks; then every "
                    "gathered record unpacked on rank 0 and checked against its sender's fetched-field digest, "
                    "padded rows checked zero"}
