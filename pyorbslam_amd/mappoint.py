"""Drop-in for MapPoint.compute_distinctive_descriptors (MapPoint.py:204-240).

The reference fills an N x N float32 matrix of pairwise descriptor distances with a per-byte Python
popcount (N(N-1)/2 calls), then keeps the observation whose row median is smallest (first one on ties).
Here the matrix comes from k_hamming_matrix (one launch per point) or, for many points at once
(compute_distinctive_descriptors_many — what LocalMapping's per-keyframe loops want), from one
k_hamming_search launch over every point's observations as CSR candidate lists.  The medians and the
choice stay the reference's expressions on the same float32 rows, so the chosen descriptor is identical.
"""
from __future__ import annotations

import numpy as np

from .matcher import hamming_csr, hamming_matrix


def _observed_descriptors(mp):
    """The reference's prologue (MapPoint.py:205-219): None when it returns early."""
    with mp.mMutexFeatures:
        if mp.mbBad:
            return None
        observations = mp.mObservations.copy()
    if not observations:
        return None
    v = [pKF.mDescriptors[idx] for pKF, idx in observations.items() if not pKF.is_bad()]
    return v or None


def _pick(mp, v, dist):
    """Median selection (MapPoint.py:221-240) on the float32 distance rows."""
    D = dist.astype(np.float32)
    best_median, best_idx = float('inf'), 0
    for i in range(len(v)):
        median = np.median(D[i])
        if median < best_median:
            best_median = median
            best_idx = i
    with mp.mMutexFeatures:
        mp.mDescriptor = v[best_idx].copy()


def compute_distinctive_descriptors(mp):
    v = _observed_descriptors(mp)
    if v is None:
        return
    d = np.stack([np.asarray(x, np.uint8).reshape(32) for x in v])
    _pick(mp, v, hamming_matrix(d, d))


def compute_distinctive_descriptors_many(mps):
    """compute_distinctive_descriptors for every point of `mps`, with one GPU launch for all matrices."""
    todo = []
    for mp in mps:
        v = _observed_descriptors(mp)
        if v is not None:
            todo.append((mp, v))
    if not todo:
        return
    desc = np.concatenate([np.stack([np.asarray(x, np.uint8).reshape(32) for x in v]) for _, v in todo])
    # query row r of point p: candidates = all rows of p (its own block of the concatenation)
    n = np.array([len(v) for _, v in todo], np.int64)
    base = np.concatenate([[0], np.cumsum(n)[:-1]])
    q_len = np.repeat(n, n)
    off = np.concatenate([[0], np.cumsum(q_len)]).astype(np.int32)
    idx = np.concatenate([np.tile(np.arange(b, b + k), k) for b, k in zip(base, n)]).astype(np.int32)
    dist = hamming_csr(desc, desc, off, idx)
    pos = 0
    for (mp, v), k in zip(todo, n):
        k = int(k)
        _pick(mp, v, dist[pos:pos + k * k].reshape(k, k))
        pos += k * k


def install(mappoint_cls) -> None:
    """Route the reference MapPoint class's method through this implementation."""
    mappoint_cls.compute_distinctive_descriptors = compute_distinctive_descriptors
