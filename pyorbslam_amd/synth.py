"""Deterministic synthetic stereo pairs (SURVEY.md §8(d) "Synthetic input").

Left image: three octaves of band-limited value noise plus random axis-aligned rectangles (edges and
corners for FAST), clipped to [0, 255].  Right image: the same canvas sampled with a per-row-block
horizontal disparity in [0, dmax] px plus +-2 intensity noise, so a left feature at uL reappears at
uR = uL - d (the geometry Frame.compute_stereo_matches searches, Frame.py:197-215).

Pure numpy; the same seed gives the same bytes on every machine with numpy >= 1.17 (PCG64 streams).
"""
from __future__ import annotations

import numpy as np

KITTI_WH = (1241, 376)  # KITTI00-02.yaml Camera.width/height
EUROC_WH = (752, 480)


def _value_noise(rng: np.random.Generator, h: int, w: int, cell: int, amp: float) -> np.ndarray:
    gh, gw = h // cell + 2, w // cell + 2
    g = rng.random((gh, gw), dtype=np.float32) * amp
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0 = ys.astype(np.int32)
    x0 = xs.astype(np.int32)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def make_pair(seed: int, width: int = KITTI_WH[0], height: int = KITTI_WH[1], dmax: int = 64,
              block: int = 16) -> tuple[np.ndarray, np.ndarray]:
    """Return (left, right) u8 arrays of shape (height, width), C-contiguous."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cw = width + dmax
    canvas = np.full((height, cw), 40.0, np.float32)
    for cell, amp in ((48, 90.0), (12, 50.0), (3, 22.0)):
        canvas += _value_noise(rng, height, cw, cell, amp)
    nrect = max(8, (width * height) // 9000)
    for _ in range(nrect):
        rw, rh = rng.integers(8, 90), rng.integers(8, 60)
        x0, y0 = rng.integers(0, cw - rw), rng.integers(0, height - rh)
        canvas[y0:y0 + rh, x0:x0 + rw] += rng.uniform(-70.0, 70.0)
    left = np.clip(np.rint(canvas[:, :width]), 0, 255).astype(np.uint8)
    nblk = (height + block - 1) // block
    disp = rng.integers(0, dmax + 1, size=nblk)
    right = np.empty((height, width), np.float32)
    for b in range(nblk):
        r0, r1 = b * block, min(height, (b + 1) * block)
        d = int(disp[b])
        right[r0:r1] = canvas[r0:r1, d:d + width]
    right += rng.integers(-2, 3, size=right.shape).astype(np.float32)
    right = np.clip(np.rint(right), 0, 255).astype(np.uint8)
    return np.ascontiguousarray(left), np.ascontiguousarray(right)


def make_batch(n_pairs: int, seed0: int = 0, width: int = KITTI_WH[0], height: int = KITTI_WH[1]) -> np.ndarray:
    """(2*n_pairs, height, width) u8: images 2p / 2p+1 are the left / right of pair p (seed seed0+p)."""
    out = np.empty((2 * n_pairs, height, width), np.uint8)
    for p in range(n_pairs):
        out[2 * p], out[2 * p + 1] = make_pair(seed0 + p, width, height)
    return out


def shifted_right(left: np.ndarray, seed: int, dmax: int = 48, block: int = 16) -> np.ndarray:
    """A right view for a real left image (used with the reference's kitti06-436.png fixture)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    h, w = left.shape
    pad = np.pad(left.astype(np.float32), ((0, 0), (0, dmax)), mode="edge")
    nblk = (h + block - 1) // block
    disp = rng.integers(0, dmax + 1, size=nblk)
    right = np.empty((h, w), np.float32)
    for b in range(nblk):
        r0, r1 = b * block, min(h, (b + 1) * block)
        right[r0:r1] = pad[r0:r1, int(disp[b]):int(disp[b]) + w]
    right += rng.integers(-2, 3, size=right.shape).astype(np.float32)
    return np.ascontiguousarray(np.clip(np.rint(right), 0, 255).astype(np.uint8))
