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


# ------------------------------------------------------------------------------ moving stereo sequence
KITTI_CAM = dict(fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448)  # KITTI00-02.yaml:7-10, 37


def _texture(rng: np.random.Generator, h: int, w: int, rmax: int = 60, amp: float = 1.0) -> np.ndarray:
    t = np.full((h, w), 128.0 - 70.0 * amp, np.float32)
    for cell, a in ((40, 90.0), (10, 50.0), (3, 22.0)):
        t += _value_noise(rng, h, w, cell, a * amp)
    for _ in range(max(6, (h * w) // 2500)):
        rw, rh = rng.integers(3, min(rmax, w - 1)), rng.integers(3, min(rmax, h - 1))
        x0, y0 = rng.integers(0, w - rw), rng.integers(0, h - rh)
        t[y0:y0 + rh, x0:x0 + rw] += rng.uniform(-60.0, 60.0) * amp
    return t


class StereoSequence:
    """A rectified stereo camera moving through a scene of textured fronto-parallel planes, rendered
    deterministically (float64 ray casting, bilinear texture lookup, +-2 sensor noise per image).

    Used as the synthetic stand-in for KITTI-00 (BASELINE config C3): the camera moves
    forward (speed m/frame) with a lateral / vertical sway and a small yaw / pitch oscillation, so
    consecutive frames share most features at changing scales and the constant-velocity prediction of
    Tracking.track_with_motion_model (Tracking.py:583) is close to, but not equal to, the true pose.
    pose(k) is the ground-truth Tcw (float32 4x4, world -> camera); frame(k) the (left, right) images."""

    def __init__(self, seed: int = 0, width: int = KITTI_WH[0], height: int = KITTI_WH[1], speed: float = 0.6,
                 cam: dict | None = None, n_boxes: int = 40):
        self.seed, self.width, self.height, self.speed = int(seed), int(width), int(height), float(speed)
        self.cam = dict(KITTI_CAM if cam is None else cam)
        self.baseline = self.cam["bf"] / self.cam["fx"]
        rng = np.random.Generator(np.random.PCG64(1_000_003 + self.seed))
        # (z, x0, x1, y0, y1, texel size, texture); the background plane last
        self.layers = []
        for _ in range(n_boxes):
            z = float(rng.uniform(40.0, 160.0))
            half = 0.9 * z  # the field of view is about +-0.85 z wide and +-0.26 z high
            sx, sy = float(rng.uniform(0.06, 0.3)) * z, float(rng.uniform(0.04, 0.16)) * z
            x0, y0 = float(rng.uniform(-half, half - sx)), float(rng.uniform(-0.3 * z, 0.3 * z - sy))
            texel = float(rng.uniform(0.0006, 0.0016)) * z
            th, tw = int(sy / texel) + 2, int(sx / texel) + 2
            self.layers.append((z, x0, x0 + sx, y0, y0 + sy, texel, _texture(rng, th, tw)))
        self.layers.sort(key=lambda a: a[0])
        bg_texel = 0.5
        self.layers.append((240.0, -420.0, 420.0, -150.0, 150.0, bg_texel,
                            _texture(rng, int(300 / bg_texel) + 2, int(840 / bg_texel) + 2, rmax=24, amp=0.6)))

    def _rwc_center(self, k: int) -> tuple[np.ndarray, np.ndarray]:
        yaw, pitch = 0.03 * np.sin(0.09 * k), 0.012 * np.sin(0.13 * k + 0.5)
        cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
        ry = np.array([[cy, 0.0, sy], [0.0, 1.0, 0.0], [-sy, 0.0, cy]])
        rx = np.array([[1.0, 0.0, 0.0], [0.0, cp, -sp], [0.0, sp, cp]])
        c = np.array([2.0 * np.sin(0.07 * k), 0.3 * np.sin(0.11 * k), self.speed * k])
        return ry @ rx, c

    def pose(self, k: int) -> np.ndarray:
        rwc, c = self._rwc_center(k)
        t = np.eye(4, dtype=np.float32)
        t[:3, :3] = rwc.T.astype(np.float32)
        t[:3, 3] = (-rwc.T @ c).astype(np.float32)
        return t

    def _render(self, rwc: np.ndarray, c: np.ndarray, noise_seed: int) -> np.ndarray:
        h, w, cam = self.height, self.width, self.cam
        u = (np.arange(w, dtype=np.float64) - cam["cx"]) / cam["fx"]
        v = (np.arange(h, dtype=np.float64) - cam["cy"]) / cam["fy"]
        dc = np.stack(np.broadcast_arrays(u[None, :], v[:, None], np.ones((1, 1))), -1)  # (h, w, 3)
        dw = dc @ rwc.T
        best_t = np.full((h, w), np.inf)
        best_l = np.full((h, w), -1, np.int32)
        for li, (z, x0, x1, y0, y1, _, _) in enumerate(self.layers):
            t = (z - c[2]) / dw[..., 2]
            px, py = c[0] + t * dw[..., 0], c[1] + t * dw[..., 1]
            hit = (t > 0) & (t < best_t) & (px >= x0) & (px < x1) & (py >= y0) & (py < y1)
            best_t[hit] = t[hit]
            best_l[hit] = li
        img = np.full((h, w), 20.0, np.float64)
        for li, (z, x0, x1, y0, y1, texel, tex) in enumerate(self.layers):
            m = best_l == li
            if not m.any():
                continue
            t = best_t[m]
            tx = (c[0] + t * dw[..., 0][m] - x0) / texel
            ty = (c[1] + t * dw[..., 1][m] - y0) / texel
            ix, iy = np.floor(tx).astype(np.int64), np.floor(ty).astype(np.int64)
            fx, fy = tx - ix, ty - iy
            ix = np.clip(ix, 0, tex.shape[1] - 2)
            iy = np.clip(iy, 0, tex.shape[0] - 2)
            a, b = tex[iy, ix].astype(np.float64), tex[iy, ix + 1].astype(np.float64)
            cc, d = tex[iy + 1, ix].astype(np.float64), tex[iy + 1, ix + 1].astype(np.float64)
            img[m] = (a * (1 - fx) + b * fx) * (1 - fy) + (cc * (1 - fx) + d * fx) * fy
        rng = np.random.Generator(np.random.PCG64(noise_seed))
        img += rng.integers(-2, 3, size=img.shape)
        return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))

    def frame(self, k: int) -> tuple[np.ndarray, np.ndarray]:
        rwc, c = self._rwc_center(k)
        left = self._render(rwc, c, 7_000_000 + 1000 * self.seed + 2 * k)
        right = self._render(rwc, c + rwc @ np.array([self.baseline, 0.0, 0.0]), 7_000_000 + 1000 * self.seed + 2 * k + 1)
        return left, right
