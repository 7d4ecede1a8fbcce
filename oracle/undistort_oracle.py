"""TEST INFRASTRUCTURE ONLY — cv::undistortPoints(pts, K, D, noArray(), P=K) restated in Python doubles
(OpenCV 4.x cvUndistortPointsInternal: TermCriteria(COUNT, 5, 0.01), the icdist < 0 guard, P = K), the call
of the reference's Frame.undistort_keypoints (Frame.py:306) and Tracking.compute_image_bounds
(Tracking.py:132).

PARITY UNPINNED: OpenCV is not in this image and the reference's distorted branch cannot run (it reads the
undefined name `mvKeys` at Frame.py:299), so nothing of the reference's own pins this; the restatement
follows OpenCV's published algorithm operation for operation (Python floats are IEEE doubles, evaluated in
the same order), and the GPU kernel k_undistort is checked against it bit for bit."""
from __future__ import annotations

import numpy as np


def undistort_points(xy: np.ndarray, K, dist) -> np.ndarray:
    """xy: (n, 2) float32 pixels; K: 3x3 (float32 in the reference); dist: (k1, k2, p1, p2[, k3]).
    Returns (n, 2) float32."""
    xy = np.asarray(xy, np.float32).reshape(-1, 2)
    K = np.asarray(K, np.float32)
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    d = [float(v) for v in np.asarray(dist, np.float32).ravel()]
    k1, k2, p1, p2 = d[:4]
    k3 = d[4] if len(d) > 4 else 0.0
    ifx, ify = 1.0 / fx, 1.0 / fy
    out = np.empty_like(xy)
    for i, (u, v) in enumerate(xy.astype(np.float64).tolist()):
        x0 = x = (u - cx) * ifx
        y0 = y = (v - cy) * ify
        for _ in range(5):
            r2 = x * x + y * y
            icdist = 1.0 / (1.0 + ((k3 * r2 + k2) * r2 + k1) * r2)
            if icdist < 0:
                x, y = x0, y0
                break
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        out[i, 0] = np.float32(x * fx + cx)
        out[i, 1] = np.float32(y * fy + cy)
    return out
