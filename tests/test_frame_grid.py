"""frame.assign_features_to_grid (the vectorised drop-in) against the reference method's restatement in
the C3 harness (seq_harness.SeqFrame.assign_features_to_grid, itself pinned by the sequence golden's grid
cells), on random keypoints incl. points off the grid and exact half-cell positions (np.round: half to
even)."""
import numpy as np
import pytest

import seq_harness as H
from pyorbslam_amd import frame as F, synth


class _Ref(H.SeqFrame):
    def __init__(self, kps, fa):
        (self.fx, self.fy, self.cx, self.cy, self.invfx, self.invfy, self.mfGridElementWidthInv,
         self.mfGridElementHeightInv, self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY, self.FRAME_GRID_ROWS,
         self.FRAME_GRID_COLS) = fa
        self.mvKeys = kps
        self.N = len(kps)


class _DropIn(_Ref):
    pass


F.install(_DropIn)


@pytest.mark.parametrize("seed", range(3))
def test_grid_matches_reference(seed):
    fa = H.frame_args(H.settings(synth.KITTI_CAM), 1241, 376)
    rng = np.random.default_rng(seed)
    n = 2500
    x = rng.uniform(-40, 1300, n).astype(np.float32)
    y = rng.uniform(-40, 420, n).astype(np.float32)
    # exact half-cell positions: (x - minX) * inv = k + 0.5
    minx, invw = fa[8], fa[6]
    x[:50] = np.float32(minx + (np.arange(50) + 0.5) / invw)
    kps = [H.KeyPoint(float(a), float(b), 7.0, 0.0, 1.0, 0) for a, b in zip(x, y)]
    ref, new = _Ref(kps, fa), _DropIn(kps, fa)
    ref.assign_features_to_grid()
    new.assign_features_to_grid()
    assert new.mGrid == ref.mGrid
    assert all(type(i) is int for col in new.mGrid for cell in col for i in cell)
    # the CSR kept for the matcher describes the same grid
    _, off, flat = new._orbfe_grid
    rows = new.FRAME_GRID_ROWS
    for ix, col in enumerate(new.mGrid):
        for iy, cell in enumerate(col):
            c = ix * rows + iy
            assert flat[off[c]:off[c + 1]].tolist() == cell
    # the matcher's grid arrays from the coordinates the drop-in kept equal the ones read from the keypoints
    from pyorbslam_amd import matcher as M
    new.mvKeysUn = new.mvKeys
    kept = M._frame_grid(new)
    ref.mvKeysUn, ref.mGrid = ref.mvKeys, new.mGrid
    read = M._frame_grid(ref)  # no _orbfe_grid / _orbfe_pts: rebuilt from mGrid and the KeyPoint objects
    assert new._orbfe_pts[0] is new.mvKeys and not hasattr(ref, "_orbfe_pts")
    for a, b in zip(kept[:6], read[:6]):
        assert a.dtype == b.dtype and np.array_equal(a, b)


def test_grid_empty_frame_runs_reference():
    fa = H.frame_args(H.settings(synth.KITTI_CAM), 1241, 376)
    ref, new = _Ref([], fa), _DropIn([], fa)
    ref.assign_features_to_grid()
    new.assign_features_to_grid()
    assert new.mGrid == ref.mGrid
