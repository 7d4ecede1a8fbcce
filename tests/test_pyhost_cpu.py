"""The host-side CPython extension _pyhost (csrc/orbfe_pyhost.cpp) builds the reference data model's per-frame
objects in C: it must give the same objects, with the same element types, as the Python constructions it
replaces (KeyPoint tuples, Frame.mGrid, mvuRight / mvDepth)."""
import numpy as np
import pytest

from pyorbslam_amd._lib import KP_DTYPE, pyhost
from pyorbslam_amd.frame import to_reference_lists
from pyorbslam_amd.pyORBExtractor import keypoint_tuples


def _types(rows):
    return [tuple(map(type, r)) if isinstance(r, tuple) else type(r) for r in rows]


def test_keypoint_tuples():
    rng = np.random.default_rng(0)
    a = np.zeros(1000, KP_DTYPE)
    for f in ("x", "y", "size", "angle", "response"):
        a[f] = (rng.random(1000) * 2000 - 500).astype(np.float32)
    a["octave"] = rng.integers(0, 8, 1000)
    assert keypoint_tuples(a) == a.tolist() and _types(keypoint_tuples(a)) == _types(a.tolist())
    assert keypoint_tuples(a[::3]) == a[::3].tolist()  # non-contiguous: copied first
    assert keypoint_tuples(a[:0]) == []
    with pytest.raises(TypeError):
        keypoint_tuples(np.zeros(3, np.float32))


def test_grid_lists():
    rng = np.random.default_rng(1)
    cols, rows = 64, 48
    cell = np.sort(rng.integers(0, cols * rows, 1500))
    flat = rng.permutation(1500).astype(np.int32)
    off = np.zeros(cols * rows + 1, np.int32)
    np.cumsum(np.bincount(cell, minlength=cols * rows), out=off[1:])
    g = pyhost().grid_lists(flat, off, cols, rows)
    fl, o = flat.tolist(), off.tolist()
    ref = [[fl[o[ix * rows + iy]:o[ix * rows + iy + 1]] for iy in range(rows)] for ix in range(cols)]
    assert g == ref
    cells = [c for col in g for c in col]
    assert len({id(c) for c in cells}) == cols * rows  # a new list per cell
    bad = off.copy()
    bad[5] = bad[6] + 1
    with pytest.raises(ValueError):
        pyhost().grid_lists(flat, bad, cols, rows)
    with pytest.raises(ValueError):
        pyhost().grid_lists(flat, off[:-1], cols, rows)


def test_stereo_lists_match_the_python_construction():
    rng = np.random.default_rng(2)
    n = 700
    st = rng.integers(0, 3, n).astype(np.int8)
    res = dict(u_right=rng.random(n).astype(np.float32) * 900, depth=rng.random(n).astype(np.float32) * 50, status=st)
    kps = np.zeros(n, KP_DTYPE)
    kps["x"] = rng.random(n).astype(np.float32) * 1200
    for mbf in (386.1448, 47.90639384423901):
        uR, dep = to_reference_lists(res, kps, mbf)
        ru, rd = list(res["u_right"]), list(res["depth"])
        for i in np.flatnonzero(st == 0).tolist():
            ru[i] = rd[i] = -1
        for i in np.flatnonzero(st == 2).tolist():
            ru[i], rd[i] = float(kps["x"][i]) - 0.01, mbf / 0.01
        assert uR == ru and dep == rd and _types(uR) == _types(ru) and _types(dep) == _types(rd)
    # a numpy mbf keeps the Python path (mbf / 0.01 keeps its numpy type there)
    uR, dep = to_reference_lists(res, kps, np.float64(386.1448))
    assert type(dep[int(np.flatnonzero(st == 2)[0])]) is np.float64


def test_grid_assign_matches_the_numpy_construction():
    """Cells by round-half-even of the same double expression (values exactly at .5 included), keypoints
    outside the grid skipped, keypoint order inside a cell."""
    rng = np.random.default_rng(4)
    cols, rows = 64, 48
    minx, miny, wi, hi = 0.0, 0.0, 64 / 1241.0, 48 / 376.0
    pts = np.column_stack((rng.random(3000) * 1300 - 30, rng.random(3000) * 400 - 12))
    pts[:50, 0] = (np.arange(50) + 0.5) / wi  # exact halves
    pts[50:60] = [[-40.0, 10.0]] * 10
    g, off, flat = pyhost().grid_assign(np.ascontiguousarray(pts), minx, miny, wi, hi, cols, rows)
    px = np.round((pts[:, 0] - minx) * wi).astype(int)
    py = np.round((pts[:, 1] - miny) * hi).astype(int)
    keep = np.flatnonzero((px >= 0) & (px < cols) & (py >= 0) & (py < rows))
    cell = px[keep] * rows + py[keep]
    rflat = keep[np.argsort(cell, kind="stable")].astype(np.int32)
    roff = np.zeros(cols * rows + 1, np.int32)
    np.cumsum(np.bincount(cell, minlength=cols * rows), out=roff[1:])
    assert np.array_equal(off, roff) and np.array_equal(flat, rflat) and off.dtype == flat.dtype == np.int32
    assert g == pyhost().grid_lists(rflat, roff, cols, rows)
