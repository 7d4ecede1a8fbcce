"""ORBMatcher Hamming searches: oracle (CPU) and the GPU drop-in against the reference's own outputs."""
import numpy as np
import pytest

from conftest import GOLDEN
import matcher_frames as MF
from oracle import matcher_oracle as MO


def test_distance_oracle_golden():
    z = np.load(GOLDEN / "matcher_distance.npz")
    assert [MO.dist(a, b) for a, b in zip(z["a"], z["b"])] == z["dist"].tolist()


@pytest.mark.parametrize("case", range(6))
def test_fp_oracle_golden(case):
    fr, mps, th, n, assigned = MF.load_fp(case)
    assert MO.search_f_p(fr, mps, th, 0.8) == n
    assert np.array_equal(MF.encode_fp(fr, mps), assigned)


@pytest.mark.parametrize("case", range(6))
def test_ff_oracle_golden(case):
    cur, last, mps, extra, z = MF.load_ff(case)
    assert MO.search_f_f(cur, last, float(z["th"])) == int(z["n_matches"])
    assert np.array_equal(MF.encode_ff(cur, mps, extra), z["assigned"])


@pytest.mark.gpu
def test_distance_gpu_golden():
    from pyorbslam_amd.matcher import ORBMatcher, hamming_matrix
    z = np.load(GOLDEN / "matcher_distance.npz")
    m = ORBMatcher(0.8, True)
    assert [m.descriptor_distance(a, b) for a, b in zip(z["a"][:16], z["b"][:16])] == z["dist"][:16].tolist()
    full = hamming_matrix(z["a"], z["b"])
    assert np.array_equal(np.diag(full), z["dist"])
    ref = np.array([[MO.dist(a, b) for b in z["b"][:40]] for a in z["a"][:40]])
    assert np.array_equal(full[:40, :40], ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6))
def test_fp_gpu_golden(case):
    from pyorbslam_amd.matcher import ORBMatcher
    fr, mps, th, n, assigned = MF.load_fp(case)
    assert ORBMatcher(0.8, True).search_by_projection_f_p(fr, mps, th) == n
    assert np.array_equal(MF.encode_fp(fr, mps), assigned)


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(6))
def test_ff_gpu_golden(case):
    from pyorbslam_amd.matcher import ORBMatcher
    cur, last, mps, extra, z = MF.load_ff(case)
    assert ORBMatcher(0.8, True).search_by_projection_f_f(cur, last, float(z["th"])) == int(z["n_matches"])
    assert np.array_equal(MF.encode_ff(cur, mps, extra), z["assigned"])


@pytest.mark.gpu
def test_hamming_search_top2_matches_sequential_scan():
    """k_hamming_search's (dist, position) top-2 equals the reference's sequential best / second scan."""
    import ctypes as C
    from pyorbslam_amd import matcher
    from pyorbslam_amd._lib import call, ptr
    rng = np.random.default_rng(0)
    q = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (900, 32), dtype=np.uint8)
    t[::7] = t[3]  # duplicate descriptors -> ties
    lens = rng.integers(0, 150, 300)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    idx = rng.integers(0, 900, off[-1]).astype(np.int32)
    bd, bi, sd, si = (np.zeros(300, np.int32) for _ in range(4))
    call("orbfe_hamming_search", matcher._h(), ptr(q), 300, ptr(t), 900, ptr(off), ptr(idx), ptr(bd), ptr(bi), ptr(sd),
         ptr(si))
    for k in range(300):
        b1, i1, b2, i2 = 256, -1, 256, -1
        for c in idx[off[k]:off[k + 1]]:
            d = MO.dist(q[k], t[c])
            if d < b1:
                b2, i2, b1, i1 = b1, i1, d, int(c)
            elif d < b2:
                b2, i2 = d, int(c)
        assert (bd[k], bi[k], sd[k], si[k]) == (b1, i1, b2, i2), k


@pytest.mark.gpu
def test_hamming_concurrent_threads():
    """ORBMatcher / MapPoint are called from the Tracking, LocalMapping and LoopClosing threads at once
    (System.py:59-64): concurrent hamming_csr / hamming_matrix calls at different sizes (so the scratch
    buffers are re-allocated while the other thread runs) must each return numpy's popcounts."""
    import threading
    from pyorbslam_amd import matcher as M
    lut = np.array([bin(i).count("1") for i in range(256)], np.int32)
    errors = []

    def work(seed):
        rng = np.random.default_rng(seed)
        try:
            for it in range(40):
                nq, nt = int(rng.integers(1, 400)), int(rng.integers(1, 900))
                q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
                t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
                cnt = rng.integers(0, 12, nq)
                off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
                idx = rng.integers(0, nt, int(off[-1])).astype(np.int32)
                got = M.hamming_csr(q, t, off, idx)
                qi = np.repeat(np.arange(nq), cnt)
                want = lut[q[qi] ^ t[idx]].sum(1)
                if not np.array_equal(got, want):
                    errors.append(("csr", seed, it))
                a, b = q[: min(nq, 50)], t[: min(nt, 70)]
                if not np.array_equal(M.hamming_matrix(a, b), lut[a[:, None, :] ^ b[None, :, :]].sum(2)):
                    errors.append(("matrix", seed, it))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("raised", seed, repr(e)))

    ths = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:5]


def test_descriptor_distance_host_golden():
    """The one-pair drop-in (liborbfe host popcount, no device call) against the reference's own
    descriptor_distance outputs (ORBMatcher.py:12-14)."""
    from pyorbslam_amd.matcher import ORBMatcher
    z = np.load(GOLDEN / "matcher_distance.npz", allow_pickle=False)
    m = ORBMatcher(0.8, True)
    got = [m.descriptor_distance(z["a"][i], z["b"][i]) for i in range(len(z["a"]))]
    assert got == z["dist"].tolist()
    assert all(type(v) is int for v in got)


def cpu_csr(qd, train, off, idx):
    """orbfe_hamming_csr on the host (numpy popcount): the one GPU call of the matcher searches."""
    q = np.repeat(np.arange(len(off) - 1), np.diff(off))
    t = np.asarray(train, np.uint8).reshape(-1, 32)
    x = np.bitwise_xor(np.asarray(qd, np.uint8).reshape(-1, 32)[q], t[np.asarray(idx, np.int64)])
    return np.unpackbits(x, axis=1).sum(1).astype(np.int32)


def _cpu_matcher(monkeypatch, native=True):
    """The drop-in ORBMatcher with its one GPU call (the batched Hamming distances) answered on the host:
    the host logic — batched grid queries (orbfe_grid_query), the stacked projection, the native candidate
    selection (orbfe_select_f_f / _f_p, host code) or, with native=False, the Python replay — runs as in
    production."""
    from pyorbslam_amd import matcher

    monkeypatch.setattr(matcher.ORBMatcher, "_csr", staticmethod(cpu_csr))
    if not native:
        monkeypatch.setattr(matcher.ORBMatcher, "_f_f_native", lambda self, *a: None)
        monkeypatch.setattr(matcher.ORBMatcher, "_f_p_native", lambda self, *a: None)
    return matcher.ORBMatcher


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("case", range(6))
def test_fp_host_logic_golden(case, native, monkeypatch):
    fr, mps, th, n, assigned = MF.load_fp(case)
    assert _cpu_matcher(monkeypatch, native)(0.8, True).search_by_projection_f_p(fr, mps, th) == n
    assert np.array_equal(MF.encode_fp(fr, mps), assigned)


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("case", range(6))
def test_ff_host_logic_golden(case, native, monkeypatch):
    cur, last, mps, extra, z = MF.load_ff(case)
    m = _cpu_matcher(monkeypatch, native)(0.8, True)
    assert m.search_by_projection_f_f(cur, last, float(z["th"])) == int(z["n_matches"])
    assert np.array_equal(MF.encode_ff(cur, mps, extra), z["assigned"])


def test_grid_query_matches_frame_method():
    """orbfe_grid_query against the grid restatement's per-query method (itself pinned by the goldens),
    random queries incl. windows past the image and level filters."""
    from pyorbslam_amd.matcher import features_in_areas
    fr, _, _, _, _ = MF.load_fp(0)
    rng = np.random.default_rng(2)
    qs = [(float(rng.uniform(-50, 1300)), np.float64(rng.uniform(-50, 420)), float(rng.uniform(0.5, 80)),
           int(rng.integers(-1, 8)), int(rng.integers(-1, 8))) for _ in range(3000)]
    qs += [(np.array([q[0]]), q[1], q[2], q[3], q[4]) for q in qs[:200]]  # 1-element float64 arrays
    assert features_in_areas(fr, qs) == [fr.get_features_in_area(*q) for q in qs]
    q32 = [(np.float32(q[0]), q[1], q[2], q[3], q[4]) for q in qs[:100]]  # float32: the frame's own method
    assert features_in_areas(fr, q32) == [fr.get_features_in_area(*q) for q in q32]


def test_stacked_projection_equals_per_point_matmul():
    """search_by_projection_f_f projects all map points with one stacked matmul; it must equal the
    reference's per-point `Rcw @ x3Dw + tcw` bit for bit under this NumPy build."""
    rng = np.random.default_rng(0)
    for dt in (np.float32, np.float64):
        for rdt in (np.float32, np.float64):
            R, t = rng.normal(size=(3, 3)).astype(rdt), rng.normal(size=(3, 1)).astype(rdt)
            X = (rng.normal(size=(2000, 3, 1)) * 30).astype(dt)
            assert np.array_equal(R @ X + t, np.stack([R @ X[k] + t for k in range(len(X))]))


def _select_ff_py(off, idx, dist, u, invzc, radius, q_obs, u_right, blocked, mbf, th_high):
    """ORBMatcher.py:348-372 as written, over the same arrays (Python float arithmetic)."""
    out = []
    for q in range(len(off) - 1):
        best_dist, best = 256, -1
        for k in range(off[q], off[q + 1]):
            i2 = int(idx[k])
            if blocked[i2]:
                continue
            if u_right[i2] > 0:
                ur = float(u[q]) - mbf * float(invzc[q])
                if abs(ur - float(u_right[i2])) > float(radius[q]):
                    continue
            if dist[k] < best_dist:
                best_dist, best = int(dist[k]), i2
        if best_dist <= th_high:
            out.append(best)
            blocked[best] = q_obs[q]
        else:
            out.append(-1)
    return out


def _select_fp_py(off, idx, dist, xr, rs, octv, q_obs, u_right, blocked, nnratio, th_high):
    """ORBMatcher.py:246-281 as written."""
    out = []
    for q in range(len(off) - 1):
        bd, bl, bd2, bl2, bi = 256, -1, 256, -1, -1
        for k in range(off[q], off[q + 1]):
            i = int(idx[k])
            if blocked[i]:
                continue
            if u_right[i] > 0 and abs(float(xr[q]) - float(u_right[i])) > float(rs[q]):
                continue
            d = int(dist[k])
            if d < bd:
                bd2, bd, bl2, bl, bi = bd, d, bl, int(octv[i]), i
            elif d < bd2:
                bl2, bd2 = int(octv[i]), d
        if bd <= th_high and not (bl == bl2 and bd > nnratio * bd2):
            out.append(bi)
            blocked[bi] = q_obs[q]
        else:
            out.append(-1)
    return out


@pytest.mark.parametrize("seed", range(4))
def test_native_selection_matches_python_loop(seed):
    """orbfe_select_f_f / _f_p (host code) against the reference loops restated in Python, on random
    candidate sets with stereo gates, pre-blocked slots, ties, empty queries and repeated slots."""
    from pyorbslam_amd._lib import call, ptr
    rng = np.random.default_rng(seed)
    n_frame, nq = 300, 400
    cnt = rng.integers(0, 12, nq)
    cnt[rng.random(nq) < 0.1] = 0
    off = np.zeros(nq + 1, np.int32)
    np.cumsum(cnt, out=off[1:])
    idx = rng.integers(0, n_frame, off[-1]).astype(np.int32)
    dist = rng.integers(0, 140, off[-1]).astype(np.int32)
    u_right = np.where(rng.random(n_frame) < 0.6, rng.uniform(0, 1200, n_frame), -1.0)
    blocked0 = (rng.random(n_frame) < 0.1).astype(np.uint8)
    q_obs = (rng.random(nq) < 0.5).astype(np.uint8)
    u = rng.uniform(0, 1240, nq)
    invzc = rng.uniform(0.01, 0.2, nq)
    radius = rng.uniform(2, 40, nq)
    mbf = 386.1448
    got = np.empty(nq, np.int32)
    blocked = blocked0.copy()
    call("orbfe_select_f_f", nq, ptr(off), ptr(idx), ptr(dist), ptr(u), ptr(invzc), ptr(radius), ptr(q_obs),
         ptr(u_right), ptr(blocked), n_frame, mbf, 100, ptr(got))
    b2 = blocked0.copy()
    assert got.tolist() == _select_ff_py(off, idx, dist, u, invzc, radius, q_obs, u_right, b2, mbf, 100)
    assert np.array_equal(blocked, b2)
    xr = rng.uniform(0, 1240, nq)
    octv = rng.integers(0, 8, n_frame).astype(np.int32)
    blocked = blocked0.copy()
    call("orbfe_select_f_p", nq, ptr(off), ptr(idx), ptr(dist), ptr(xr), ptr(radius), ptr(octv), ptr(q_obs),
         ptr(u_right), ptr(blocked), n_frame, 0.8, 100, ptr(got))
    b2 = blocked0.copy()
    assert got.tolist() == _select_fp_py(off, idx, dist, xr, radius, octv, q_obs, u_right, b2, 0.8, 100)
    assert np.array_equal(blocked, b2)


def test_native_selection_rejects_bad_index():
    from pyorbslam_amd import _lib
    off = np.array([0, 2], np.int32)
    idx = np.array([0, 5], np.int32)  # 5 >= n_frame
    dist = np.zeros(2, np.int32)
    z = np.zeros(4, np.float64)
    flags = np.zeros(4, np.uint8)
    out = np.empty(1, np.int32)
    rc = _lib.lib().orbfe_select_f_f(1, _lib.ptr(off), _lib.ptr(idx), _lib.ptr(dist), _lib.ptr(z), _lib.ptr(z),
                                     _lib.ptr(z), _lib.ptr(flags), _lib.ptr(z), _lib.ptr(flags), 4, 1.0, 100,
                                     _lib.ptr(out))
    assert rc < 0 and "out of range" in _lib.lib().orbfe_last_error().decode()


@pytest.mark.parametrize("case", range(3))
def test_fp_python_float_xr_takes_the_float32_path(case, monkeypatch):
    """with a Python-float mTrackProjXR and np.float32 mvuRight entries, the reference's
    abs(XR - mvuRight[idx]) evaluates in float32 (NEP 50); the native double selection must not run then,
    and the result must equal the Python replay's on the same inputs."""
    from pyorbslam_amd import matcher
    fr, mps, th, _, _ = MF.load_fp(case)
    fr.mvuRight = [np.float32(v) if float(v) > 0 else v for v in fr.mvuRight]
    for m in mps:
        if m is not None and hasattr(m, "mTrackProjXR"):
            m.mTrackProjXR = float(np.asarray(m.mTrackProjXR).ravel()[0])
    called = []
    orig = matcher.ORBMatcher._f_p_native

    def spy(self, *a):
        r = orig(self, *a)
        called.append(r)
        return r

    monkeypatch.setattr(matcher.ORBMatcher, "_csr", staticmethod(cpu_csr))
    monkeypatch.setattr(matcher.ORBMatcher, "_f_p_native", spy)
    n_native = matcher.ORBMatcher(0.8, True).search_by_projection_f_p(fr, mps, th)
    assert called and all(r is None for r in called)
    got = MF.encode_fp(fr, mps)
    fr2, mps2, th2, _, _ = MF.load_fp(case)
    fr2.mvuRight = [np.float32(v) if float(v) > 0 else v for v in fr2.mvuRight]
    for m in mps2:
        if m is not None and hasattr(m, "mTrackProjXR"):
            m.mTrackProjXR = float(np.asarray(m.mTrackProjXR).ravel()[0])
    monkeypatch.setattr(matcher.ORBMatcher, "_f_p_native", lambda self, *a: None)
    assert matcher.ORBMatcher(0.8, True).search_by_projection_f_p(fr2, mps2, th2) == n_native
    assert np.array_equal(MF.encode_fp(fr2, mps2), got)


def test_fp_inputs_equal_the_reference_loop():
    """search_by_projection_f_p's vectorised prologue (_f_p_inputs) keeps the reference loop's map points
    (tracked in view, then not bad), levels and radii (ORBMatcher.py:224-232, `r *= th` when th != 1), takes
    the radii point by point for a float32 view cosine (compares in float32), and declines (None) where the
    loop must run: an overridden radius_by_viewing_cos, a numpy th."""
    from pyorbslam_amd.matcher import ORBMatcher

    class MP:
        def __init__(self, inview, bad, vcos, lvl):
            self.mbTrackInView, self._bad, self.mTrackViewCos, self.mnTrackScaleLevel = inview, bad, vcos, lvl

        def is_bad(self):
            return self._bad

    rng = np.random.default_rng(3)
    kinds = [float, np.float64, lambda v: np.array([v], np.float64)]
    mps = [MP(bool(rng.random() < 0.8), bool(rng.random() < 0.1),
              kinds[i % 3](float(rng.choice([0.998, 0.9980001, 0.5, 0.9999, 1.0]))), int(rng.integers(0, 8)))
           for i in range(300)]

    def loop(m, th):
        out = ([], [], [])
        for p in mps:
            if not p.mbTrackInView or p.is_bad():
                continue
            r = m.radius_by_viewing_cos(p.mTrackViewCos)
            if th != 1.0:
                r *= th
            out[0].append(p), out[1].append(p.mnTrackScaleLevel), out[2].append(r)
        return out

    m = ORBMatcher(0.8, True)
    for th in (1, 1.0, 3, 2.5):
        got = m._f_p_inputs(mps, th, th != 1.0)
        ref = loop(m, th)
        assert got[0] == ref[0] and got[1] == ref[1]
        assert got[2] == ref[2] and all(type(v) is float for v in got[2])
    assert m._f_p_inputs(mps, np.float32(2.0), True) is None
    # a float32 view cosine: the radii go point by point (the float32 comparison), over the points already
    # selected — each point's mbTrackInView / is_bad() read once, as in the reference loop
    mps[0].mbTrackInView, mps[0]._bad, mps[0].mTrackViewCos = True, False, np.float32(0.998)
    calls = []
    for p in mps:
        p.is_bad = (lambda q=p: calls.append(q) or q._bad)
    for th in (1, 2.5):
        calls.clear()
        got = m._f_p_inputs(mps, th, th != 1.0)
        n_calls = len(calls)
        ref = loop(m, th)
        assert n_calls == sum(p.mbTrackInView for p in mps)
        assert got[0] == ref[0] and got[1] == ref[1] and got[2] == ref[2]
        assert [type(v) for v in got[2]] == [type(v) for v in ref[2]]

    class M2(ORBMatcher):
        def radius_by_viewing_cos(self, view_cos):
            return 3.0

    assert M2(0.8, True)._f_p_inputs(mps, 1, False) is None


def test_prime_u_right_equals_the_list_widening():
    """frame.compute_stereo_matches primes the matcher's per-frame mvuRight doubles from the stereo arrays;
    they equal what _u_right computes from the reference's list (same doubles, same all-double flag)."""
    from pyorbslam_amd import matcher as Mt
    from pyorbslam_amd.frame import to_reference_lists

    class Fr:
        pass

    rng = np.random.default_rng(3)
    for statuses in ((0, 1, 2), (0, 2), (1,)):
        n = 500
        st = rng.choice(statuses, n).astype(np.int8)
        u = rng.uniform(0, 1200, n).astype(np.float32)
        res = dict(u_right=u, depth=rng.uniform(1, 50, n).astype(np.float32), status=st)
        kps = np.zeros(n, dtype=[("x", np.float32)])
        kps["x"] = rng.uniform(0, 1240, n).astype(np.float32)
        for mbf in (386.1448, np.float64(386.1448)):
            a, b = Fr(), Fr()
            a.mvuRight, _ = to_reference_lists(res, kps, mbf)
            b.mvuRight = a.mvuRight
            Mt.prime_u_right(a, res, kps["x"])
            got, got_d = Mt._u_right(a, with_kinds=True)
            exp, exp_d = Mt._u_right(b, with_kinds=True)
            assert got.tobytes() == exp.tobytes() and got_d == exp_d
