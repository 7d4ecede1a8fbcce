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
