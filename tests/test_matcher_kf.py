"""Keyframe-level ORBMatcher searches and MapPoint.compute_distinctive_descriptors against goldens made
by the reference itself (tests/golden/gen_golden_matcher_kf.py).

CPU tests drive pyorbslam_amd.matcher's host control flow with distances from the oracle's numpy
popcount (the GPU is replaced only there); GPU tests run the real path (k_hamming_search)."""
import threading

import numpy as np
import pytest

import matcher_world as MW
from conftest import GOLDEN
from oracle import matcher_oracle as MO

CASES = range(7)
# the stand-in grid search converts 1-element arrays to int exactly as the reference's callers feed it
pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


def load(case):
    return np.load(GOLDEN / f"matcher_kf_{case}.npz", allow_pickle=False)


def _cpu_batched(queries, train):
    return [np.array([MO.dist(d, train[i]) for i in c], np.int32) for d, c in queries]


def check_case(Matcher, case):
    z = load(case)
    res = MW.drive(Matcher, z, case, lambda key: z[f"sel_{key}"])
    for k, v in res.items():
        g = z[k]
        assert np.asarray(v).shape == g.shape and np.array_equal(np.asarray(v), g), f"case {case}: {k} differs"


def cpu_matcher(monkeypatch):
    from pyorbslam_amd import matcher
    monkeypatch.setattr(matcher.ORBMatcher, "_batched", staticmethod(_cpu_batched))
    return matcher.ORBMatcher


@pytest.mark.parametrize("case", CASES)
def test_kf_searches_host_logic_golden(case, monkeypatch):
    check_case(cpu_matcher(monkeypatch), case)


def test_triangulation_stop_iteration_escapes(monkeypatch):
    """Case 5's feature vectors end so that the reference's merge walk raises StopIteration."""
    z = load(5)
    assert int(z["tri0_stop"]) == 1 and int(z["tri1_stop"]) == 1
    assert int(load(6)["tri0_stop"]) == 0
    M = cpu_matcher(monkeypatch)
    w = MW.build(z)
    with pytest.raises(StopIteration):
        M(0.7, True).search_for_triangulation(w.kfs[0], w.kfs[1], z["tri0_F12"], False)


class _KFD:
    def __init__(self, desc, bad):
        self.mDescriptors = desc
        self._bad = bool(bad)

    def is_bad(self):
        return self._bad


class _MP:
    def __init__(self, obs, bad):
        self.mMutexFeatures = threading.Lock()
        self.mbBad = bool(bad)
        self.mObservations = obs
        self.mDescriptor = np.zeros(32, np.uint8)


def distinctive_points():
    z = np.load(GOLDEN / "mappoint_distinctive.npz", allow_pickle=False)
    kfs = [_KFD(z["kf_desc"][j], z["kf_bad"][j]) for j in range(len(z["kf_desc"]))]
    off = z["obs_off"]
    mps = [_MP({kfs[int(k)]: int(i) for k, i in zip(z["obs_k"][off[p]:off[p + 1]], z["obs_i"][off[p]:off[p + 1]])},
               z["mp_bad"][p]) for p in range(len(off) - 1)]
    return mps, z["out"]


def test_distinctive_host_logic_golden(monkeypatch):
    from pyorbslam_amd import mappoint
    monkeypatch.setattr(mappoint, "hamming_matrix",
                        lambda a, b: np.array([[MO.dist(x, y) for y in b] for x in a], np.int32))
    mps, out = distinctive_points()
    for mp in mps:
        mappoint.compute_distinctive_descriptors(mp)
    assert np.array_equal(np.stack([m.mDescriptor for m in mps]), out)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_kf_searches_gpu_golden(case):
    from pyorbslam_amd.matcher import ORBMatcher
    check_case(ORBMatcher, case)


@pytest.mark.gpu
def test_distinctive_gpu_golden():
    from pyorbslam_amd import mappoint
    mps, out = distinctive_points()
    for mp in mps:
        mappoint.compute_distinctive_descriptors(mp)
    assert np.array_equal(np.stack([m.mDescriptor for m in mps]), out)
    mps, out = distinctive_points()
    mappoint.compute_distinctive_descriptors_many(mps)
    assert np.array_equal(np.stack([m.mDescriptor for m in mps]), out)
