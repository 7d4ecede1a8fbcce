"""Generate reference goldens for the keyframe-level ORBMatcher searches and
MapPoint.compute_distinctive_descriptors (build container only; the reference never travels).

Imports the REFERENCE ORBMatcher.py and MapPoint.py read-only from /root/reference (both import only
numpy / threading), runs them on stand-in worlds (tests/matcher_world.py) built from seeded arrays, and
stores the arrays plus every result and side effect in tests/golden/matcher_kf_<case>.npz and
tests/golden/mappoint_distinctive.npz.

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_matcher_kf.py
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import matcher_world as MW  # noqa: E402

REF = Path("/root/reference")
# case 4: sparse vocabulary words (feature vectors mostly disjoint); cases 5, 6: tiny keyframes whose
# feature vectors end so that search_for_triangulation's merge lets StopIteration escape (5) or not (6)
N_CASES = 7
SEEDS = [9000, 9001, 9002, 9003, 9004, 9103, 9100]
SIZES = [(1000, 600, 160), (1400, 900, 160), (700, 450, 160), (1000, 700, 160), (900, 600, 3000), (40, 25, 5000),
         (40, 25, 5000)]


def import_reference():
    sys.path.insert(0, str(REF))
    import ORBMatcher as RMatcher  # noqa: E402
    import MapPoint as RMapPoint  # noqa: E402
    return RMatcher, RMapPoint


_SEL = {}


def res_pts(z, rng, key):
    """Selections of map points / slots per search, drawn once per case and stored with the golden."""
    if key in _SEL:
        return _SEL[key]
    n_mp = len(z["mp_desc"])
    n_kf1 = len(z["kf1_x"])
    if key == "fuse_scw":
        v = rng.choice(n_mp, n_mp // 2, replace=False).astype(np.int32)
    elif key == "fuse_p":
        v = rng.choice(n_mp, n_mp // 2, replace=False).astype(np.int32)
        v = np.concatenate([v, v[:40], np.full(10, -1, np.int32)])
        v = v[rng.permutation(len(v))]
    elif key == "sim3":
        slots = np.nonzero(z["kfmp1"] >= 0)[0]
        obs0 = {int(m): int(i) for m, k, i in z["obs"] if k == 0}
        pairs = [(obs0[int(z["kfmp1"][i2])], int(i2)) for i2 in slots[:30] if int(z["kfmp1"][i2]) in obs0]
        v = np.array(pairs, np.int32).reshape(-1, 2)
    elif key == "ckf_pts":
        v = rng.choice(n_mp, n_mp // 2, replace=False).astype(np.int32)
    elif key == "ckf_matched":
        v = np.full(n_kf1, -1, np.int32)
        k = min(40, n_kf1 // 4, n_mp)
        idx = rng.choice(n_kf1, k, replace=False)
        v[idx] = rng.choice(n_mp, k, replace=False)
    elif key == "fkf_found":
        v = rng.choice(n_mp, min(30, n_mp // 3), replace=False).astype(np.int32)
    _SEL[key] = v
    return v


def gen_distinctive(RMapPoint):
    """MapPoint.compute_distinctive_descriptors (MapPoint.py:204-240) on stand-in observations."""
    import threading
    rng = np.random.Generator(np.random.PCG64(77))
    w = MW.World()
    kfd = rng.integers(0, 256, (12, 400, 32), dtype=np.uint8)

    class KFD:
        def __init__(self, j, bad):
            self.mDescriptors = kfd[j]
            self._bad = bad

        def is_bad(self):
            return self._bad

    kfs = [KFD(j, j == 11) for j in range(12)]
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    obs_k, obs_i, obs_off, bad, out = [], [], [0], [], []
    for p in range(300):
        n_obs = int(rng.choice([0, 1, 2, 3, 5, 8, 12]))
        ks = rng.choice(12, n_obs, replace=False)
        # descriptors near a per-point centre, so medians differ and ties happen at small n
        centre = MW.noisy_desc(rng, base, int(rng.integers(0, 80)))
        for k in ks:
            i = int(rng.integers(0, 400))
            kfd[k, i] = MW.noisy_desc(rng, centre, int(rng.integers(0, 40)))
            obs_k.append(int(k))
            obs_i.append(i)
        obs_off.append(len(obs_k))
        bad.append(bool(rng.random() < 0.05))
    # every descriptor is final before the first point reads it
    for p in range(300):
        mp = object.__new__(RMapPoint.MapPoint)
        mp.mMutexFeatures = threading.Lock()
        mp.mbBad = bad[p]
        mp.mObservations = {kfs[int(k)]: int(i) for k, i in zip(obs_k[obs_off[p]:obs_off[p + 1]],
                                                                 obs_i[obs_off[p]:obs_off[p + 1]])}
        mp.mDescriptor = np.zeros(32, np.uint8)
        mp.compute_distinctive_descriptors()
        out.append(mp.mDescriptor.copy())
    del w
    np.savez_compressed(HERE / "mappoint_distinctive.npz", kf_desc=kfd, kf_bad=np.arange(12) == 11,
                        obs_k=np.array(obs_k, np.int32), obs_i=np.array(obs_i, np.int32),
                        obs_off=np.array(obs_off, np.int32), mp_bad=np.array(bad), out=np.stack(out))


def main():
    RMatcher, RMapPoint = import_reference()
    for case in range(N_CASES):
        rng = np.random.Generator(np.random.PCG64(SEEDS[case]))
        n, n_mp, n_words = SIZES[case]
        z = MW.make_world(rng, n_kf=2, n=n, n_mp=n_mp, with_frame=True, n_words=n_words)
        arr = _Arrays(z)
        _SEL.clear()
        res = MW.drive(RMatcher.ORBMatcher, arr, case, lambda key: res_pts(arr, rng, key))
        sel = {f"sel_{k}": v for k, v in _SEL.items()}
        np.savez_compressed(HERE / f"matcher_kf_{case}.npz", **z, **sel, **res)
        print(f"case {case}:", {k: int(v) for k, v in res.items() if k.endswith("_n") or k.endswith("_stop")},
              "tri pairs", len(res["tri0_pairs"]), len(res["tri1_pairs"]), "fuse events", len(res["fp_log"]))
    gen_distinctive(RMapPoint)


class _Arrays:
    """dict of arrays with the np.load(...) interface MW.build expects (.files, [key])."""

    def __init__(self, d):
        self._d = d
        self.files = list(d.keys())

    def __getitem__(self, k):
        return self._d[k]


if __name__ == "__main__":
    main()
