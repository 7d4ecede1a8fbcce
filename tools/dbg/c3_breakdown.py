"""Debug aid: where the C3 Frame constructor's time goes (medians over the 96 recorded frames, GPU box).

Times, per frame: the pair enqueue + fetch (operator_kd_stereo), each ExtractORB call (tuples + KeyPoint
objects), GetImagePyramid, compute_stereo_matches, assign_features_to_grid and the whole constructor."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import seq_harness as H  # noqa: E402
from pyorbslam_amd import frame as F, synth  # noqa: E402
from pyorbslam_amd.matcher import ORBMatcher  # noqa: E402
from pyorbslam_amd.pyORBExtractor import ORBextractor  # noqa: E402

g = H.load_golden()
meta = json.loads(str(g["meta"]))
seq = synth.StereoSequence(meta["seq"]["seed"], meta["width"], meta["height"], meta["seq"]["speed"])
frames = [seq.frame(k) for k in range(meta["n_frames"])]
T: dict = {}


def timed(name, fn, *a, **k):
    t = time.perf_counter()
    try:
        return fn(*a, **k)
    finally:
        T.setdefault(name, []).append(time.perf_counter() - t)


import pyorbslam_amd.pyORBExtractor as PX  # noqa: E402

_call = PX.call


def _timed_call(name, *a):
    return timed("call:" + name, _call, name, *a)


PX.call = _timed_call
_rel = PX.ORBextractor._release_frame
PX.ORBextractor._release_frame = lambda self, **k: timed("release", _rel, self, **k)


class Cached:
    def frame(self, k):
        return frames[k]


class TEx(ORBextractor):
    def operator_kd_stereo(self, *a, **k):
        return timed("kd_stereo", super().operator_kd_stereo, *a, **k)

    def GetImagePyramid(self, *a, **k):
        return timed("pyramid", super().GetImagePyramid, *a, **k)


class DropInFrame(H.SeqFrame):
    pass


F.install(DropInFrame)


class TFrame(DropInFrame):
    def __init__(self, *a, **k):
        timed("ctor", super().__init__, *a, **k)

    def ExtractORB(self, flag, image):
        return timed(f"extract{flag}", super().ExtractORB, flag, image)

    def compute_stereo_matches(self):
        return timed("stereo", super().compute_stereo_matches)

    def assign_features_to_grid(self):
        return timed("grid", super().assign_features_to_grid)


ex = (TEx(**H.PARAMS), TEx(**H.PARAMS))
H.replay(g, Cached(), ex, ORBMatcher, TFrame, n_frames=3)
T.clear()
timer: dict = {}
bad = H.replay(g, Cached(), ex, ORBMatcher, TFrame, timer=timer)
print("bad", bad[:3])
T.update(timer)
for k, v in T.items():
    v = sorted(v)
    print(f"{k:10s} n={len(v):4d} p50 {1e3 * v[len(v) // 2]:.3f} ms  p90 {1e3 * v[int(len(v) * 0.9)]:.3f} ms")
for e in ex:
    st = e.graph_stats() if hasattr(e, "graph_stats") else None
    if st is None:
        c, l, n = C.c_int64(), C.c_int64(), C.c_int32()
        PX.call("orbfe_graph_stats", e.handle, C.byref(c), C.byref(l), C.byref(n))
        st = (c.value, l.value, n.value)
    print("graph captures / launches / cached", st)
