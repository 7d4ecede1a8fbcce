"""Debug aid: cProfile of the C3 replay's timed calls alone (the Frame constructor, search_by_projection_f_f /
_f_p) on the GPU box; prints their wall times and the profile of those calls only (argv[2]: sort key,
argv[3]: profile only this section: frame, f_f or f_p)."""
import cProfile
import json
import pstats
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
prof = cProfile.Profile()
T = {"f_f": [], "f_p": [], "frame": []}
on = [False]


ONLY = sys.argv[3] if len(sys.argv) > 3 else None


class PM(ORBMatcher):
    def search_by_projection_f_f(self, *a):
        if on[0] and ONLY in (None, "f_f"):
            prof.enable()
        t = time.perf_counter()
        try:
            return super().search_by_projection_f_f(*a)
        finally:
            prof.disable()
            T["f_f"].append(time.perf_counter() - t)

    def search_by_projection_f_p(self, *a):
        if on[0] and ONLY in (None, "f_p"):
            prof.enable()
        t = time.perf_counter()
        try:
            return super().search_by_projection_f_p(*a)
        finally:
            prof.disable()
            T["f_p"].append(time.perf_counter() - t)


class DropInFrame(H.SeqFrame):
    def __init__(self, *a, **k):
        if on[0] and ONLY in (None, "frame"):
            prof.enable()
        t = time.perf_counter()
        try:
            super().__init__(*a, **k)
        finally:
            prof.disable()
            T["frame"].append(time.perf_counter() - t)


F.install(DropInFrame)
ex = (ORBextractor(**H.PARAMS), ORBextractor(**H.PARAMS))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
bad = H.replay(g, seq, ex, PM, DropInFrame, n_frames=n)
print("bad", bad[:3])
for k, v in T.items():
    print(k, "median ms (unprofiled)", round(1e3 * sorted(v)[len(v) // 2], 3))
on[0] = True
H.replay(g, seq, ex, PM, DropInFrame, n_frames=n)
pstats.Stats(prof).sort_stats(sys.argv[2] if len(sys.argv) > 2 else "tottime").print_stats(40)
