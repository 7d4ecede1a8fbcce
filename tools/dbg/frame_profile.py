"""Debug aid: cProfile of the C3 per-frame replay (bench.py --mode frame's loop) on the GPU box."""
import cProfile
import json
import pstats
import sys
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


class Cached:
    def frame(self, k):
        return frames[k]


class DropInFrame(H.SeqFrame):
    pass


F.install(DropInFrame)
ex = (ORBextractor(**H.PARAMS), ORBextractor(**H.PARAMS))
H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, n_frames=3)
timer = {}
pr = cProfile.Profile()
pr.enable()
bad = H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, timer=timer)
pr.disable()
print("bad", bad[:3])
for k, v in timer.items():
    print(k, "median ms", round(1e3 * sorted(v)[len(v) // 2], 3))
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
