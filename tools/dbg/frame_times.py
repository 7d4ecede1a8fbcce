"""Debug aid: per-frame stage times of the C3 replay (outliers), with and without the cyclic GC."""
import gc
import json
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
for gc_on in (True, False):
    if not gc_on:
        gc.disable()
    timer = {}
    H.replay(g, Cached(), ex, ORBMatcher, DropInFrame, timer=timer)
    print("gc", gc_on)
    for k in range(len(timer["frame"])):
        print(k, " ".join(f"{n}={1e3 * timer[n][k]:.2f}" for n in ("frame", "f_f", "f_p")))
