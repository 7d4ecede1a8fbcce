import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

KITTI = dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
EUROC = dict(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
BF = 386.1448
FX = 718.856


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def pytest_collection_modifyitems(config, items):
    have_gpu = None
    for it in items:
        if "gpu" in it.keywords:
            if have_gpu is None:
                try:
                    import torch
                    have_gpu = torch.cuda.is_available()
                except Exception:
                    have_gpu = False
            if not have_gpu:
                it.add_marker(pytest.mark.skip(reason="no GPU in this environment"))


@pytest.fixture(scope="session")
def kitti_png():
    from PIL import Image
    return np.array(Image.open(GOLDEN / "kitti06-436.png").convert("L"))


def load_golden(name):
    z = np.load(GOLDEN / f"stereo_{name}.npz", allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_case_images(name, kitti_png=None):
    """Regenerate the input pair of a stereo golden from its recorded recipe."""
    import json
    from pyorbslam_amd import synth
    g = load_golden(name)
    meta = json.loads(str(g["meta"]))
    if meta["kind"] == "synth":
        L, R = synth.make_pair(meta["seed"], meta["w"], meta["h"])
    elif meta["kind"] == "identical":
        L, _ = synth.make_pair(meta["seed"])
        R = L.copy()
    else:
        L = kitti_png
        R = synth.shifted_right(L, seed=meta["right_seed"])
    return L, R, meta["params"], g


STEREO_CASES = ["kitti_synth_s0", "kitti_synth_s1", "kitti_synth_s2", "kitti06_436", "euroc_synth_s100",
                "identical_s3"]
