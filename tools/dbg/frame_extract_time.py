"""Debug aid: wall time of one orbfe_frame_extract (pair-batched Frame path) and of its pieces."""
import sys
import time
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from pyorbslam_amd import synth
from pyorbslam_amd.pyORBExtractor import ORBextractor
L, R = synth.make_pair(3)
a, b = ORBextractor(2000, 1.2, 8, 20, 7), ORBextractor(2000, 1.2, 8, 20, 7)
for pyr in (True, False):
    for _ in range(5):
        a.operator_kd_stereo(L, R, b, 386.1448, np.float32(718.856), want_pyramid=pyr)
    t = time.perf_counter()
    for _ in range(50):
        a.operator_kd_stereo(L, R, b, 386.1448, np.float32(718.856), want_pyramid=pyr)
    print("operator_kd_stereo pyramid", pyr, "ms", round((time.perf_counter() - t) / 50 * 1e3, 3))
t = time.perf_counter()
for _ in range(50):
    a.GetImagePyramid(); b.GetImagePyramid()
print("GetImagePyramid x2 ms", round((time.perf_counter() - t) / 50 * 1e3, 3))
