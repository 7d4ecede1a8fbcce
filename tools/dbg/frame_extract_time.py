"""Debug aid: wall time of one orbfe_frame_extract (pair-batched Frame path), graphs on / off, with and without
the sheared pyramids; run under rocprofv3 --runtime-trace --stats for the HIP API time per call.
usage: python tools/dbg/frame_extract_time.py [iterations]"""
import ctypes as C
import sys
import time
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from pyorbslam_amd import synth  # noqa: E402
from pyorbslam_amd._lib import call, ptr  # noqa: E402
from pyorbslam_amd.pyORBExtractor import ORBextractor  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
L, R = synth.make_pair(3)
a, b = ORBextractor(2000, 1.2, 8, 20, 7), ORBextractor(2000, 1.2, 8, 20, 7)
h = a.handle
H, W = L.shape
for graphs in (1, 0):
    call("orbfe_set_graphs", h, graphs)
    for pyr in (1, 0):
        for _ in range(5):
            call("orbfe_frame_extract", h, ptr(L), ptr(R), W, H, W, 386.1448, float(np.float32(718.856)), pyr)
        ts = []
        for _ in range(n):
            t = time.perf_counter()
            call("orbfe_frame_extract", h, ptr(L), ptr(R), W, H, W, 386.1448, float(np.float32(718.856)), pyr)
            ts.append(time.perf_counter() - t)
        ts.sort()
        print(f"orbfe_frame_extract graphs {graphs} pyramid {pyr}: p50 {1e3 * ts[n // 2]:.3f} ms  min {1e3 * ts[0]:.3f}")
call("orbfe_set_graphs", h, 1)
for gap, spin in ((0.007, True), (0.007, False), (0.002, True)):  # host work (spin) or idle (sleep) between frames
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        if spin:
            while time.perf_counter() - t0 < gap:
                pass
        else:
            time.sleep(gap)
        t = time.perf_counter()
        call("orbfe_frame_extract", h, ptr(L), ptr(R), W, H, W, 386.1448, float(np.float32(718.856)), 1)
        ts.append(time.perf_counter() - t)
    ts.sort()
    print(f"orbfe_frame_extract after {1e3 * gap:.0f} ms {'spin' if spin else 'sleep'}: p50 {1e3 * ts[50]:.3f} ms  min {1e3 * ts[0]:.3f}")
t = time.perf_counter()
for _ in range(50):
    a.operator_kd_stereo(L, R, b, 386.1448, np.float32(718.856))
print("operator_kd_stereo ms", round((time.perf_counter() - t) / 50 * 1e3, 3))
t = time.perf_counter()
for _ in range(50):
    a.GetImagePyramid()
    b.GetImagePyramid()
print("GetImagePyramid x2 ms", round((time.perf_counter() - t) / 50 * 1e3, 3))
