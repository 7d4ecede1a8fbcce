"""Container-only: time the REFERENCE's Frame.compute_stereo_matches (imported read-only from
/root/reference, as tests/golden/gen_golden.py does) against oracle/stereo_loop.py (the restatement that
bench.py's cpu_baseline times on the GPU box, where the reference cannot go) on the same synthetic pairs,
1 thread, and record the ratio in profiles/cpu_ratio.json.  The extractor has no such ratio: the
reference's C++ extractor needs OpenCV, which is absent, so its CPU time is the oracle's.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_ratio.py [n_pairs]
"""
from __future__ import annotations

import json
import platform
import sys
import time
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

from gen_golden import BF, FX, import_reference, reference_stereo  # noqa: E402
from oracle import stereo_oracle  # noqa: E402
from oracle.oracle import OracleExtractor  # noqa: E402
from oracle.stereo_loop import compute_stereo_matches_loop  # noqa: E402
from pyorbslam_amd import synth  # noqa: E402


def cpu_model() -> str:
    for line in Path("/proc/cpuinfo").read_text().splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main(n: int = 8):
    RFrame, _ = import_reference()
    prm = dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    t_ext = t_ref = t_loop = t_vec = 0.0
    for i in range(n):
        L, R = synth.make_pair(10_000 + i)
        exL, exR = OracleExtractor(**prm), OracleExtractor(**prm)
        t0 = time.perf_counter()
        kl, dl = exL.extract(L)
        kr, dr = exR.extract(R)
        t_ext += time.perf_counter() - t0
        pl, pr, tab = exL.sheared_pyramid(), exR.sheared_pyramid(), exL.tables()
        t0 = time.perf_counter()
        ru, rd = reference_stereo(RFrame, kl, dl, kr, dr, pl, pr, tab)
        t1 = time.perf_counter()
        lu, ld = compute_stereo_matches_loop(kl, kr, dl, dr, pl, pr, tab["scale"], tab["inv_scale"], BF, np.float32(FX))
        t2 = time.perf_counter()
        stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, pl, pr, tab["scale"], tab["inv_scale"], BF, np.float32(FX))
        t3 = time.perf_counter()
        t_ref, t_loop, t_vec = t_ref + t1 - t0, t_loop + t2 - t1, t_vec + t3 - t2
        for a, b in ((ru, lu), (rd, ld)):
            sa, va = stereo_oracle.encode(a)
            sb, vb = stereo_oracle.encode(b)
            assert np.array_equal(sa, sb) and np.array_equal(va, vb), "restatement differs from the reference"
    out = dict(pairs=n, host=cpu_model(), threads=1, python=platform.python_version(), numpy=np.__version__,
               oracle_extract_s_per_pair=t_ext / n, reference_stereo_s_per_pair=t_ref / n,
               loop_restatement_stereo_s_per_pair=t_loop / n, vectorised_checker_stereo_s_per_pair=t_vec / n,
               ratio_reference_over_loop=t_ref / t_loop,
               note="reference = /root/reference/Frame.py compute_stereo_matches imported read-only; extractor "
                    "time is the oracle's (the reference C++ extractor needs OpenCV, absent)")
    (ROOT / "profiles").mkdir(exist_ok=True)
    (ROOT / "profiles" / "cpu_ratio.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
