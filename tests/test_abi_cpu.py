"""The C-ABI library loads on a GPU-less host and exports exactly what include/orbfe.h declares
(no compute calls here)."""
import ctypes as C
import re
import subprocess

from conftest import ROOT

HEADER = ROOT / "include" / "orbfe.h"


def declared():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(orbfe_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    names = declared()
    for must in ["orbfe_create", "orbfe_extract", "orbfe_pyramid", "orbfe_stereo_match", "orbfe_hamming_search",
                 "orbfe_frontend_batch_device"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    from pyorbslam_amd import _lib
    L = _lib.lib()
    for n in declared():
        assert hasattr(L, n), n
    out = subprocess.check_output(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)]).decode()
    exported = set(re.findall(r" T (orbfe_\w+)", out))
    assert exported == set(declared())
    assert set(_lib.SIGNATURES) == set(declared())


def test_struct_layouts():
    from pyorbslam_amd import _lib
    assert C.sizeof(_lib.Params) == 24
    assert _lib.KP_DTYPE.itemsize == 24
    assert _lib.version().startswith("orbfe")


def test_create_and_tables_without_gpu():
    """Handle creation and the scale tables are host-only (ORBextractor.cpp:410-470)."""
    from pyorbslam_amd.pyORBExtractor import ORBextractor
    from oracle.oracle import OracleExtractor
    e = ORBextractor(2000, 1.2, 8, 20, 7)
    t = OracleExtractor(2000, 1.2, 8, 20, 7).tables()
    assert e.GetScaleFactors() == [float(v) for v in t["scale"]]
    assert e.GetInverseScaleFactors() == [float(v) for v in t["inv_scale"]]
    assert e.GetScaleSigmaSquares() == [float(v) for v in t["sigma2"]]
    assert e.GetInverseScaleSigmaSquares() == [float(v) for v in t["inv_sigma2"]]
    assert e.features_per_level() == t["n_per_level"].tolist()
    assert e.GetLevels() == 8 and e.GetScaleFactor() == 1.2000000476837158


def test_bad_params_fail_loudly():
    import pytest
    from pyorbslam_amd._lib import OrbfeError
    from pyorbslam_amd.pyORBExtractor import ORBextractor
    with pytest.raises(OrbfeError):
        ORBextractor(2000, 1.2, 0, 20, 7)
    with pytest.raises(OrbfeError):
        ORBextractor(2000, 1.2, 8, 20, 7, resize_simd_lanes=8)


def test_driver_scripts_compile():
    """bench.py, __graft_entry__.py and the tools compile (the driver runs them on the GPU box)."""
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    for f in [root / "bench.py", root / "__graft_entry__.py", *sorted((root / "tools").glob("*.py"))]:
        compile(f.read_text(), str(f), "exec")
