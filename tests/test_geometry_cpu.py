"""Which image geometries the library accepts, decided on the host before any device work (build_geometry),
so it runs without a GPU: orbfe_batch_reserve either refuses a geometry with ORBFE_EINVAL and a message, or goes
on to allocate (ORBFE_ENOMEM without a device here; success on the GPU box).

Accepted (round 6): every level of at most 2^24 pixels whose geometry the reference's own DistributeOctTree
takes — level sides above 4 095 px (packed level keys hold the row-major pixel index, orbfe_common.h
kKeyXYBits), and widths past the ~5 600 px the resize band staging used to allow (16-row bands halve for
wider levels, LevelGeo::rs_rows).  Refused: more than 2^24 pixels in a level; tall levels whose nIni rounds to 0
(the reference indexes vpIniNodes out of range, ORBextractor.cpp:543-568)."""
import ctypes as C

import pytest

from pyorbslam_amd import _lib

EINVAL = -1


def reserve(w, h, scale=1.2, nlevels=8, nfeatures=2000):
    L = _lib.lib()
    p = _lib.make_params(nfeatures, scale, nlevels, 20, 7, 16)
    hd = C.c_void_p()
    assert L.orbfe_create(C.byref(p), C.byref(hd)) == 0
    try:
        rc = L.orbfe_batch_reserve(hd, w, h, 2)
        return rc, L.orbfe_last_error().decode(errors="replace")
    finally:
        L.orbfe_destroy(hd)


@pytest.mark.parametrize("wh", [(1241, 376), (752, 480), (4500, 600), (4500, 2300), (2500, 4500), (4096, 4096),
                                (6000, 600), (16000, 600), (12000, 1300), (27962, 600)])
def test_accepted_geometries(wh):
    rc, msg = reserve(*wh)
    assert rc != EINVAL, msg


@pytest.mark.parametrize("wh,needle", [((4200, 4000), "2^24"), ((27963, 600), "2^24"), ((3000, 6000), "2^24"),
                                       ((600, 4500), "DistributeOctTree"), ((2500, 6000), "DistributeOctTree")])
def test_refused_geometries(wh, needle):
    rc, msg = reserve(*wh)
    assert rc == EINVAL and needle in msg, (rc, msg)


def test_parameter_limits():
    """scale factors above 3.0 (the resize tap windows) and a level needing more than 150 KiB of
    octree LDS are refused; the reference's own parameters on large images are not."""
    assert reserve(1241, 376, 3.0, 2)[0] != EINVAL
    rc, msg = reserve(1241, 376, 3.2, 2)
    assert rc == EINVAL and "tap windows" in msg
    rc, msg = reserve(4000, 3000, 3.0, 2)
    assert rc == EINVAL and "octree LDS" in msg
    for wh in ((4000, 3000), (3840, 2160), (5000, 3000)):
        assert reserve(*wh, 1.2, 8, 4000)[0] != EINVAL
