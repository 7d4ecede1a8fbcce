"""GPU parity of the extractor, stage by stage, against the CPU oracle (bit-exact: integer pixels,
integer keypoint coordinates / scores, float32 keypoint fields compared bitwise, descriptor bytes)."""
import ctypes as C

import numpy as np
import pytest

from conftest import KITTI, EUROC
from oracle import oracle as O
from pyorbslam_amd import synth
from pyorbslam_amd._lib import call, ptr
from pyorbslam_amd.pyORBExtractor import ORBextractor

pytestmark = pytest.mark.gpu
NAMES = ["kitti_L", "kitti_R", "kitti06", "euroc", "noise", "small", "odd", "patch", "clusters"]


def _images(kitti_png):
    L0, R0 = synth.make_pair(0)
    Le, _ = synth.make_pair(100, 752, 480)
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (376, 1241)).astype(np.uint8)
    small = synth.make_pair(9, 211, 157)[0]
    odd = synth.make_pair(11, 641, 333)[1]
    # octree stress: every candidate of a level inside one small patch (the list divides far below the
    # depth k_octree_bins keeps bins for), and a few dense clusters on a flat image
    patch = np.full((376, 1241), 90, np.uint8)
    patch[170:202, 600:632] = rng.integers(0, 256, (32, 32))
    clusters = np.full((376, 1241), 120, np.uint8)
    for cy, cx in ((60, 100), (64, 130), (300, 1100), (200, 640), (205, 655)):
        clusters[cy:cy + 14, cx:cx + 14] = rng.integers(0, 256, (14, 14))
    return {"kitti_L": (L0, KITTI), "kitti_R": (R0, KITTI), "kitti06": (kitti_png, KITTI), "euroc": (Le, EUROC),
            "noise": (noise, KITTI), "small": (small, dict(KITTI, nfeatures=500)), "odd": (odd, KITTI),
            "patch": (patch, KITTI), "clusters": (clusters, KITTI)}


def _debug(ex, fn, level, cap=400000):
    buf = np.zeros((cap, 3), np.int32)
    n = C.c_int32()
    call(fn, ex.handle, level, ptr(buf), cap, C.byref(n))
    return buf[:n.value].copy()


def _first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i].tobytes() != b[i].tobytes():
            return i, a[i], b[i]
    return n, None, None


@pytest.fixture(scope="module")
def cases(kitti_png):
    out = {}
    for name, (img, params) in _images(kitti_png).items():
        ex = ORBextractor(**params)
        kps, desc = ex.extract(img)
        orc = O.OracleExtractor(**params)
        okps, odesc = orc.extract(img)
        out[name] = (img, params, ex, kps.copy(), desc.copy(), orc, okps, odesc)
    return out


@pytest.mark.parametrize("name", NAMES)
def test_pyramid(cases, name):
    img, params, ex, *_rest = cases[name]
    orc = cases[name][5]
    for l, (g, o) in enumerate(zip(ex.GetImagePyramid(sheared=False), orc.pyramid())):
        assert g.shape == o.shape and np.array_equal(g, o), f"level {l}"
    for l, (g, o) in enumerate(zip(ex.GetImagePyramid(), orc.sheared_pyramid())):
        assert np.array_equal(g, o), f"sheared level {l}"


@pytest.mark.parametrize("name", NAMES)
def test_fast_cells(cases, name):
    img, params, ex, kps, desc, orc, okps, odesc = cases[name]
    p = O.Params(params["nfeatures"], params["scaleFactor"], params["nlevels"], params["iniThFAST"],
                 params["minThFAST"], 16)
    for l, lvl in enumerate(orc.pyramid()):
        got = _debug(ex, "orbfe_debug_candidates", l)
        exp = O.level_candidates(p, lvl)
        assert len(got) == len(exp), f"level {l}: {len(got)} vs {len(exp)}"
        i, a, b = _first_diff(got, exp)
        assert a is None, f"level {l} first diff at {i}: {a} vs {b}"


@pytest.mark.parametrize("name", NAMES)
def test_octree(cases, name):
    img, params, ex, kps, desc, orc, okps, odesc = cases[name]
    npl = ex.features_per_level()
    for l, lvl in enumerate(orc.pyramid()):
        h, w = lvl.shape
        cand = _debug(ex, "orbfe_debug_candidates", l)
        got = _debug(ex, "orbfe_debug_selected", l)
        exp = O.octree(cand, 16, w - 16, 16, h - 16, npl[l])
        assert len(got) == len(exp), f"level {l}: {len(got)} vs {len(exp)}"
        i, a, b = _first_diff(got, exp)
        assert a is None, f"level {l} first diff at {i}: {a} vs {b}"


@pytest.mark.parametrize("name", NAMES)
def test_keypoints_and_descriptors_bit_exact(cases, name):
    img, params, ex, kps, desc, orc, okps, odesc = cases[name]
    assert len(kps) == len(okps)
    for f in ("x", "y", "size", "angle", "response", "octave"):
        i, a, b = _first_diff(kps[f], okps[f])
        assert a is None, f"field {f} differs at {i}: {a} vs {b}"
    assert desc.shape == odesc.shape
    bad = np.nonzero((desc != odesc).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} descriptors differ, first at {bad[:5]} (octaves {kps['octave'][bad[:5]]})"


def test_operator_kd_surface(cases):
    img, params, ex, kps, desc, orc, okps, odesc = cases["kitti_L"]
    tuples, d = ex.operator_kd(img)
    assert isinstance(tuples, list) and isinstance(tuples[0], tuple) and len(tuples[0]) == 6
    assert all(isinstance(v, float) for v in tuples[0][:5]) and isinstance(tuples[0][5], int)
    assert d.dtype == np.uint8 and d.shape == (len(tuples), 32)
    assert np.array_equal(d, odesc)
    assert tuples[0] == tuple(float(okps[0][f]) for f in ("x", "y", "size", "angle", "response")) + (
        int(okps[0]["octave"]),)


def test_empty_and_featureless_images():
    ex = ORBextractor(**KITTI)
    t, d = ex.operator_kd(np.zeros((0, 0), np.uint8))
    assert t == [] and d.shape == (0, 0)
    t, d = ex.operator_kd(np.full((376, 1241), 77, np.uint8))  # flat: no FAST corner anywhere
    assert t == [] and d.shape == (0, 0)
    with pytest.raises(RuntimeError):
        ex.operator_kd(np.zeros((10, 10), np.float64))


@pytest.mark.parametrize("simd", [0, 32])
def test_resize_simd_modes(simd):
    img, _ = synth.make_pair(4)
    ex = ORBextractor(**KITTI, resize_simd_lanes=simd)
    kps, desc = ex.extract(img)
    orc = O.OracleExtractor(**KITTI, resize_simd_lanes=simd)
    okps, odesc = orc.extract(img)
    for g, o in zip(ex.GetImagePyramid(sheared=False), orc.pyramid()):
        assert np.array_equal(g, o)
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)


def test_deterministic_repeat(cases):
    img, params, ex, kps, desc, *_ = cases["kitti06"]
    for _ in range(3):
        k2, d2 = ex.extract(img)
        assert k2.tobytes() == kps.tobytes() and np.array_equal(d2, desc)


# extractor configurations other than the two cameras' (ORBextractor(nfeatures, scaleFactor, nlevels,
# iniThFAST, minThFAST), ORBextractor.cpp:410-470): feature budgets, scale factors / level counts,
# thresholds (including iniTh == minTh, where the fallback cannot change anything), other image sizes
CONFIGS = [
    ((376, 1241), dict(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)),
    ((376, 1241), dict(nfeatures=3000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)),
    ((376, 1241), dict(nfeatures=2000, scaleFactor=1.1, nlevels=12, iniThFAST=20, minThFAST=7)),
    ((376, 1241), dict(nfeatures=2000, scaleFactor=1.5, nlevels=5, iniThFAST=20, minThFAST=7)),
    ((376, 1241), dict(nfeatures=1200, scaleFactor=1.3, nlevels=4, iniThFAST=12, minThFAST=5)),
    ((376, 1241), dict(nfeatures=2000, scaleFactor=1.2, nlevels=1, iniThFAST=20, minThFAST=7)),
    ((376, 1241), dict(nfeatures=500, scaleFactor=1.2, nlevels=8, iniThFAST=30, minThFAST=15)),
    ((376, 1241), dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=9, minThFAST=9)),
    ((720, 1280), dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)),
    ((1080, 1920), dict(nfeatures=4000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)),
    # exact 2x steps (cv::resize's INTER_AREA fast path: 620x188 -> 310x94 -> 155x47; the
    # first step, 1241 -> 620, is linear), and levels of 19 px or less (iterated reflect-101 padding)
    ((376, 1241), dict(nfeatures=2000, scaleFactor=2.0, nlevels=4, iniThFAST=20, minThFAST=7)),
    ((400, 400), dict(nfeatures=1000, scaleFactor=2.0, nlevels=6, iniThFAST=20, minThFAST=7)),
    ((128, 128), dict(nfeatures=300, scaleFactor=1.2, nlevels=12, iniThFAST=20, minThFAST=7)),
]


@pytest.mark.parametrize("ci", range(len(CONFIGS)))
def test_extractor_configurations_bit_exact(ci):
    (h, w), params = CONFIGS[ci]
    img = synth.make_pair(200 + ci, w, h)[0]
    kps, desc = ORBextractor(**params).extract(img)
    okps, odesc = O.OracleExtractor(**params).extract(img)
    assert len(kps) == len(okps) and len(kps) > 0
    i, a, b = _first_diff(kps, okps)
    assert i == len(kps), f"{params}: keypoint {i} differs: {a} vs {b}"
    assert np.array_equal(desc, odesc), f"{params}: descriptors differ"


def test_octree_key_walk_fallback():
    """k_octree_bins keeps every key's cell in the node-list LDS when the level's keys fit (about 2 800 at
    nfeatures = 100: 25-node lists); the noise image's level 0 holds far more, so its first sweep walks each
    key's cell from its 16-key block's first cell instead.  Both paths must select the reference's keys."""
    rng = np.random.default_rng(21)
    img = rng.integers(0, 256, (376, 1241)).astype(np.uint8)
    params = dict(KITTI, nfeatures=100)
    ex = ORBextractor(**params)
    kps, desc = ex.extract(img)
    assert len(_debug(ex, "orbfe_debug_candidates", 0)) > 8000
    okps, odesc = O.OracleExtractor(**params).extract(img)
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)
    npl = ex.features_per_level()
    cand = _debug(ex, "orbfe_debug_candidates", 0)
    exp = O.octree(cand, 16, 1241 - 16, 16, 376 - 16, npl[0])
    assert np.array_equal(_debug(ex, "orbfe_debug_selected", 0), exp)


def test_strided_view_input_follows_the_reference_caster():
    """A sliced ROI view is read as nh x nw consecutive bytes from its first element (the reference caster
    ignores strides, opencv_type_casters.h:200): the drop-in's result equals the oracle's on those bytes and
    differs from the result on the pixels the view shows (tests/test_input_contract.py pins the bytes)."""
    img, _ = synth.make_pair(8)
    v = img[30:330, 150:1000]
    nh, nw = v.shape
    first = 30 * img.shape[1] + 150
    raw = img.reshape(-1)[first:first + nh * nw].reshape(nh, nw).copy()
    kps, desc = ORBextractor(**KITTI).extract(v)
    okps, odesc = O.OracleExtractor(**KITTI).extract(raw)
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)
    shown, _ = O.OracleExtractor(**KITTI).extract(np.ascontiguousarray(v))
    assert shown.tobytes() != kps.tobytes()


@pytest.mark.parametrize("ci", [len(CONFIGS) - 2, len(CONFIGS) - 1])
def test_tiny_levels_sheared_pyramid(ci):
    """Levels of 19 px or less: GetImagePyramid's sheared views read the 19-px padding, which reflects more than
    once (copyMakeBorder REFLECT_101, ORBextractor.cpp:1122-1128) — against the oracle's view of each level."""
    (h, w), params = CONFIGS[ci]
    img = synth.make_pair(300 + ci, w, h)[0]
    ex = ORBextractor(**params)
    ex.extract(img)
    oe = O.OracleExtractor(**params)
    oe.extract(img)
    got, want = ex.GetImagePyramid(), oe.sheared_pyramid()
    assert len(got) == len(want) and min(p.shape[0] for p in want) <= 19
    for l, (a, b) in enumerate(zip(got, want)):
        assert a.shape == b.shape and np.array_equal(a, b), f"level {l}"


def test_reference_refused_geometries_gpu():
    """A level lower than 32 px but wider makes the reference's DistributeOctTree throw (vpIniNodes.resize of a
    negative nIni, ORBextractor.cpp:543-550; pybind11 raises std::length_error as ValueError): the drop-in
    raises ValueError for the same geometries, the oracle too."""
    for (h, w), prm in (((96, 160), dict(KITTI, nlevels=12)), ((376, 1241), dict(KITTI, scaleFactor=2.0))):
        img = synth.make_pair(5, w, h)[0]
        with pytest.raises(ValueError):
            ORBextractor(**prm).extract(img)
        with pytest.raises(ValueError):
            O.OracleExtractor(**prm).extract(img)


# level sides above 4 095 px.  The packed level keys hold a pixel's row-major index in 24
# bits (orbfe_common.h kKeyXYBits), so every level of at most 2^24 pixels is accepted, whatever its aspect.
# (h, w): wide-short, wide, tall (level 0 above 4 095 px); then widths whose resize bands need fewer than 16 rows
# to fit the LDS (LevelGeo::rs_rows) and whose level-0 octree takes the per-candidate k_octree (bins past 150 KiB)
BIG = [(600, 4500), (2300, 4500), (4500, 2500), (600, 16000), (1300, 12000)]


@pytest.mark.parametrize("hw", BIG)
def test_level_sides_above_4095_px_bit_exact(hw):
    """One extraction of a 4 500 px wide (or high) image — the cascade pyramid, FAST cells, the octree over
    a level of more than 4 096 columns (or rows), k_orb — and its sheared pyramid, against the oracle."""
    h, w = hw
    img = synth.make_pair(410 + w % 7, w, h)[0]
    ex = ORBextractor(**KITTI)
    kps, desc = ex.extract(img)
    oe = O.OracleExtractor(**KITTI)
    okps, odesc = oe.extract(img)
    assert len(kps) > 1000
    i, a, b = _first_diff(kps, okps)
    assert i == len(kps) == len(okps), f"{hw}: keypoint {i} differs: {a} vs {b}"
    assert np.array_equal(desc, odesc)
    k0 = kps[kps["octave"] == 0]
    assert max(k0["x"].max(), k0["y"].max()) > 4095
    got, want = ex.GetImagePyramid(), oe.sheared_pyramid()
    for l, (p, q) in enumerate(zip(got, want)):
        assert p.shape == q.shape and np.array_equal(p, q), f"{hw} level {l}"


def test_level_sides_above_4095_px_frame_and_batch():
    """The 4 500 x 600 geometry through the per-frame stereo path (both extractions, the row buckets fused in
    k_orb, k_stereo, the lazy sheared views) and through a 16-pair batch (32 images: the per-level k_resize_rows
    launches with their chunk loop, the 4-cell k_detect waves, 256-thread octree workgroups, the compact
    records), pairs checked bit for bit against the oracle and the stereo restatement."""
    import torch
    from oracle import stereo_oracle
    from pyorbslam_amd import dist as D
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd.frame import to_reference_lists
    from conftest import BF, FX
    h, w = 600, 4500
    pairs = [synth.make_pair(430 + i, w, h) for i in range(16)]

    def oracle_pair(L, R):
        oL, oR = O.OracleExtractor(**KITTI), O.OracleExtractor(**KITTI)
        kl, dl = oL.extract(L)
        kr, dr = oR.extract(R)
        t = oL.tables()
        ou, od, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, oL.sheared_pyramid(), oR.sheared_pyramid(),
                                                         t["scale"], t["inv_scale"], BF, np.float32(FX))
        return kl, dl, kr, dr, ou, od, oL.sheared_pyramid(), oR.sheared_pyramid()

    def same_lists(a, b):
        sa, va = stereo_oracle.encode(a)
        sb, vb = stereo_oracle.encode(b)
        return np.array_equal(sa, sb) and np.array_equal(va, vb)

    # per-frame path
    left, right = ORBextractor(**KITTI), ORBextractor(**KITTI)
    L, R = pairs[0]
    gk, gd, hk, hd = left.operator_kd_stereo(L, R, right, BF, np.float32(FX))
    kl, dl, kr, dr, ou, od, pl, pr = oracle_pair(L, R)
    assert gk.tobytes() == kl.tobytes() and np.array_equal(gd, dl)
    assert hk.tobytes() == kr.tobytes() and np.array_equal(hd, dr)
    u, d = to_reference_lists(left.stereo_result, gk, BF)
    assert same_lists(u, ou) and same_lists(d, od)
    assert sum(s == 1 for s in left.stereo_result["status"]) > 100
    for a, b in zip(list(left.GetImagePyramid()) + list(right.GetImagePyramid()), list(pl) + list(pr)):
        assert np.array_equal(a, b)
    # batch path, 16 pairs in one enqueue
    fe = StereoFrontEnd(w, h, max_pairs=16, lanes=1)
    imgs = torch.from_numpy(np.stack([x for p in pairs for x in p])).cuda()
    fe.enqueue(imgs, 16, BF, np.float32(FX), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert fe.overflow() == 0
    for p in (5, 15):
        kl, dl, kr, dr, ou, od, _, _ = oracle_pair(*pairs[p])
        k, dd = fe.fetch_image(2 * p)
        k2, dd2 = fe.fetch_image(2 * p + 1)
        assert k.tobytes() == kl.tobytes() and np.array_equal(dd, dl), f"pair {p} left"
        assert k2.tobytes() == kr.tobytes() and np.array_equal(dd2, dr), f"pair {p} right"
        u, d = to_reference_lists(fe.fetch_stereo(p), k, BF)
        assert same_lists(u, ou) and same_lists(d, od), f"pair {p} stereo"
    # compact records (14-bit level coordinates) rebuild the 4 500 px keypoints exactly
    buf = torch.zeros((16, D.compact_record_bytes(fe.kp_cap)), dtype=torch.uint8, device="cuda")
    D.pack_device([fe], [16], buf, compact=True)
    torch.cuda.synchronize()
    rec = D.unpack_compact(fe.kp_cap, buf[15].cpu().numpy(), fe.scales)
    k, _ = fe.fetch_image(30)
    assert rec["kps_left"].tobytes() == k.tobytes() and (k["x"] > 4095).any()


def test_levels_above_2_pow_24_pixels_refused():
    """The documented limit: a level of more than 2^24 pixels does not fit the packed keys
    and is refused with ORBFE_EINVAL naming the limit (the reference accepts it); a 600 x 4 500 image (tall,
    aspect below 0.5) is refused as the reference's DistributeOctTree indexes out of range on it
    (nIni = round(spanX / spanY) = 0, ORBextractor.cpp:543-568), ValueError like the oracle's refusal."""
    from pyorbslam_amd._lib import OrbfeError
    img = np.zeros((4200, 4200), np.uint8)
    img[::7, ::5] = 200
    with pytest.raises(OrbfeError, match="2\\^24"):
        ORBextractor(**KITTI).extract(img)
    tall = synth.make_pair(5, 600, 4500)[0]
    with pytest.raises(ValueError, match="DistributeOctTree"):
        ORBextractor(**KITTI).extract(tall)
    with pytest.raises(ValueError):
        O.OracleExtractor(**KITTI).extract(tall)
