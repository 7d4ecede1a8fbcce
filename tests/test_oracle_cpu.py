"""CPU tests of the checker itself: the oracle against the reference's golden vectors / known answers and
against independent small-case restatements (pure Python / numpy)."""
import ctypes as C
import hashlib
import json
import math

import numpy as np
import pytest

from conftest import GOLDEN, KITTI, EUROC, BF, FX, STEREO_CASES, golden_case_images
from oracle import oracle as O
from oracle import stereo_oracle
from pyorbslam_amd import synth


# ----------------------------------------------------------------------------------- known answers
def test_tables_known_answers():
    t = O.OracleExtractor(**KITTI).tables()
    # SURVEY.md §8 level table (restated from ORBextractor.cpp:410-446)
    assert t["n_per_level"].tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    assert t["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    exp = [1.0, 1.2000000477, 1.4400000572, 1.7280001640, 2.0736002922, 2.4883203506, 2.9859845638, 3.5831816196]
    assert np.allclose(t["scale"], exp, rtol=0, atol=1e-9)
    assert t["scale"].dtype == np.float32
    e = O.OracleExtractor(**EUROC).tables()
    assert e["n_per_level"].tolist() == [217, 181, 151, 126, 105, 87, 73, 60]


def test_level_sizes_known_answers():
    ex = O.OracleExtractor(**KITTI)
    assert ex.level_sizes(1241, 376) == [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151),
                                         (416, 126), (346, 105)]
    assert [w * h for w, h in ex.level_sizes(1241, 376)] and sum(w * h for w, h in ex.level_sizes(1241, 376)) == 1444097
    assert ex.level_sizes(752, 480)[7] == (210, 134)


def test_pattern_matches_reference_digest():
    g = json.loads((GOLDEN / "brief_pattern.json").read_text())
    txt = (O.HERE.parent / "pyorbslam_amd" / "csrc" / "brief_pattern.inc").read_text().splitlines()
    vals = [int(v) for line in txt if not line.startswith("//") for v in line.replace(",", " ").split()]
    assert len(vals) == 1024
    assert hashlib.sha256(",".join(map(str, vals)).encode()).hexdigest() == g["sha256"]


# ----------------------------------------------------------------------------------- glibc sincosf
def test_glibc_sincosf_replica_matches_host_libm():
    libm = C.CDLL("libm.so.6")
    libm.cosf.argtypes = libm.sinf.argtypes = [C.c_float]
    libm.cosf.restype = libm.sinf.restype = C.c_float
    L = O.lib()
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 2 * math.pi, 20000), rng.uniform(0, 0.01, 5000),
                         np.arange(0, 360, 0.25) * np.float32(math.pi / 180.0)]).astype(np.float32)
    bad = 0
    for x in xs.tolist():
        bad += L.oracle_cosf(x) != libm.cosf(x)
        bad += L.oracle_sinf(x) != libm.sinf(x)
    # The replica is of the x86-64 FMA ifunc variant; on a host without FMA/AVX2 glibc picks another one.
    flags = open("/proc/cpuinfo").read()
    if " fma " in flags and " avx2 " in flags:
        assert bad == 0


def test_fast_atan2_properties():
    L = O.lib()
    assert L.oracle_fast_atan2(0.0, 0.0) == 0.0
    for y, x, ref in [(1, 1, 45), (1, 0, 90), (0, -1, 180), (-1, 0, 270), (-1, 1, 315)]:
        assert abs(L.oracle_fast_atan2(float(y), float(x)) - ref) < 0.02
    rng = np.random.default_rng(0)
    for y, x in rng.integers(-3_000_000, 3_000_000, (2000, 2)).tolist():
        a = L.oracle_fast_atan2(float(y), float(x))
        assert 0.0 <= a < 360.0 or a == 360.0
        assert abs(((a - math.degrees(math.atan2(y, x))) + 180) % 360 - 180) < 0.01


# ----------------------------------------------------------------------------------- FAST
def _fast_brute(img, th):
    """cv::FAST(img, kps, th, nonmax=true) TYPE_9_16 by definition (pure Python, small images)."""
    circ = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
            (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    h, w = img.shape
    I = img.astype(int)
    score = np.zeros((h, w), int)
    corner = np.zeros((h, w), bool)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = I[y, x]
            d = [v - I[y + dy, x + dx] for dx, dy in circ]
            M = max(max(min(d[(k + j) % 16] for j in range(9)), min(-d[(k + j) % 16] for j in range(9)))
                    for k in range(16))
            if M > th:
                corner[y, x] = True
                score[y, x] = M - 1
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            if corner[y, x] and all(score[y, x] > score[y + a, x + b] for a in (-1, 0, 1) for b in (-1, 0, 1)
                                    if (a or b)):
                out.append((x, y, score[y, x]))
    return out


@pytest.mark.parametrize("seed", range(6))
def test_fast_oracle_vs_definition(seed):
    rng = np.random.default_rng(seed)
    h, w = rng.integers(8, 40), rng.integers(8, 40)
    img = rng.integers(0, 256, (h, w)).astype(np.uint8)
    if seed % 2:
        img = (np.clip(rng.normal(128, 40, (h, w)), 0, 255)).astype(np.uint8)
    th = int(rng.integers(0, 40))
    got = [tuple(r) for r in O.fast(img, th).tolist()]
    assert got == _fast_brute(img, th)


# ----------------------------------------------------------------------------------- resize / blur
def _resize_py(src, dw, dh, simd):
    """cv::resize INTER_LINEAR 8U restated with numpy (coefficients in float32 / float64 like OpenCV)."""
    sh, sw = src.shape
    sx_scale, sy_scale = 1.0 / (dw / sw), 1.0 / (dh / sh)

    def coefs(n_dst, n_src, scale, clamp):
        idx, a0, a1 = [], [], []
        for d in range(n_dst):
            f = np.float32((d + 0.5) * scale - 0.5)
            s = math.floor(f)
            f = np.float32(f - np.float32(s))
            if clamp:
                if s < 0:
                    f, s = np.float32(0), 0
                if s >= n_src - 1:
                    f, s = np.float32(0), n_src - 1
            idx.append(s)
            a0.append(int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048))))
            a1.append(int(np.rint(f * np.float32(2048))))
        return np.array(idx), np.array(a0), np.array(a1)

    xs, ax0, ax1 = coefs(dw, sw, sx_scale, True)
    ys, by0, by1 = coefs(dh, sh, sy_scale, False)
    S = src.astype(np.int64)
    xs1 = np.minimum(xs + 1, sw - 1)
    Hrow = S[:, xs] * ax0 + S[:, xs1] * ax1
    xv = 0
    if simd:
        while xv <= dw - simd:
            xv += simd
        while xv < dw - simd // 2:
            xv += simd // 2
    out = np.zeros((dh, dw), np.uint8)
    for dy in range(dh):
        r0, r1 = min(max(ys[dy], 0), sh - 1), min(max(ys[dy] + 1, 0), sh - 1)
        h0, h1 = Hrow[r0], Hrow[r1]
        sc = (h0 * by0[dy] + h1 * by1[dy] + (1 << 21)) >> 22
        vec = ((((np.minimum(h0 >> 4, 32767) * by0[dy]) >> 16) + ((np.minimum(h1 >> 4, 32767) * by1[dy]) >> 16) + 2)
               >> 2)
        row = np.where(np.arange(dw) < xv, vec, sc)
        out[dy] = np.clip(row, 0, 255)
    return out


@pytest.mark.parametrize("simd", [0, 16, 32])
def test_resize_oracle_vs_numpy(simd):
    rng = np.random.default_rng(simd)
    src = rng.integers(0, 256, (97, 173)).astype(np.uint8)
    for dw, dh in [(144, 81), (120, 67), (173, 97), (50, 30)]:
        assert np.array_equal(O.resize(src, dw, dh, simd), _resize_py(src, dw, dh, simd)), (dw, dh)


def test_blur_oracle_vs_numpy():
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (41, 57)).astype(np.uint8)
    k = np.array([18, 34, 48, 56, 48, 34, 18], np.int64)
    p = np.pad(src.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    hpass = sum(k[i] * p[:, i:i + src.shape[1]] for i in range(7))
    v = sum(k[j] * hpass[j:j + src.shape[0], :] for j in range(7))
    assert np.array_equal(O.blur7(src), ((v + 32768) >> 16).astype(np.uint8))


def test_gaussian_q8_kernel_from_definition():
    """OpenCV's bit-exact 7-tap sigma-2 kernel: normalized Gaussian x 256 with error diffusion."""
    g = np.exp(-(np.arange(7) - 3.0) ** 2 / (2 * 2.0 ** 2))
    g /= g.sum()
    res, err = [0] * 7, 0.0
    for i in range(3):
        a = g[i] * 256 + err
        r = int(np.rint(a))
        err = a - r
        res[i] = res[6 - i] = r
    res[3] = 256 - 2 * sum(res[:3])
    assert res == [18, 34, 48, 56, 48, 34, 18]


# ----------------------------------------------------------------------------------- octree
class _Node:
    __slots__ = ("keys", "x0", "y0", "x1", "y1", "nomore", "cid")


def _octree_py(K, minX, maxX, minY, maxY, N, reverse_ties=False):
    """DistributeOctTree (ORBextractor.cpp:539-762) on a Python list; ties by creation id (the careful phase
    divides the most recently created of equal-size nodes first), or with reverse_ties the oldest first — a
    second admissible heap-address order."""
    if not K:
        return []
    nIni = int(math.floor(np.float32(maxX - minX) / np.float32(maxY - minY) + np.float32(0.5)))
    hX = np.float32(np.float32(maxX - minX) / np.float32(nIni))
    ctr = [0]

    def mk(keys, x0, y0, x1, y1):
        n = _Node()
        n.keys, n.x0, n.y0, n.x1, n.y1, n.nomore = keys, x0, y0, x1, y1, len(keys) == 1
        n.cid = ctr[0]
        ctr[0] += 1
        return n

    ini = [mk([], int(np.float32(hX * np.float32(i))), 0, int(np.float32(hX * np.float32(i + 1))), maxY - minY)
           for i in range(nIni)]
    for i, k in enumerate(K):
        ini[int(np.float32(np.float32(k[0]) / hX))].keys.append(i)
    nodes = []
    for n in ini:
        if n.keys:
            n.nomore = len(n.keys) == 1
            nodes.append(n)

    def divide(n):
        hx, hy = (n.x1 - n.x0 + 1) // 2, (n.y1 - n.y0 + 1) // 2
        mx, my = n.x0 + hx, n.y0 + hy
        parts = [[], [], [], []]
        for i in n.keys:
            parts[(0 if K[i][0] < mx else 1) + (0 if K[i][1] < my else 2)].append(i)
        boxes = [(n.x0, n.y0, mx, my), (mx, n.y0, n.x1, my), (n.x0, my, mx, n.y1), (mx, my, n.x1, n.y1)]
        return [(parts[q], boxes[q]) for q in range(4)]

    while True:
        prev = len(nodes)
        front, keep, expand = [], [], []
        for n in nodes:
            if n.nomore:
                keep.append(n)
                continue
            for keys, b in divide(n):
                if keys:
                    c = mk(keys, *b)
                    front.insert(0, c)
                    if len(keys) > 1:
                        expand.append(c)
        nodes = front + keep
        if len(nodes) >= N or len(nodes) == prev:
            break
        if len(nodes) + 3 * len(expand) > N:
            while True:
                prev = len(nodes)
                todo = sorted(expand, key=lambda n: (len(n.keys), -n.cid if reverse_ties else n.cid))
                expand = []
                done = False
                for n in reversed(todo):
                    kids = []
                    for keys, b in divide(n):
                        if keys:
                            c = mk(keys, *b)
                            kids.insert(0, c)
                            if len(keys) > 1:
                                expand.append(c)
                    nodes.remove(n)
                    nodes = kids + nodes
                    if len(nodes) >= N:
                        done = True
                        break
                if done or len(nodes) >= N or len(nodes) == prev:
                    break
            break
    out = []
    for n in nodes:
        best = n.keys[0]
        for i in n.keys[1:]:
            if K[i][2] > K[best][2]:
                best = i
        out.append(K[best])
    return out


@pytest.mark.parametrize("seed", range(8))
def test_octree_oracle_vs_python(seed):
    rng = np.random.default_rng(seed)
    W, H = int(rng.integers(80, 400)), int(rng.integers(60, 200))
    n = int(rng.integers(1, 900))
    xs = rng.integers(3, W - 4, n)
    ys = rng.integers(3, H - 4, n)
    pts = sorted(set(zip(ys.tolist(), xs.tolist())))
    K = [(x, y, int(rng.integers(7, 60))) for y, x in pts]
    N = int(rng.integers(5, 200))
    got = O.octree(np.array(K, np.int32), 16, 16 + W, 16, 16 + H, N)
    exp = _octree_py(K, 16, 16 + W, 16, 16 + H, N)
    assert [tuple(r) for r in got.tolist()] == [tuple(r) for r in exp]
    assert len(got) <= max(N + 2, 4 * max(1, round(W / H)))


# ----------------------------------------------------------------------------------- stereo vs reference goldens
@pytest.mark.parametrize("name", STEREO_CASES)
def test_stereo_oracle_matches_reference_golden(name, kitti_png):
    L, R, params, g = golden_case_images(name, kitti_png)
    assert hashlib.sha256(L.tobytes()).hexdigest() == str(g["left_sha"])
    assert hashlib.sha256(R.tobytes()).hexdigest() == str(g["right_sha"])
    exL, exR = O.OracleExtractor(**params), O.OracleExtractor(**params)
    kl, dl = exL.extract(L)
    kr, dr = exR.extract(R)
    # the extraction fed to the reference when the golden was made
    assert hashlib.sha256(kl.tobytes()).hexdigest() == str(g["kps_left_sha"])
    assert hashlib.sha256(dl.tobytes()).hexdigest() == str(g["desc_left_sha"])
    assert hashlib.sha256(kr.tobytes()).hexdigest() == str(g["kps_right_sha"])
    assert hashlib.sha256(dr.tobytes()).hexdigest() == str(g["desc_right_sha"])
    t = exL.tables()
    u, d, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, exL.sheared_pyramid(), exR.sheared_pyramid(),
                                                   t["scale"], t["inv_scale"], BF, np.float32(FX))
    su, vu = stereo_oracle.encode(u)
    sd, vd = stereo_oracle.encode(d)
    assert np.array_equal(su, g["status"]) and np.array_equal(sd, g["status"])
    assert np.array_equal(vu, g["u_right"]) and np.array_equal(vd, g["depth"])  # bit-exact


def test_sheared_view_definition():
    lvl = np.arange(30 * 40, dtype=np.int64).reshape(30, 40).astype(np.uint8)
    s = O.sheared(lvl)
    pad = np.pad(lvl, 19, mode="reflect")
    flat = pad.ravel()
    assert np.array_equal(s.ravel(), flat[19 * 78 + 19: 19 * 78 + 19 + 1200])
    assert np.array_equal(s[0], lvl[0])  # row 0 is unsheared


@pytest.mark.parametrize("name", ["kitti_synth_s0", "identical_s3"])
def test_stereo_loop_restatement_matches_reference_golden(name, kitti_png):
    """oracle/stereo_loop.py (the per-candidate-loop restatement bench.py times as the reference's CPU
    path) gives the reference's outputs, types included."""
    from oracle.stereo_loop import compute_stereo_matches_loop
    L, R, params, g = golden_case_images(name, kitti_png)
    exL, exR = O.OracleExtractor(**params), O.OracleExtractor(**params)
    kl, dl = exL.extract(L)
    kr, dr = exR.extract(R)
    t = exL.tables()
    u, d = compute_stereo_matches_loop(kl, kr, dl, dr, exL.sheared_pyramid(), exR.sheared_pyramid(), t["scale"],
                                       t["inv_scale"], BF, np.float32(FX))
    su, vu = stereo_oracle.encode(u)
    sd, vd = stereo_oracle.encode(d)
    assert np.array_equal(su, g["status"]) and np.array_equal(sd, g["status"])
    assert np.array_equal(vu, g["u_right"]) and np.array_equal(vd, g["depth"])


# oracle_octree_ties of synthetic pair 0's left image (synth.make_pair(0)), per level: straddle, tie runs,
# careful iterations, straddled run's nodes, of which divided (profiles/octree_ties.json has the workloads)
TIES_PAIR0_LEFT = [[1, 10, 1, 13, 3], [1, 5, 1, 14, 13], [1, 4, 1, 8, 2], [1, 22, 2, 7, 4], [1, 14, 2, 8, 2],
                   [1, 15, 2, 7, 4], [0, 10, 2, 0, 0], [1, 6, 3, 6, 1]]
TIES_KITTI06 = [[1, 24, 1, 7, 2], [0, 19, 1, 0, 0], [0, 10, 1, 0, 0], [1, 7, 1, 5, 4], [0, 5, 1, 0, 0], [1, 13, 2, 6, 2],
                [1, 14, 2, 5, 3], [1, 9, 2, 2, 1]]


def test_octree_tie_report(kitti_png):
    """SURVEY H1 / VERDICT r4 item 3: the tie report of the oracle, pinned, and shown to mean what it says by a
    second admissible address order (the oldest of equal-size nodes divided first): on a level without a
    straddle both orders keep the same keypoints (at most their order differs, and only where equal-size runs
    were divided); on a straddled level the kept set may differ — it does on most of them."""
    ex = O.OracleExtractor()
    assert ex.octree_ties(kitti_png).tolist() == TIES_KITTI06
    L = synth.make_pair(0)[0]
    ties = ex.octree_ties(L)
    assert ties.tolist() == TIES_PAIR0_LEFT
    ex.extract(L)
    n_per = ex.tables()["n_per_level"]
    set_differs = []
    for l, lvl in enumerate(ex.pyramid()):
        h, w = lvl.shape
        K = [tuple(r) for r in O.level_candidates(ex.p, lvl).tolist()]
        a = _octree_py(K, 16, w - 16, 16, h - 16, int(n_per[l]))
        b = _octree_py(K, 16, w - 16, 16, h - 16, int(n_per[l]), reverse_ties=True)
        assert [tuple(r) for r in O.octree(np.array(K, np.int32), 16, w - 16, 16, h - 16, int(n_per[l])).tolist()] == a
        if ties[l, 0] == 0:
            assert sorted(a) == sorted(b), f"level {l}: no straddle reported, yet the kept keypoints differ"
        else:
            set_differs.append(sorted(a) != sorted(b))
        if ties[l, 1] == 0:
            assert a == b, f"level {l}: no tie run reported, yet the keypoint order differs"
    assert sum(set_differs) > len(set_differs) // 2, set_differs


def _area2_py(src, simd):
    """cv::resize's INTER_AREA fast path for an exact 2x step, from its definition (OpenCV 4.x resize.cpp:
    resizeAreaFast_Invoker + ResizeAreaFastVec_SIMD_8u): (sum + 2) >> 2 over the vector span, sum * 0.25f rounded
    half to even after it."""
    h, w = src.shape[0] // 2, src.shape[1] // 2
    s = src.astype(np.int32)
    tot = s[0::2, 0::2][:h, :w] + s[0::2, 1::2][:h, :w] + s[1::2, 0::2][:h, :w] + s[1::2, 1::2][:h, :w]
    lanes = simd // 2
    xv = w // lanes * lanes if lanes else 0
    out = np.rint(tot.astype(np.float32) * np.float32(0.25)).astype(np.int32)  # np.rint: half to even
    out[:, :xv] = (tot[:, :xv] + 2) >> 2
    return out.astype(np.uint8)


@pytest.mark.parametrize("simd", [0, 16, 32])
def test_resize_area_fast_path(simd):
    """an exact 2x step takes OpenCV's INTER_AREA fast path; the two roundings differ (sum % 4
    == 2 with an even quotient), so widths that are not a multiple of the vector step exercise both."""
    rng = np.random.default_rng(simd)
    for h, w in ((94, 310), (50, 38), (12, 12), (2, 18)):
        src = rng.integers(0, 256, (2 * h, 2 * w)).astype(np.uint8)
        got = O.resize(src, w, h, simd)
        assert np.array_equal(got, _area2_py(src, simd)), (h, w)
    # an odd source width is not an exact 2x step: the linear path (1241 -> 620)
    src = rng.integers(0, 256, (376, 1241)).astype(np.uint8)
    assert np.array_equal(O.resize(src, 620, 188, simd), _resize_py(src, 620, 188, simd))


def test_reference_refused_geometries():
    """levels of 19 px or less are taken (square images: nIni = 1 on every level); a level
    lower than 32 px but wider makes the reference's DistributeOctTree throw (vpIniNodes.resize(nIni < 0)) and
    the oracle refuses it as ValueError, as pybind11 raises the reference's std::length_error."""
    img = synth.make_pair(3, 128, 128)[0]
    ex = O.OracleExtractor(nfeatures=300, scaleFactor=1.2, nlevels=12)
    kps, desc = ex.extract(img)
    assert len(kps) > 0 and min(p.shape[0] for p in ex.pyramid()) <= 19
    sq = O.OracleExtractor(nfeatures=1000, scaleFactor=2.0, nlevels=6)
    sq.extract(synth.make_pair(4, 400, 400)[0])
    assert [p.shape for p in sq.pyramid()] == [(400, 400), (200, 200), (100, 100), (50, 50), (25, 25), (12, 12)]
    for (h, w), prm in (((96, 160), dict(nlevels=12)), ((376, 1241), dict(scaleFactor=2.0, nlevels=8))):
        with pytest.raises(ValueError):
            O.OracleExtractor(**prm).extract(synth.make_pair(5, w, h)[0])
    assert len(O.OracleExtractor(scaleFactor=2.0, nlevels=4).extract(synth.make_pair(5)[0])[0]) > 0
