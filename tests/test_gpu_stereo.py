"""GPU stereo matching against the REFERENCE's own outputs (tests/golden/stereo_*.npz were produced by
calling the reference Frame.compute_stereo_matches, Frame.py:161-279).  Tolerance: none — the reference's
float32 chain is reproduced bit for bit (uR, depth as np.float32; zero-disparity entries in double)."""
import hashlib

import numpy as np
import pytest

from conftest import BF, FX, KITTI, STEREO_CASES, golden_case_images
from oracle import stereo_oracle
from pyorbslam_amd import frame as F
from pyorbslam_amd import synth
from pyorbslam_amd.pyORBExtractor import ORBextractor

pytestmark = pytest.mark.gpu


def _encode_gpu(res, kl):
    u, d = F.to_reference_lists(res, kl, BF)
    su, vu = stereo_oracle.encode(u)
    sd, vd = stereo_oracle.encode(d)
    return su, vu, sd, vd


@pytest.mark.parametrize("name", STEREO_CASES)
def test_stereo_matches_reference_golden(name, kitti_png):
    L, R, params, g = golden_case_images(name, kitti_png)
    exL, exR = ORBextractor(**params), ORBextractor(**params)
    kl, dl = exL.extract(L)
    kr, dr = exR.extract(R)
    # inputs identical to those the reference was fed (extractor parity)
    assert hashlib.sha256(kl.tobytes()).hexdigest() == str(g["kps_left_sha"])
    assert hashlib.sha256(dl.tobytes()).hexdigest() == str(g["desc_left_sha"])
    assert hashlib.sha256(kr.tobytes()).hexdigest() == str(g["kps_right_sha"])
    assert hashlib.sha256(dr.tobytes()).hexdigest() == str(g["desc_right_sha"])
    res = F.stereo_match_arrays(exL, exR, BF, np.float32(FX))
    su, vu, sd, vd = _encode_gpu(res, kl)
    st = g["status"]
    bad = np.nonzero(su != st)[0]
    assert bad.size == 0, f"{bad.size} status mismatches, first {bad[:5]}: gpu {su[bad[:5]]} ref {st[bad[:5]]}"
    assert np.array_equal(vu, g["u_right"]) and np.array_equal(vd, g["depth"])


class _FrameLike:
    pass


def test_frame_drop_in_types():
    L, R = synth.make_pair(3)
    f = _FrameLike()
    f.mpORBextractorLeft, f.mpORBextractorRight = ORBextractor(**KITTI), ORBextractor(**KITTI)
    f.mvKeys_, f.mDescriptors = f.mpORBextractorLeft.operator_kd(L)
    f.mpORBextractorRight.operator_kd(R)
    f.N = len(f.mvKeys_)
    f.mbf = BF
    f.mK = np.eye(3, dtype=np.float32)
    f.mK[0, 0] = FX
    F.compute_stereo_matches(f)
    assert len(f.mvuRight) == f.N == len(f.mvDepth)
    kinds = {type(v) for v in f.mvuRight}
    assert kinds <= {int, np.float32, float}
    assert all(v == -1 for v in f.mvuRight if isinstance(v, int))
    assert any(isinstance(v, np.float32) for v in f.mvuRight)


def test_batch_path_equals_single_path():
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    imgs = synth.make_batch(3, seed0=0)
    fe = StereoFrontEnd(max_pairs=4)
    d = torch.from_numpy(imgs).cuda()
    fe.enqueue(d, 3)
    torch.cuda.synchronize()
    for p in range(3):
        exL, exR = ORBextractor(**KITTI), ORBextractor(**KITTI)
        kl, dl = exL.extract(imgs[2 * p])
        kr, dr = exR.extract(imgs[2 * p + 1])
        bk, bd = fe.fetch_image(2 * p)
        assert bk.tobytes() == kl.tobytes() and np.array_equal(bd, dl)
        bk, bd = fe.fetch_image(2 * p + 1)
        assert bk.tobytes() == kr.tobytes() and np.array_equal(bd, dr)
        single = F.stereo_match_arrays(exL, exR, BF, np.float32(FX))
        batch = fe.fetch_stereo(p)
        for k in ("status", "u_right", "depth", "match_r"):
            assert np.array_equal(single[k], batch[k]), k


def test_batch_repeat_is_deterministic():
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    imgs = torch.from_numpy(synth.make_batch(4, seed0=20)).cuda()
    fe = StereoFrontEnd(max_pairs=4)
    fe.enqueue(imgs)
    torch.cuda.synchronize()
    first = [fe.fetch_stereo(p) for p in range(4)]
    k0 = fe.fetch_image(5)
    fe.enqueue(imgs)
    torch.cuda.synchronize()
    for p in range(4):
        r = fe.fetch_stereo(p)
        assert all(np.array_equal(first[p][k], r[k]) for k in r)
    assert fe.fetch_image(5)[0].tobytes() == k0[0].tobytes()


@pytest.mark.parametrize("lanes", [1, 2, 3, 4])
def test_lanes_do_not_change_results(lanes):
    """orbfe_set_lanes splits the batch into concurrent chunks on internal streams (5 pairs: uneven
    chunks); every image and pair must come out exactly as with one lane."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    imgs = torch.from_numpy(synth.make_batch(5, seed0=40)).cuda()
    ref = StereoFrontEnd(max_pairs=5, lanes=1)
    fe = StereoFrontEnd(max_pairs=5, lanes=lanes)
    ref.enqueue(imgs)
    fe.enqueue(imgs)
    torch.cuda.synchronize()
    for i in range(10):
        a, b = ref.fetch_image(i), fe.fetch_image(i)
        assert a[0].tobytes() == b[0].tobytes() and np.array_equal(a[1], b[1])
    for p in range(5):
        a, b = ref.fetch_stereo(p), fe.fetch_stereo(p)
        assert all(np.array_equal(a[k], b[k]) for k in a)


# other extractor configurations and baselines: GPU stereo against the numpy restatement (itself pinned to
# the reference goldens above, tests/test_oracle_cpu.py), bit for bit
STEREO_CONFIGS = [
    ((376, 1241), dict(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7), 386.1448, 718.856),
    ((376, 1241), dict(nfeatures=2000, scaleFactor=1.1, nlevels=12, iniThFAST=20, minThFAST=7), 386.1448, 718.856),
    ((376, 1241), dict(nfeatures=1500, scaleFactor=1.5, nlevels=5, iniThFAST=15, minThFAST=5), 386.1448, 718.856),
    ((480, 752), dict(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7), 47.90639384423901,
     435.2046959714599),
    ((720, 1280), dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7), 250.0, 700.0),
]


@pytest.mark.parametrize("ci", range(len(STEREO_CONFIGS)))
def test_stereo_configurations_match_restatement(ci):
    from oracle.oracle import OracleExtractor
    (h, w), params, bf, fx = STEREO_CONFIGS[ci]
    L, R = synth.make_pair(300 + ci, w, h)
    exL, exR = ORBextractor(**params), ORBextractor(**params)
    kl, dl = exL.extract(L)
    kr, dr = exR.extract(R)
    res = F.stereo_match_arrays(exL, exR, bf, np.float32(fx))
    u, d = F.to_reference_lists(res, kl, bf)
    oL, oR = OracleExtractor(**params), OracleExtractor(**params)
    okl, odl = oL.extract(L)
    okr, odr = oR.extract(R)
    assert kl.tobytes() == okl.tobytes() and kr.tobytes() == okr.tobytes()
    t = oL.tables()
    ou, od, _ = stereo_oracle.compute_stereo_matches(okl, okr, odl, odr, oL.sheared_pyramid(), oR.sheared_pyramid(),
                                                     t["scale"], t["inv_scale"], bf, np.float32(fx))
    for a, b in ((u, ou), (d, od)):
        sa, va = stereo_oracle.encode(a)
        sb, vb = stereo_oracle.encode(b)
        assert np.array_equal(sa, sb) and np.array_equal(va, vb)
    assert int((res["status"] > 0).sum()) > 0


@pytest.mark.parametrize("wh", [(641, 333), (211, 157)])
def test_batch_path_misaligned_images(wh):
    """Odd W*H: every second image of a (2P, H, W) batch starts at an address that is not 4-byte aligned
    (and so does the whole batch when it is a slice starting at an odd image).  The buffer loads of
    k_resize / k_detect / k_orb / k_stereo must re-align from the dword at or below the image base; results equal
    the single-image path, whose staging buffer is aligned."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    w, h = wh
    prm = dict(nfeatures=600, scaleFactor=1.2, nlevels=4 if w < 300 else 8, iniThFAST=20, minThFAST=7)
    pairs = [synth.make_pair(60 + i, w, h) for i in range(3)]
    host = np.stack([im for p in pairs for im in p] + [pairs[0][0]])  # 7 images: a spare one in front
    host = np.concatenate([host[-1:], host[:-1]])
    d = torch.from_numpy(np.ascontiguousarray(host)).cuda()
    fe = StereoFrontEnd(w, h, max_pairs=3, **prm)
    fe.enqueue(d[1:], 3)  # base = spare image + W*H bytes: odd offset
    torch.cuda.synchronize()
    for p, (L, R) in enumerate(pairs):
        exL, exR = ORBextractor(**prm), ORBextractor(**prm)
        kl, dl = exL.extract(L)
        kr, dr = exR.extract(R)
        bk, bd = fe.fetch_image(2 * p)
        assert bk.tobytes() == kl.tobytes() and np.array_equal(bd, dl), f"pair {p} left"
        bk, bd = fe.fetch_image(2 * p + 1)
        assert bk.tobytes() == kr.tobytes() and np.array_equal(bd, dr), f"pair {p} right"
        single = F.stereo_match_arrays(exL, exR, BF, np.float32(FX))
        batch = fe.fetch_stereo(p)
        for k in ("status", "u_right", "depth", "match_r"):
            assert np.array_equal(single[k], batch[k]), (p, k)


def test_pair_path_equals_single_path_and_oracle_pyramids():
    """operator_kd_stereo (one enqueue per frame, orbfe_frame_extract) against two operator_kd calls plus
    orbfe_stereo_match, and its device-built sheared pyramids against the oracle's (GetImagePyramid,
    orb_extractor.cpp:30)."""
    from oracle.oracle import OracleExtractor
    for seed, (w, h), prm in ((5, (1241, 376), KITTI), (6, (641, 333), dict(KITTI, nfeatures=700))):
        L, R = synth.make_pair(seed, w, h)
        a, b = ORBextractor(**prm), ORBextractor(**prm)
        kl, dl, kr, dr = a.operator_kd_stereo(L, R, b, BF, np.float32(FX))
        sL, sR = ORBextractor(**prm), ORBextractor(**prm)
        skl, sdl = sL.extract(L)
        skr, sdr = sR.extract(R)
        assert kl.tobytes() == skl.tobytes() and np.array_equal(dl, sdl)
        assert kr.tobytes() == skr.tobytes() and np.array_equal(dr, sdr)
        assert b.last_keypoints.tobytes() == skr.tobytes()
        single = F.stereo_match_arrays(sL, sR, BF, np.float32(FX))
        for k in ("status", "u_right", "depth", "match_r"):
            assert np.array_equal(single[k], a.stereo_result[k]), k
        for ex, img in ((a, L), (b, R)):
            o = OracleExtractor(**prm)
            o.extract(img)
            got, want = ex.GetImagePyramid(), o.sheared_pyramid()
            assert len(got) == len(want)
            for g_, w_ in zip(got, want):
                assert g_.shape == w_.shape and np.array_equal(g_, w_)
        # the right extractor's results wait for ExtractORB(1, R) exactly once
        assert b.take_pending(R) is not None and b.take_pending(R) is None


def test_pair_path_empty_image():
    a, b = ORBextractor(**KITTI), ORBextractor(**KITTI)
    e = np.zeros((0, 0), np.uint8)
    kl, dl, kr, dr = a.operator_kd_stereo(e, e, b, BF, np.float32(FX))
    assert len(kl) == 0 and dl.shape == (0, 0) and len(kr) == 0 and dr.shape == (0, 0)
    assert len(a.stereo_result["status"]) == 0


@pytest.mark.parametrize("compact", [False, True])
def test_device_pack_records_match_fetch(compact):
    """k_pack / k_pack_compact (orbfe_batch_pack_device / _compact_device) build the gather and host-fed
    records of dist.py on the device: every field of every pair decodes (unpack / unpack_compact, which
    rebuilds x, y, size and response from level coordinates, octave and score) to exactly what
    orbfe_batch_fetch / _fetch_stereo return, for the KITTI and the EuRoC geometries."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd import dist as D
    from pyorbslam_amd.batch import StereoFrontEnd
    for w, h, nf in ((1241, 376, 2000), (752, 480, 1000)):
        imgs = torch.from_numpy(synth.make_batch(3, seed0=70, width=w, height=h)).cuda()
        fes = [StereoFrontEnd(w, h, max_pairs=3, nfeatures=nf, lanes=1), StereoFrontEnd(w, h, max_pairs=3, nfeatures=nf,
                                                                                    lanes=2)]
        for f in fes:
            f.enqueue(imgs, 3)
        torch.cuda.synchronize()
        rb = (D.compact_record_bytes if compact else D.record_bytes)(fes[0].kp_cap)
        buf = torch.zeros((6, rb), dtype=torch.uint8, device="cuda")
        D.pack_device(fes, [3, 3], buf, compact)
        torch.cuda.synchronize()
        host = buf.cpu().numpy()
        _check_records(fes, host, compact, D)


def _check_records(fes, host, compact, D):
    for i, f in enumerate(fes):
        for p in range(3):
            u = D.unpack_compact(f.kp_cap, host[3 * i + p], f.scales) if compact else D.unpack(f.kp_cap, host[3 * i + p])
            kl, dl = f.fetch_image(2 * p)
            kr, dr = f.fetch_image(2 * p + 1)
            s = f.fetch_stereo(p)
            assert u["kps_left"].tobytes() == kl.tobytes() and u["kps_right"].tobytes() == kr.tobytes()
            assert np.array_equal(u["desc_left"], dl) and np.array_equal(u["desc_right"], dr)
            for k in ("u_right", "depth", "status"):
                assert np.array_equal(u[k], s[k]), k


def test_undistort_points_matches_opencv_restatement():
    """k_undistort against oracle/undistort_oracle.py (cv::undistortPoints restated; parity with OpenCV
    itself is unpinned: OpenCV is absent and the reference's distorted branch is unreachable)."""
    from oracle.undistort_oracle import undistort_points as ref
    rng = np.random.default_rng(5)
    xy = np.stack([rng.uniform(0, 752, 3000), rng.uniform(0, 480, 3000)], 1).astype(np.float32)
    xy[:4] = [[0, 0], [752, 0], [0, 480], [752, 480]]  # Tracking.compute_image_bounds' corners
    K = np.eye(3, dtype=np.float32)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = 458.654, 457.296, 367.215, 248.375  # EuRoC cam0
    for dist in ([-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05],        # EuRoC cam0 (4 coefficients)
                 [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.01],  # + k3
                 [-2.0, -5.0, 0.0, 0.0],                                      # icdist < 0 at the corners
                 [0.0, 0.0, 0.0, 0.0]):
        got = F.undistort_points(xy, K, np.array(dist, np.float32).reshape(-1, 1))
        want = ref(xy, K, dist)
        assert got.dtype == np.float32 and np.array_equal(got, want), dist


def test_undistort_keypoints_drop_in():
    from oracle.undistort_oracle import undistort_points as ref
    import seq_harness as H

    class Fr(H.SeqFrame):
        pass

    F.install(Fr)
    s = H.settings(synth.KITTI_CAM)
    dist = np.array([[-0.28], [0.07], [0.0002], [0.00002]], np.float32)
    L, R = synth.make_pair(9)
    f = Fr(L, R, 0.0, ORBextractor(**KITTI), ORBextractor(**KITTI), None, s["mK"], dist, s["mbf"], s["mThDepth"],
           H.frame_args(s, 1241, 376))
    pts = np.array([k.pt for k in f.mvKeys], np.float32)
    want = ref(pts, s["mK"], dist.ravel())
    assert len(f.mvKeysUn) == f.N
    assert all(u.pt == (float(w[0]), float(w[1])) and u.octave == k.octave and u.angle == k.angle
               for u, k, w in zip(f.mvKeysUn, f.mvKeys, want))


def test_default_bench_configuration_sampled():
    """The exact default bench step (bench.Shard: 512 KITTI pairs as 4 handles x 128 pairs on 4 streams, lanes
    1) and the bench's own parity check: every handle's overflow word, 16 pairs of every handle (first, last and
    evenly spaced between) bit for bit against the oracle extractor and the stereo restatement."""
    torch = pytest.importorskip("torch")
    import bench
    P, S = 512, 4
    host = synth.make_batch(P, seed0=0)
    images = torch.from_numpy(host).cuda()
    sh = bench.Shard(images, P, S, torch.device("cuda", 0), 1241, 376, 2000)
    assert sh.counts == [128] * 4
    for _ in range(2):  # the bench repeats the step on the same buffers
        sh.step()
    torch.cuda.synchronize()
    checked, ovf, bad = bench.parity_check(sh.fes, sh.counts, host, 1241, 376, 2000)
    assert ovf == 0 and not bad and checked == 64, bad


def test_c4_shards_and_host_fed():
    """C4's shards (64 pairs over 1, 2, 4 or 8 ranks: 64, 32, 16, 8 pairs, up to 4 handles each), uneven
    handle splits, and the host-fed pass (pinned H2D + compute + packed records D2H, double-buffered) whose
    records must equal the handles' own results; parity of the uneven shard against the oracle."""
    torch = pytest.importorskip("torch")
    import bench
    dev = torch.device("cuda", 0)
    for world in (1, 2, 4, 8):
        assert sum(bench.shard(64, world, r)[1] for r in range(world)) == 64
    host = synth.make_batch(7, seed0=300)
    images = torch.from_numpy(host).to(dev)
    sh = bench.Shard(images, 7, 4, dev, 1241, 376, 2000)
    assert sh.counts == [3, 2, 2]  # one handle per 3 pairs, rounded up (bench.Shard)
    sh.step()
    torch.cuda.synchronize()
    checked, ovf, bad = bench.parity_check(sh.fes, sh.counts, host, 1241, 376, 2000)
    assert ovf == 0 and not bad and checked == 7, bad
    hf = bench.host_fed(sh, host, dev, 1, 3, 1)
    assert hf["record_check"] and hf["value"] > 0


def test_pack_orders_after_batch_on_another_stream():
    """orbfe_batch_pack_device on a stream other than the batch's waits for that batch: pack right
    after enqueue, without a host synchronisation in between."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd import dist as D
    from pyorbslam_amd.batch import StereoFrontEnd
    imgs = torch.from_numpy(synth.make_batch(4, seed0=90)).cuda()
    f = StereoFrontEnd(max_pairs=4, lanes=1)
    side, other = torch.cuda.Stream(), torch.cuda.Stream()
    rb = D.record_bytes(f.kp_cap)
    buf = torch.zeros((4, rb), dtype=torch.uint8, device="cuda")
    f.enqueue(imgs, 4, stream_ptr=side.cuda_stream)
    with torch.cuda.stream(other):
        D.pack_device([f], [4], buf)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    for p in range(4):
        u = D.unpack(f.kp_cap, host[p])
        kl, dl = f.fetch_image(2 * p)
        assert u["kps_left"].tobytes() == kl.tobytes() and np.array_equal(u["desc_left"], dl), p


def test_frame_results_invalidated_by_other_work():
    """after orbfe_frame_extract, a reservation of another size or a batch extraction on the same
    handle ends the frame's results; the frame getters then fail with ESTATE instead of reading stale offsets."""
    import ctypes as C
    torch = pytest.importorskip("torch")
    from pyorbslam_amd import _lib
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.batch import StereoFrontEnd
    L, R = synth.make_pair(11)
    fe = StereoFrontEnd(max_pairs=1, lanes=1)
    h = fe.handle
    call("orbfe_frame_extract", h, _lib.ptr(L), _lib.ptr(R), 1241, 376, 1241, BF, float(np.float32(FX)), 0)
    n = C.c_int32()
    kps = np.empty(fe.kp_cap, _lib.KP_DTYPE)
    desc = np.empty((fe.kp_cap, 32), np.uint8)
    call("orbfe_frame_fetch", h, 0, _lib.ptr(kps), _lib.ptr(desc), fe.kp_cap, C.byref(n))  # valid
    assert n.value > 0
    call("orbfe_batch_reserve", h, 641, 333, 2)
    out = np.zeros(1241 * 376, np.uint8)
    w, hh = C.c_int32(), C.c_int32()
    for fn, args in (("orbfe_frame_pyramid", (h, 0, 0, _lib.ptr(out), C.byref(w), C.byref(hh))),
                     ("orbfe_frame_fetch", (h, 0, _lib.ptr(kps), _lib.ptr(desc), fe.kp_cap, C.byref(n)))):
        with pytest.raises(_lib.OrbfeError) as e:
            call(fn, *args)
        assert e.value.code == -5, fn
    call("orbfe_batch_reserve", h, 1241, 376, 2)
    call("orbfe_frame_extract", h, _lib.ptr(L), _lib.ptr(R), 1241, 376, 1241, BF, float(np.float32(FX)), 0)
    imgs = torch.from_numpy(synth.make_batch(1, seed0=12)).cuda()
    fe.enqueue(imgs, 1)
    with pytest.raises(_lib.OrbfeError) as e:
        call("orbfe_frame_pyramid", h, 1, 2, _lib.ptr(out), C.byref(w), C.byref(hh))
    assert e.value.code == -5


def test_right_extractor_keeps_its_pyramid_after_the_left_moves_on():
    """the right extractor of pair 1 keeps pair 1's right pyramid after the left extractor runs
    pair 2 with another right extractor, or a plain extract() — like the reference's independent extractors."""
    from oracle.oracle import OracleExtractor
    L1, R1 = synth.make_pair(21, 641, 333)
    L2, R2 = synth.make_pair(22, 641, 333)
    prm = dict(KITTI, nfeatures=700)
    left, rA, rB = ORBextractor(**prm), ORBextractor(**prm), ORBextractor(**prm)
    o = OracleExtractor(**prm)
    o.extract(R1)
    want = o.sheared_pyramid()
    left.operator_kd_stereo(L1, R1, rA, BF, np.float32(FX))
    left.operator_kd_stereo(L2, R2, rB, BF, np.float32(FX))
    for g_, w_ in zip(rA.GetImagePyramid(), want):
        assert np.array_equal(g_, w_)
    left.extract(L1)
    for g_, w_ in zip(rA.GetImagePyramid(), want):
        assert np.array_equal(g_, w_)
    o.extract(R2)
    for g_, w_ in zip(rB.GetImagePyramid(), o.sheared_pyramid()):
        assert np.array_equal(g_, w_)


@pytest.mark.parametrize("resize_first", [False, True])
def test_lazy_pyramid_first_read_after_a_plain_extract(resize_first):
    """a lazy frame's pyramids first read only after the left extractor ran a plain
    extract() — at the frame's size (the handle's last call is then no frame) or at another size (which clears
    the device ring, so every unread list is fetched first).  Both extractors' lists, and a Frame-style list
    taken before, still equal the oracle's sheared views of their own images."""
    from oracle.oracle import OracleExtractor
    L1, R1 = synth.make_pair(31, 641, 333)
    prm = dict(KITTI, nfeatures=700)
    left, rA = ORBextractor(**prm), ORBextractor(**prm)
    o = OracleExtractor(**prm)
    left.operator_kd_stereo(L1, R1, rA, BF, np.float32(FX))
    taken_left = left.GetImagePyramid()
    other = synth.make_pair(32, 500, 300)[0] if resize_first else L1
    left.extract(other)
    o.extract(R1)
    for g_, w_ in zip(rA.GetImagePyramid(), o.sheared_pyramid()):
        assert np.array_equal(g_, w_)
    o.extract(L1)
    for g_, w_ in zip(taken_left, o.sheared_pyramid()):
        assert np.array_equal(g_, w_)
    o.extract(other)
    for g_, w_ in zip(left.GetImagePyramid(), o.sheared_pyramid()):
        assert np.array_equal(g_, w_)


def test_lazy_frame_pyramids_ring():
    """the frame path's sheared pyramids stay in a device ring (ORBFE_FRAME_RING frames) and
    cross PCIe only when read.  Lists read late, copied lazily (Frame.copy) or forced out by the ring's
    eviction all equal the oracle's views of their own frame; unread lists of dropped frames cost nothing."""
    from oracle.oracle import OracleExtractor
    from pyorbslam_amd.pyORBExtractor import FRAME_RING, LazyPyramid
    seq = synth.StereoSequence(1, 1241, 376, 1.0)
    left, right = ORBextractor(**KITTI), ORBextractor(**KITTI)
    kept = []
    for k in range(FRAME_RING + 3):
        L, R = seq.frame(k)
        left.operator_kd_stereo(L, R, right, BF, np.float32(FX))
        pl, pr = left.GetImagePyramid(), right.GetImagePyramid()
        assert isinstance(pl, LazyPyramid) and not pl.filled and len(pl) == KITTI["nlevels"]
        kept.append((k, pl, pr.copy()))
        if 1 <= k <= FRAME_RING:
            assert not kept[1][1].filled  # frame 1's lists are still on the device ...
    # ... frames 0 .. 2 left the ring while their lists were alive: fetched at eviction
    assert all(kept[k][1].filled and kept[k][2].filled for k in range(3))
    assert not any(kept[k][1].filled or kept[k][2].filled for k in range(3, FRAME_RING + 3))
    o = OracleExtractor(**KITTI)
    for k in (0, 2, 3, FRAME_RING + 2):
        L, R = seq.frame(k)
        o.extract(L)
        assert all(np.array_equal(a, b) for a, b in zip(kept[k][1], o.sheared_pyramid())), f"left, frame {k}"
        o.extract(R)
        assert all(np.array_equal(a, b) for a, b in zip(kept[k][2], o.sheared_pyramid())), f"right, frame {k}"
    # the extractors' own GetImagePyramid of the last frame, and the eager path (built on request)
    last_r = right.GetImagePyramid()
    assert all(np.array_equal(a, b) for a, b in zip(last_r, o.sheared_pyramid()))
    L, R = seq.frame(FRAME_RING + 2)
    left.operator_kd_stereo(L, R, right, BF, np.float32(FX), want_pyramid=False)
    eager = right.GetImagePyramid()
    assert isinstance(eager, list) and all(np.array_equal(a, b) for a, b in zip(eager, o.sheared_pyramid()))
