"""GPU tests of the execution paths that round 3 left unexercised:
HIP-graph replay against the stream path, the per-candidate octree kernel, the automatic octree choice,
k_detect's one-pass (queues met) path, a maximum-density FAST lattice, texture only in a corner (the
octree's last-lane bin maximum), and rows wider than 2 048 px at pyramid level 1 (k_resize_rows' chunk
loop).  Every result is compared bit for bit with the oracle or with the other path."""
import ctypes as C

import numpy as np
import pytest

from conftest import BF, FX, KITTI, EUROC
from oracle import oracle as O
from oracle import stereo_oracle
from pyorbslam_amd import synth
from pyorbslam_amd._lib import call
from pyorbslam_amd.pyORBExtractor import ORBextractor

pytestmark = pytest.mark.gpu


def _same_batches(a, b, n_pairs):
    for i in range(2 * n_pairs):
        x, y = a.fetch_image(i), b.fetch_image(i)
        assert x[0].tobytes() == y[0].tobytes() and np.array_equal(x[1], y[1]), f"image {i}"
    for p in range(n_pairs):
        x, y = a.fetch_stereo(p), b.fetch_stereo(p)
        assert all(np.array_equal(x[k], y[k]) for k in x), f"pair {p}"


@pytest.mark.parametrize("n_pairs", [1, 8])
def test_graph_replay_equals_stream_path(n_pairs):
    """The captured graph (default) against the launch-by-launch stream path on the same inputs: one pair
    and one rank's share of 8-way C4 (8 pairs), replayed several times and across two input buffers (the
    host-fed double buffering gives the graph cache two keys)."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    a_host = synth.make_batch(n_pairs, seed0=500)
    b_host = synth.make_batch(n_pairs, seed0=600)
    bufs = [torch.from_numpy(a_host).cuda(), torch.from_numpy(b_host).cuda()]
    ref = StereoFrontEnd(max_pairs=n_pairs, lanes=1, graphs=False)
    fe = StereoFrontEnd(max_pairs=n_pairs, lanes=1, graphs=True)
    st = torch.cuda.Stream()
    for it in range(5):
        d = bufs[it % 2]
        ref.enqueue(d, n_pairs)
        fe.enqueue(d, n_pairs, stream_ptr=st.cuda_stream)
        torch.cuda.synchronize()
        _same_batches(ref, fe, n_pairs)
        assert fe.overflow() == 0
    gs = fe.graph_stats()
    assert gs["captures"] == 2 and gs["launches"] == 5 and gs["cached"] == 2, gs
    assert ref.graph_stats()["launches"] == 0
    # and against the oracle, so that both paths are not merely equal to each other
    kl, dl = fe.fetch_image(0)
    okl, odl = O.OracleExtractor(**KITTI).extract(a_host[0])  # the last step read bufs[0]
    assert kl.tobytes() == okl.tobytes() and np.array_equal(dl, odl)


@pytest.mark.parametrize("lanes", [2, 3])
def test_multilane_graph_equals_stream_path(lanes):
    """the multi-lane fork / join (orbfe_set_lanes: the pairs as `lanes` chunks on internal
    streams, forked from and joined into the caller's stream with events) captured as ONE graph with parallel
    branches, replayed across two input buffers, against the one-lane stream path."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    n_pairs = 8
    bufs = [torch.from_numpy(synth.make_batch(n_pairs, seed0=s0)).cuda() for s0 in (520, 620)]
    ref = StereoFrontEnd(max_pairs=n_pairs, lanes=1, graphs=False)
    fe = StereoFrontEnd(max_pairs=n_pairs, lanes=lanes, graphs=True)
    st = torch.cuda.Stream()
    for it in range(5):
        d = bufs[it % 2]
        ref.enqueue(d, n_pairs)
        fe.enqueue(d, n_pairs, stream_ptr=st.cuda_stream)
        torch.cuda.synchronize()
        _same_batches(ref, fe, n_pairs)
        assert fe.overflow() == 0
    gs = fe.graph_stats()
    assert gs["captures"] == 2 and gs["launches"] == 5 and gs["cached"] == 2, gs


def test_graph_cache_eviction_with_new_inputs_every_step():
    """with graphs on and a new input buffer every step, every enqueue captures a graph
    and, past the 8-entry cache, evicts the oldest one while earlier steps are still queued on the caller's
    stream (no synchronisation between enqueues).  Eviction must wait for the evicted executable's last
    launch; the results of every step stay bit-exact to the stream path."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    n_pairs, steps = 2, 12
    hosts = [synth.make_batch(n_pairs, seed0=700 + 10 * k) for k in range(steps)]
    ref = StereoFrontEnd(max_pairs=n_pairs, lanes=1, graphs=False)
    fe = StereoFrontEnd(max_pairs=n_pairs, lanes=1, graphs=True)
    st = torch.cuda.Stream()
    bufs = [torch.from_numpy(h).cuda() for h in hosts]  # 12 distinct pointers: 12 keys
    torch.cuda.synchronize()
    for d in bufs:  # back to back, no synchronisation: evictions overlap queued replays
        fe.enqueue(d, n_pairs, stream_ptr=st.cuda_stream)
    st.synchronize()
    ref.enqueue(bufs[-1], n_pairs)
    torch.cuda.synchronize()
    _same_batches(ref, fe, n_pairs)
    gs = fe.graph_stats()
    assert gs["captures"] == steps and gs["launches"] == steps and gs["cached"] == 8, gs
    assert fe.overflow() == 0
    # a second round over the same pointers: all evicted keys are captured again, results still exact
    for d in bufs:
        fe.enqueue(d, n_pairs, stream_ptr=st.cuda_stream)
    st.synchronize()
    _same_batches(ref, fe, n_pairs)
    kl, dl = fe.fetch_image(1)
    okl, odl = O.OracleExtractor(**KITTI).extract(hosts[-1][1])
    assert kl.tobytes() == okl.tobytes() and np.array_equal(dl, odl)


def test_graph_frame_path_equals_stream_path():
    """orbfe_frame_extract (Frame(L, R) drop-in) replayed from its graph vs the stream path, over frames of a
    moving sequence (new image contents every call, the same staging buffers), with and without pyramids."""
    seq = synth.StereoSequence(0, 1241, 376, 1.0)
    a, ar = ORBextractor(**KITTI), ORBextractor(**KITTI)
    b, br = ORBextractor(**KITTI), ORBextractor(**KITTI)
    call("orbfe_set_graphs", b.handle, 0)
    for k in range(4):
        L, R = seq.frame(k)
        pyr = k % 2 == 0
        ga = a.operator_kd_stereo(L, R, ar, BF, np.float32(FX), want_pyramid=pyr)
        gb = b.operator_kd_stereo(L, R, br, BF, np.float32(FX), want_pyramid=pyr)
        for x, y in zip(ga, gb):
            assert x.tobytes() == y.tobytes()
        for key in a.stereo_result:
            assert np.array_equal(a.stereo_result[key], b.stereo_result[key])
        for x, y in zip(ar.GetImagePyramid(), br.GetImagePyramid()):
            assert np.array_equal(x, y)
    cap, lau = C.c_int64(), C.c_int64()
    call("orbfe_graph_stats", a.handle, C.byref(cap), C.byref(lau), None)
    assert cap.value == 1 and lau.value == 4  # lazy pyramids (k_shear behind the graph) or none: one graph
    kl, dl = O.OracleExtractor(**KITTI).extract(seq.frame(3)[0])
    assert ga[0].tobytes() == kl.tobytes() and np.array_equal(ga[1], dl)


def _octree_kernel(ex):
    k, b = C.c_int32(), C.c_int64()
    call("orbfe_get_octree_kernel", ex.handle, C.byref(k), C.byref(b))
    return k.value, b.value


def _stress_images():
    rng = np.random.default_rng(21)
    # every 4th pixel of every 4th row a bright dot on black: each dot is an isolated FAST corner (its
    # 16 circle pixels are dark, no other dot lies on the circle), all with the same score; the densest
    # lattice of corners a strict 3x3 NMS keeps
    lattice = np.zeros((376, 1241), np.uint8)
    lattice[::4, ::4] = 255
    # texture only in the top-left corner: every level's keys fall in the first octree bins, and the last
    # key of a sweep sits in bin 0 (the tail of the per-bin maximum)
    corner = np.full((376, 1241), 100, np.uint8)
    corner[:48, :48] = rng.integers(0, 256, (48, 48))
    return {"lattice": lattice, "corner": corner}


@pytest.mark.parametrize("name", ["lattice", "corner"])
def test_stress_images_bit_exact(name):
    img = _stress_images()[name]
    ex = ORBextractor(**KITTI)
    kps, desc = ex.extract(img)  # raises on an overflow code
    okps, odesc = O.OracleExtractor(**KITTI).extract(img)
    assert len(kps) == len(okps) > 0
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)


def _detect_stats(img_pair):
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    fe = StereoFrontEnd(max_pairs=1, lanes=1)
    fe.enqueue(torch.from_numpy(np.stack(img_pair)).cuda(), 1)
    ovf = fe.overflow()
    st = (C.c_int64 * 3)()
    call("orbfe_debug_detect_stats", fe.handle, st)
    return fe, ovf, list(st)


def test_fast_lattice_stays_in_capacity():
    """The densest lattice of isolated corners: every candidate a cell can hold under the strict NMS
    (slot_cap) and the octree's equal-score ties; the overflow word stays 0 and the result is bit-exact."""
    img = _stress_images()["lattice"]
    fe, ovf, st = _detect_stats((img, img))
    assert ovf == 0 and st[0] == 2 * 1220, st
    kl, dl = fe.fetch_image(0)
    okl, odl = O.OracleExtractor(**KITTI).extract(img)
    assert kl.tobytes() == okl.tobytes() and np.array_equal(dl, odl)


def test_noise_takes_the_one_pass_path():
    """Uniform noise passes the cardinal pre-test at both thresholds almost everywhere, so a cell's minTh
    queue (from the front) and iniTh queue (from the back) meet and the cell takes k_detect's one-pass path
    (both thresholds over the minTh queue; orbfe_debug_detect_stats[1]); bit-exact against the oracle."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (376, 1241)).astype(np.uint8)
    fe, ovf, st = _detect_stats((img, img))
    assert ovf == 0 and st[1] > st[0] // 2, st
    kl, dl = fe.fetch_image(0)
    okl, odl = O.OracleExtractor(**KITTI).extract(img)
    assert kl.tobytes() == okl.tobytes() and np.array_equal(dl, odl)


def test_natural_images_take_the_two_queue_path():
    """On the synthetic KITTI image no cell's queues meet; most cells fall back to minTh."""
    _, ovf, st = _detect_stats(tuple(synth.make_batch(1, seed0=0)))
    assert ovf == 0 and st[0] == 2 * 1220 and st[1] == 0 and st[2] > st[0] // 3, st


NAMES = ["kitti", "euroc", "noise", "patch", "lattice", "corner"]


def _octree_images():
    rng = np.random.default_rng(5)
    patch = np.full((376, 1241), 90, np.uint8)
    patch[170:202, 600:632] = rng.integers(0, 256, (32, 32))
    out = {"kitti": (synth.make_pair(0)[0], KITTI), "euroc": (synth.make_pair(100, 752, 480)[0], EUROC),
           "noise": (rng.integers(0, 256, (376, 1241)).astype(np.uint8), KITTI), "patch": (patch, KITTI)}
    out.update({k: (v, KITTI) for k, v in _stress_images().items()})
    return out


@pytest.mark.parametrize("name", NAMES)
def test_per_candidate_octree_kernel_bit_exact(name):
    """orbfe_set_octree_kernel(1) forces k_octree (the automatic fallback of k_octree_bins) on images that
    the bins kernel handles by default: both must give the oracle's keypoints and descriptors."""
    img, params = _octree_images()[name]
    ex = ORBextractor(**params)
    call("orbfe_set_octree_kernel", ex.handle, 1)
    kps, desc = ex.extract(img)
    assert _octree_kernel(ex)[0] == 1
    okps, odesc = O.OracleExtractor(**params).extract(img)
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)
    call("orbfe_set_octree_kernel", ex.handle, 0)
    k2, d2 = ex.extract(img)
    assert _octree_kernel(ex)[0] == 0
    assert k2.tobytes() == okps.tobytes() and np.array_equal(d2, odesc)


def test_automatic_octree_choice_of_tested_geometries():
    """Every camera / configuration the suites test runs k_octree_bins (its LDS carve fits 150 KiB); the
    per-candidate fallback is reached only by forcing it (DESIGN §4 gives the bound)."""
    from test_gpu_extract import CONFIGS
    geos = [((376, 1241), KITTI), ((480, 752), EUROC), ((360, 640), dict(EUROC)), ((400, 2560), KITTI)] + CONFIGS
    for (h, w), params in geos:
        ex = ORBextractor(**params)
        ex.extract(synth.make_pair(1, w, h)[0])
        k, lds = _octree_kernel(ex)
        assert k == 0 and 0 < lds <= 150 * 1024, ((h, w), params, lds)


@pytest.mark.parametrize("w", [2460, 2560, 3000])
def test_wide_images_resize_and_extract(w):
    """level 1 of these widths is wider than 2 048 px (> 8 chunks of 64 four-pixel groups),
    so k_resize_rows' waves walk several chunks; pyramid, keypoints and descriptors against the oracle."""
    img = synth.make_pair(77, w, 400)[0]
    ex = ORBextractor(**KITTI)
    kps, desc = ex.extract(img)
    orc = O.OracleExtractor(**KITTI)
    okps, odesc = orc.extract(img)
    for l, (g, o) in enumerate(zip(ex.GetImagePyramid(sheared=False), orc.pyramid())):
        assert np.array_equal(g, o), f"level {l}"
    assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc)


def test_graph_stereo_against_restatement_after_replays():
    """Three replays of one pair's graph; the last results against the stereo restatement."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    from pyorbslam_amd.frame import to_reference_lists
    host = synth.make_batch(1, seed0=42)
    fe = StereoFrontEnd(max_pairs=1, lanes=1)
    d = torch.from_numpy(host).cuda()
    for _ in range(3):
        fe.enqueue(d, 1)
    torch.cuda.synchronize()
    oL, oR = O.OracleExtractor(**KITTI), O.OracleExtractor(**KITTI)
    kl, dl = oL.extract(host[0])
    kr, dr = oR.extract(host[1])
    t = oL.tables()
    ou, od, _ = stereo_oracle.compute_stereo_matches(kl, kr, dl, dr, oL.sheared_pyramid(), oR.sheared_pyramid(),
                                                     t["scale"], t["inv_scale"], BF, np.float32(FX))
    u, dd = to_reference_lists(fe.fetch_stereo(0), fe.fetch_image(0)[0], BF)
    for a, b in ((u, ou), (dd, od)):
        sa, va = stereo_oracle.encode(a)
        sb, vb = stereo_oracle.encode(b)
        assert np.array_equal(sa, sb) and np.array_equal(va, vb)


@pytest.mark.parametrize("shape,params", [((376, 1241), KITTI), ((480, 752), EUROC), ((333, 641), KITTI),
                                          ((157, 211), dict(KITTI, nfeatures=500)), ((400, 2560), KITTI),
                                          ((376, 1241), dict(KITTI, scaleFactor=1.1, nlevels=12)),
                                          # exact 2x steps (INTER_AREA fast path) and levels down to 6 / 17 px
                                          ((376, 1241), dict(KITTI, scaleFactor=2.0, nlevels=4)),
                                          ((400, 400), dict(KITTI, nfeatures=1000, scaleFactor=2.0, nlevels=7)),
                                          ((128, 128), dict(KITTI, nfeatures=300, nlevels=12))])
def test_resize_cascade_equals_per_level_launches(shape, params):
    """k_resize_cascade (the one-launch pyramid of small batches, strips with halo rows) against the
    per-level k_resize_rows launches and the oracle, at several strip counts (orbfe_microbench stage 0:
    variant 7 = per-level, 100 + S = the cascade with S strips)."""
    h, w = shape
    img = synth.make_pair(31, w, h)[0]
    ex = ORBextractor(**params)
    ex.extract(img)  # one image: the cascade path
    auto = ex.GetImagePyramid(sheared=False)
    orc = O.OracleExtractor(**params)
    orc.extract(img)
    for l, (g, o) in enumerate(zip(auto, orc.pyramid())):
        assert np.array_equal(g, o), f"cascade level {l}"
    ms = C.c_float()
    call("orbfe_microbench", ex.handle, 0, 7, 1, C.byref(ms))
    for l, (g, o) in enumerate(zip(ex.GetImagePyramid(sheared=False), orc.pyramid())):
        assert np.array_equal(g, o), f"per-level level {l}"
    top_h = orc.pyramid()[-1].shape[0]
    for S in sorted({1, 2, 5, max(1, top_h // 3), top_h}):
        call("orbfe_microbench", ex.handle, 0, 100 + S, 1, C.byref(ms))
        for l, (g, o) in enumerate(zip(ex.GetImagePyramid(sheared=False), orc.pyramid())):
            assert np.array_equal(g, o), f"cascade S={S} level {l}"


def test_deep_octree_nodes_batch_and_single():
    """Frames 60-75 of the C3 sequence cluster their level-0 / level-1 corners so that the octree divides
    hundreds of nodes below the bin depth D0 (tools/octree_profile.py --seq; DESIGN §4 k_octree_bins, round
    4): the all-wave deep sweeps over the cached keys, in the 256-thread batch variant (32 images) and the
    1 024-thread one (one image), against the oracle on a sample of the images."""
    torch = pytest.importorskip("torch")
    from pyorbslam_amd.batch import StereoFrontEnd
    seq = synth.StereoSequence(0, 1241, 376, 0.6)
    imgs = np.stack([im for k in range(60, 76) for im in seq.frame(k)])
    fe = StereoFrontEnd(max_pairs=16, lanes=1)
    fe.enqueue(torch.from_numpy(imgs).cuda(), 16)
    assert fe.overflow() == 0
    ex = ORBextractor(**KITTI)
    ox = O.OracleExtractor(**KITTI)
    for i in (0, 9, 19, 30):
        okps, odesc = ox.extract(imgs[i])
        kps, desc = fe.fetch_image(i)
        assert kps.tobytes() == okps.tobytes() and np.array_equal(desc, odesc), f"batch image {i}"
        k1, d1 = ex.extract(imgs[i])
        assert k1.tobytes() == okps.tobytes() and np.array_equal(d1, odesc), f"single image {i}"
