"""C3 tracking-loop replay (BASELINE config C3) against the golden made by running the REFERENCE's Frame /
MapPoint / ORBMatcher code on a synthetic moving stereo sequence (tests/golden/gen_golden_sequence.py,
tests/seq_harness.py).  Tolerance: none — extraction digests, stereo lists (types and values), grid cells
and both searches' assignments and counts must be identical in every frame.

  CPU: the golden's shape, and the first frames replayed through the oracle (extractor restatement,
       stereo restatement, matcher restatement), which pins the harness's own restated pieces.
  GPU: all 96 frames through the drop-in path — pyORBExtractor.ORBextractor with the pair-batched
       Frame.ExtractORB, compute_stereo_matches and Frame.copy installed by pyorbslam_amd.frame.install on
       the restated Frame class, and matcher.ORBMatcher."""
import json

import numpy as np
import pytest

import seq_harness as H
from pyorbslam_amd import synth

# the reference's is_in_frustum leaves 1-element arrays as projections, and get_features_in_area int()s them
pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


@pytest.fixture(scope="module")
def golden():
    return H.load_golden()


@pytest.fixture(scope="module")
def sequence(golden):
    meta = json.loads(str(golden["meta"]))
    return synth.StereoSequence(meta["seq"]["seed"], meta["width"], meta["height"], meta["seq"]["speed"])


def test_sequence_golden_shape(golden):
    meta = json.loads(str(golden["meta"]))
    n = meta["n_frames"]
    assert n >= 30
    for k in range(1, n):
        p = f"f{k}_"
        assert int(golden[p + "ff_n"]) >= 20 and int(golden[p + "fp_n"]) > 0
        assert len(golden[p + "local_ids"]) > 0
        assert golden[p + "Tpred"].dtype == np.float64
    assert golden["mp_pos"].dtype == np.float32 and len(golden["mp_pos"]) == len(golden["mp_frame"])


def test_sequence_images_reproduce(golden, sequence):
    for k in (0, 17):
        L, R = sequence.frame(k)
        assert H.sha(L) == str(golden[f"f{k}_left_sha"]) and H.sha(R) == str(golden[f"f{k}_right_sha"])


class _OracleExtractor:
    """The oracle extractor behind the reference pyORBExtractor surface (CPU test of the harness only)."""

    def __init__(self, **prm):
        from oracle.oracle import OracleExtractor
        self._o = OracleExtractor(**prm)
        self._t = self._o.tables()
        self.last_keypoints = None
        self.last_descriptors = None

    def operator_kd(self, image):
        k, d = self._o.extract(image)
        self.last_keypoints, self.last_descriptors = k, d
        return k.tolist(), d

    def GetLevels(self):
        return self._o.nlevels

    def GetScaleFactor(self):
        return float(np.float32(1.2))

    def GetScaleFactors(self):
        return [float(v) for v in self._t["scale"]]

    def GetInverseScaleFactors(self):
        return [float(v) for v in self._t["inv_scale"]]

    def GetScaleSigmaSquares(self):
        return [float(v) for v in self._t["sigma2"]]

    def GetInverseScaleSigmaSquares(self):
        return [float(v) for v in self._t["inv_sigma2"]]

    def GetImagePyramid(self):
        return self._o.sheared_pyramid()


class _OracleFrame(H.SeqFrame):
    def compute_stereo_matches(self):
        from oracle import stereo_oracle
        exL, exR = self.mpORBextractorLeft, self.mpORBextractorRight
        self.mvuRight, self.mvDepth, _ = stereo_oracle.compute_stereo_matches(
            exL.last_keypoints, exR.last_keypoints, exL.last_descriptors, exR.last_descriptors,
            self.mvImagePyramidLeft, self.mvImagePyramidRight, exL._t["scale"], exL._t["inv_scale"], self.mbf,
            self.mK[0][0])


class _OracleMatcher:
    def __init__(self, nnratio, check_ori):
        self.nnratio, self.check_ori = nnratio, check_ori

    def search_by_projection_f_f(self, cur, last, th):
        from oracle import matcher_oracle
        return matcher_oracle.search_f_f(cur, last, th, self.check_ori)

    def search_by_projection_f_p(self, frame, mps, th):
        from oracle import matcher_oracle
        return matcher_oracle.search_f_p(frame, mps, th, self.nnratio)


def test_sequence_replay_host_matcher(golden, sequence, monkeypatch):
    """Frames 0-3 through the oracle extraction and the drop-in ORBMatcher's host logic (batched grid
    queries, stacked projection, replay), its batched Hamming distances answered by the oracle popcount."""
    from pyorbslam_amd import matcher
    from oracle import matcher_oracle as MO

    from test_matcher import cpu_csr

    monkeypatch.setattr(matcher.ORBMatcher, "_csr", staticmethod(cpu_csr))
    taken = {"f_f": 0, "f_p": 0}
    for name in ("f_f", "f_p"):
        orig = getattr(matcher.ORBMatcher, f"_{name}_native")

        def spy(self, *a, _orig=orig, _name=name):
            r = _orig(self, *a)
            taken[_name] += r is not None
            return r
        monkeypatch.setattr(matcher.ORBMatcher, f"_{name}_native", spy)
    ex = (_OracleExtractor(**H.PARAMS), _OracleExtractor(**H.PARAMS))
    bad = H.replay(golden, sequence, ex, matcher.ORBMatcher, _OracleFrame, n_frames=4)
    assert not bad, bad
    assert taken["f_f"] >= 3 and taken["f_p"] >= 3, taken  # the tracking loop's doubles take the native selection


def test_sequence_replay_oracle(golden, sequence):
    """Frames 0-2 through the CPU restatements: pins SeqFrame / ReplayMP / the recorded inputs."""
    ex = (_OracleExtractor(**H.PARAMS), _OracleExtractor(**H.PARAMS))
    bad = H.replay(golden, sequence, ex, _OracleMatcher, _OracleFrame, n_frames=3)
    assert not bad, bad


@pytest.mark.gpu
def test_sequence_replay_gpu(golden, sequence):
    """All frames through the drop-in path on the GPU, bit-exact against the reference's tracking loop."""
    from pyorbslam_amd import frame as F
    from pyorbslam_amd.matcher import ORBMatcher
    from pyorbslam_amd.pyORBExtractor import ORBextractor

    class DropInFrame(H.SeqFrame):
        pass

    F.install(DropInFrame)
    ex = (ORBextractor(**H.PARAMS), ORBextractor(**H.PARAMS))
    timer = {}
    bad = H.replay(golden, sequence, ex, ORBMatcher, DropInFrame, timer=timer)
    assert not bad, bad[:10]
    assert len(timer["frame"]) == json.loads(str(golden["meta"]))["n_frames"]
