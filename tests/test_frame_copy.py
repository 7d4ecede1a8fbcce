"""Frame.copy drop-in (pyorbslam_amd.frame.frame_copy) against tests/golden/frame_copy.json, which
tests/golden/gen_golden_frame_copy.py made by running the reference Frame.copy (Frame.py:75-112) and
the drop-in on the same reference Frame and comparing every attribute."""
import json

import numpy as np

from conftest import GOLDEN
from pyorbslam_amd.frame import frame_copy


class _NoExtract:
    def operator_kd(self, img):
        raise AssertionError("frame_copy must not extract")


class StandInFrame:
    """The attribute state of a constructed, posed Frame; set_pose as Frame.py:126-135."""
    nNextId = 40

    def set_pose(self, Tcw_):
        self.mTcw = Tcw_.copy()
        self.mRcw = self.mTcw[:3, :3]
        self.mRwc = self.mRcw.T
        self.mtcw = self.mTcw[:3, 3].reshape(3, 1)
        self.mOw = -np.dot(self.mRwc, self.mtcw)


def make_frame():
    rng = np.random.default_rng(3)
    f = StandInFrame()
    n = 50
    f.frame_args = [718.856, 718.856, 607.1928, 185.2157, 1 / 718.856, 1 / 718.856, 64 / 1241, 48 / 376, 0.0, 1241.0,
                    0.0, 376.0, 48, 64]
    (f.fx, f.fy, f.cx, f.cy, f.invfx, f.invfy, f.mfGridElementWidthInv, f.mfGridElementHeightInv, f.mnMinX, f.mnMaxX,
     f.mnMinY, f.mnMaxY, f.FRAME_GRID_ROWS, f.FRAME_GRID_COLS) = f.frame_args
    f.mpORBvocabulary = object()
    f.mbf = 386.1448
    f.mK = np.array([[718.856, 0, 607.1928], [0, 718.856, 185.2157], [0, 0, 1]], np.float32)
    f.mDistCoef = np.zeros((1, 5), np.float32)
    f.mleft = rng.integers(0, 256, (376, 1241), dtype=np.uint8)
    f.mright = rng.integers(0, 256, (376, 1241), dtype=np.uint8)
    f.mTimeStamp = 0.5
    f.mThDepth = 35.0
    f.mBowVec = None
    f.mFeatVec = None
    f.mpReferenceKF = None
    f.mb = f.mbf / f.mK[0][0]
    f.mpORBextractorLeft = _NoExtract()
    f.mpORBextractorRight = _NoExtract()
    f.mvKeys_ = [(float(i), 2.0, 7.0, 10.0, 30.0, 0) for i in range(n)]
    f.mvKeysRight_ = [(float(i), 3.0, 7.0, 10.0, 30.0, 0) for i in range(n)]
    f.mvKeys = [object() for _ in range(n)]
    f.mvKeysRight = [object() for _ in range(n)]
    f.mDescriptors = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    f.mDescriptorsRight = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    f.mnScaleLevels = 8
    f.mfScaleFactor = 1.2000000476837158
    f.mfLogScaleFactor = float(np.log(f.mfScaleFactor))
    f.mvScaleFactors = [1.2 ** i for i in range(8)]
    f.mvInvScaleFactors = [1.2 ** -i for i in range(8)]
    f.mvLevelSigma2 = [1.44 ** i for i in range(8)]
    f.mvInvLevelSigma2 = [1.44 ** -i for i in range(8)]
    f.mvImagePyramidLeft = [rng.integers(0, 256, (20 - i, 30 - i), dtype=np.uint8) for i in range(8)]
    f.mvImagePyramidRight = [rng.integers(0, 256, (20 - i, 30 - i), dtype=np.uint8) for i in range(8)]
    f.N = n
    f.mvKeysUn = f.mvKeys
    f.mvuRight = [-1] * n
    f.mvDepth = [-1] * n
    f.mvpMapPoints = [None] * n
    f.mvbOutlier = [False] * n
    f.mGrid = [[[] for _ in range(48)] for _ in range(64)]
    f.mnId = 7
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = (0.1, -0.2, 1.5)
    f.set_pose(T)
    return f


def relation(a, b):
    if a is b:
        return "is"
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return "equal" if np.array_equal(np.asarray(a), np.asarray(b)) else "new"
    if isinstance(a, list) and isinstance(b, list):
        ok = len(a) == len(b) and all(relation(x, y) in ("is", "equal") for x, y in zip(a, b))
        return "equal" if ok else "new"
    return "equal" if a == b else "new"


def test_frame_copy_matches_reference_semantics():
    gold = json.loads((GOLDEN / "frame_copy.json").read_text())
    f = make_frame()
    n0 = StandInFrame.nNextId
    c = frame_copy(f, f)
    assert StandInFrame.nNextId - n0 == gold["reference_id_draws"] == gold["dropin_id_draws"]
    assert gold["dropin_extract_calls"] == 0 and gold["reference_extract_calls"] == 2
    rel = gold["attributes"]
    assert sorted(vars(c)) == sorted(rel)
    for k, r in rel.items():
        got = relation(getattr(c, k), getattr(f, k))
        # scalars the reference passes through (`is` there) may be equal-but-new here, never different
        assert got == r or (r == "is" and got == "equal" and not isinstance(getattr(f, k), (list, np.ndarray))), k
    # the shared containers stay shared, the copied arrays are fresh
    assert c.mvpMapPoints is f.mvpMapPoints and c.mGrid is f.mGrid
    assert c.mDescriptors is not f.mDescriptors and c.mvImagePyramidLeft[0] is not f.mvImagePyramidLeft[0]
