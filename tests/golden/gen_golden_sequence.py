"""Generate the C3 tracking-loop golden (tests/golden/sequence_kitti_synth.npz) by running the REFERENCE
(build container only; imported read-only from /root/reference, nothing of it is stored).

Per frame k of pyorbslam_amd.synth.StereoSequence (tests/seq_harness.py describes the loop):
  * a reference Frame is made with Frame.__new__ and given the attributes Frame.__init__ sets
    (Frame.py:13-73) from the oracle's extraction of both images (keypoints, descriptors, sheared
    pyramids, scale tables); then the reference's OWN compute_stereo_matches, assign_features_to_grid,
    set_pose, unproject_stereo and is_in_frustum run on it.  Keypoints are stand-in objects exposing
    pt / octave / angle / size / response (what those methods read of cv2.KeyPoint; cv2 is absent, and
    Frame.py's module-level `import cv2` is satisfied by an EMPTY module object);
  * Tracking.track_with_motion_model (Tracking.py:578-591): pose = velocity @ last pose, then the
    reference ORBMatcher(0.9, True).search_by_projection_f_f at th 7, and 14 if < 20 matches;
  * Tracking.search_local_points (Tracking.py:439-468): map points matched above are marked seen, the
    other local map points (the map points of the last LOCAL_WINDOW frames, update_local_points order)
    go through the reference Frame.is_in_frustum(pMP, 0.5), then ORBMatcher(0.8, True)
    .search_by_projection_f_p(frame, local, 1);
  * the g2o pose optimisation (out of scope) is replaced by the ground-truth pose; then every keypoint
    with a stereo depth and no map point gets a new REFERENCE MapPoint(x3D, frame, map, idxF=i,
    kframe_bool=False) (Tracking.update_last_frame, Tracking.py:647-651), with mp_observations() set.

Stored: image digests, extraction digests, stereo lists, grid cells, predicted poses, every map point
(creator frame / keypoint, float32 position, observations), the in-view local map points with their
recorded frustum projections, and both searches' results.  The reference's wall-clock per stage is
recorded too (this container's CPU) as the reference-path timing for bench.py --mode frame.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_sequence.py
"""
from __future__ import annotations

import json
import sys
import threading
import time
import types
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import seq_harness as H  # noqa: E402
from oracle.oracle import OracleExtractor  # noqa: E402
from pyorbslam_amd import synth  # noqa: E402


class KP:
    """What the reference Frame / ORBMatcher / MapPoint read of cv2.KeyPoint."""
    __slots__ = ("pt", "octave", "angle", "size", "response")

    def __init__(self, k):
        self.pt = (float(k["x"]), float(k["y"]))
        self.octave = int(k["octave"])
        self.angle = float(k["angle"])
        self.size = float(k["size"])
        self.response = float(k["response"])


class MapStub:
    """The one Map member MapPoint.__init__ touches (MapPoint.py:28, 54)."""
    mMutexPointCreation = threading.Lock()


def import_reference():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    sys.path.insert(0, str(REF))
    import Frame as RFrame  # noqa: E402
    import MapPoint as RMapPoint  # noqa: E402
    import ORBMatcher as RMatcher  # noqa: E402
    return RFrame, RMapPoint, RMatcher


def kind(v) -> str:
    if isinstance(v, np.ndarray):
        assert v.dtype in (np.float32, np.float64) and v.size == 1 and v.ndim in (1, 2), (v.dtype, v.shape)
        return ("f32" if v.dtype == np.float32 else "f64") + ("[1]" if v.ndim == 1 else "[1,1]")
    if isinstance(v, np.float32):
        return "f32"
    if isinstance(v, np.float64):
        return "f64"
    assert isinstance(v, float), type(v)
    return "float"


def main():
    RFrame, RMapPoint, RMatcher = import_reference()
    seq = synth.StereoSequence(H.SEQ["seed"], H.SEQ["width"], H.SEQ["height"], H.SEQ["speed"])
    s = H.settings(seq.cam)
    fa = H.frame_args(s, seq.width, seq.height)
    exL, exR = OracleExtractor(**H.PARAMS), OracleExtractor(**H.PARAMS)
    tab = exL.tables()
    out = {}
    mps = []           # reference MapPoint objects, id = index
    mp_rec = []        # (frame, kp, pos f32 3, obs)
    ids = {}
    frames = []
    kinds = {}
    t_ref = {"stereo": [], "grid": [], "f_f": [], "f_p": []}
    velocity = None
    for k in range(H.SEQ["n_frames"]):
        p = f"f{k}_"
        L, R = seq.frame(k)
        out[p + "left_sha"], out[p + "right_sha"] = np.array(H.sha(L)), np.array(H.sha(R))
        kl, dl = exL.extract(L)
        kr, dr = exR.extract(R)
        for nm, a in (("kpsL", kl), ("descL", dl), ("kpsR", kr), ("descR", dr)):
            out[p + nm + "_sha"] = np.array(H.sha(a))
        f = RFrame.Frame.__new__(RFrame.Frame)
        (f.fx, f.fy, f.cx, f.cy, f.invfx, f.invfy, f.mfGridElementWidthInv, f.mfGridElementHeightInv, f.mnMinX,
         f.mnMaxX, f.mnMinY, f.mnMaxY, f.FRAME_GRID_ROWS, f.FRAME_GRID_COLS) = fa
        f.frame_args = fa
        f.mbf, f.mK, f.mDistCoef, f.mThDepth = s["mbf"], s["mK"], s["mDistCoef"], s["mThDepth"]
        f.mb = f.mbf / f.mK[0][0]
        f.mvKeys = [KP(a) for a in kl]
        f.mDescriptors = dl
        f.mvKeysRight = [KP(a) for a in kr]
        f.mDescriptorsRight = dr
        f.mnScaleLevels = H.PARAMS["nlevels"]
        f.mfScaleFactor = float(np.float32(H.PARAMS["scaleFactor"]))
        f.mfLogScaleFactor = np.log(f.mfScaleFactor)
        f.mvScaleFactors = [float(v) for v in tab["scale"]]
        f.mvInvScaleFactors = [float(v) for v in tab["inv_scale"]]
        f.mvLevelSigma2 = [float(v) for v in tab["sigma2"]]
        f.mvInvLevelSigma2 = [float(v) for v in tab["inv_sigma2"]]
        f.mvImagePyramidLeft = exL.sheared_pyramid()
        f.mvImagePyramidRight = exR.sheared_pyramid()
        f.N = len(f.mvKeys)
        f.mvKeysUn = f.mvKeys
        t0 = time.perf_counter()
        f.compute_stereo_matches()
        t1 = time.perf_counter()
        f.mvpMapPoints = [None] * f.N
        f.mvbOutlier = [False] * f.N
        f.assign_features_to_grid()
        t2 = time.perf_counter()
        t_ref["stereo"].append(t1 - t0)
        t_ref["grid"].append(t2 - t1)
        f.mnId = k
        f.mvImagePyramidLeft = f.mvImagePyramidRight = None
        su, vu = H.stereo_encode(f.mvuRight)
        sd, vd = H.stereo_encode(f.mvDepth)
        assert np.array_equal(su, sd)
        out[p + "st_status"], out[p + "st_u"], out[p + "st_d"] = su, vu, vd
        out[p + "grid"] = H.grid_cells(f)
        Tgt = seq.pose(k)
        if k == 0:
            f.set_pose(Tgt)
        else:
            last = frames[-1]
            # the prediction mVelocity @ mLastFrame.mTcw (Tracking.py:583); frame 1 predicts with the identity
            Tpred = (np.eye(4) if velocity is None else velocity) @ last.mTcw
            out[p + "Tpred"] = Tpred
            f.set_pose(Tpred)
            m = RMatcher.ORBMatcher(0.9, True)
            ta = time.perf_counter()
            f.mvpMapPoints = [None] * f.N
            n = m.search_by_projection_f_f(f, last, 7)
            th = 7
            if n < 20:
                f.mvpMapPoints = [None] * f.N
                n = m.search_by_projection_f_f(f, last, 14)
                th = 14
            tb = time.perf_counter()
            t_ref["f_f"].append(tb - ta)
            out[p + "ff_n"], out[p + "ff_th"] = np.array(n), np.array(th)
            out[p + "ff_assign"] = np.array([-1 if q is None else ids[id(q)] for q in f.mvpMapPoints], np.int32)
            # Tracking.search_local_points (Tracking.py:439-468)
            for q in f.mvpMapPoints:
                if q is not None:
                    q.mnLastFrameSeen = f.mnId
                    q.mbTrackInView = False
            local, seen = [], set()
            for fr in frames[-H.LOCAL_WINDOW:][::-1]:
                for q in fr.mvpMapPoints:
                    if q is not None and id(q) not in seen and not q.is_bad():
                        seen.add(id(q))
                        local.append(q)
            for q in local:
                if q.mnLastFrameSeen == f.mnId:
                    continue
                f.is_in_frustum(q, 0.5)
            inview = [q for q in local if q.mbTrackInView]
            for q in inview:
                for nm, v in (("x", q.mTrackProjX), ("y", q.mTrackProjY), ("xr", q.mTrackProjXR),
                              ("vcos", q.mTrackViewCos)):
                    kd = kind(v)
                    assert kinds.setdefault(nm, kd) == kd, (nm, kinds[nm], kd)
            out[p + "local_ids"] = np.array([ids[id(q)] for q in inview], np.int32)
            out[p + "local_px"] = np.array([float(np.asarray(q.mTrackProjX).ravel()[0]) for q in inview])
            out[p + "local_py"] = np.array([float(np.asarray(q.mTrackProjY).ravel()[0]) for q in inview])
            out[p + "local_pxr"] = np.array([float(np.asarray(q.mTrackProjXR).ravel()[0]) for q in inview])
            out[p + "local_level"] = np.array([int(q.mnTrackScaleLevel) for q in inview], np.int32)
            out[p + "local_vcos"] = np.array([float(np.asarray(q.mTrackViewCos).ravel()[0]) for q in inview])
            tc = time.perf_counter()
            n = RMatcher.ORBMatcher(0.8, True).search_by_projection_f_p(f, local, 1)
            td = time.perf_counter()
            t_ref["f_p"].append(td - tc)
            out[p + "fp_n"] = np.array(n)
            out[p + "fp_assign"] = np.array([-1 if q is None else ids[id(q)] for q in f.mvpMapPoints], np.int32)
            f.set_pose(Tgt)   # stand-in for Optimizer.pose_optimization (out of scope)
            # mVelocity = mCurrentFrame.mTcw @ LastTwc, LastTwc from the last frame (Tracking.py:224-229)
            LastTwc = np.concatenate((last.get_rotation_inverse(), last.get_camera_center()), axis=1)
            LastTwc = np.concatenate((LastTwc, np.array([[0, 0, 0, 1]])), axis=0)
            velocity = f.mTcw @ LastTwc
        out[p + "Tgt"] = Tgt
        # new map points for the keypoints with a stereo depth and no map point (Tracking.py:627-651)
        for i in range(f.N):
            if f.mvpMapPoints[i] is None and f.mvDepth[i] > 0:
                x3D = f.unproject_stereo(i)
                q = RMapPoint.MapPoint(x3D, f, MapStub(), idxF=i, kframe_bool=False)
                q.nObs = H.mp_observations(k, i)
                assert q.observations() == q.nObs
                ids[id(q)] = len(mps)
                mps.append(q)
                pos = q.get_world_pos()
                assert pos.dtype == np.float32 and pos.shape == (3, 1), (pos.dtype, pos.shape)
                mp_rec.append((k, i, pos.reshape(3), q.nObs))
                f.mvpMapPoints[i] = q
        f.mvbOutlier = [H.is_outlier(k, i) for i in range(f.N)]
        out[p + "slots"] = np.array([-1 if q is None else ids[id(q)] for q in f.mvpMapPoints], np.int32)
        out[p + "outlier"] = np.array(f.mvbOutlier, bool)
        frames.append(f)
        if k > 0:
            print(f"frame {k}: N={f.N} stereo={int((su > 0).sum())} f_f={int(out[p + 'ff_n'])} (th {int(out[p + 'ff_th'])}) "
                  f"local in view={len(out[p + 'local_ids'])} f_p={int(out[p + 'fp_n'])} new MPs={len(mps)}", flush=True)
    out["mp_frame"] = np.array([r[0] for r in mp_rec], np.int32)
    out["mp_kp"] = np.array([r[1] for r in mp_rec], np.int32)
    out["mp_pos"] = np.stack([r[2] for r in mp_rec]).astype(np.float32)
    out["mp_obs"] = np.array([r[3] for r in mp_rec], np.int32)
    meta = dict(seq=H.SEQ, params=H.PARAMS, cam=seq.cam, width=seq.width, height=seq.height,
                n_frames=H.SEQ["n_frames"], local_window=H.LOCAL_WINDOW, proj_kinds=kinds,
                reference_seconds_per_frame={k: float(np.mean(v)) for k, v in t_ref.items() if v},
                reference_timing_host="build container CPU, 1 thread (reference Python code, NumPy 2)")
    out["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(H.GOLDEN_FILE, **out)
    print("wrote", H.GOLDEN_FILE, "proj kinds", kinds, "reference s/frame", meta["reference_seconds_per_frame"])


if __name__ == "__main__":
    main()
