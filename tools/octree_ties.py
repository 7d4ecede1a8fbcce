"""SURVEY H1 tie report: on how many pyramid levels is the reference extractor's own
output address-dependent?

DistributeOctTree's careful phase sorts (size, ExtractorNode*) pairs (ORBextractor.cpp:683) and stops at the
first division that reaches N (:729-730).  Equal-size nodes are therefore processed in heap-address order:
*  a level has a *straddle* when the break falls inside a run of equal-size nodes — which keypoints the
   level keeps then depends on the addresses (this build, like a monotonic allocator, divides the most
   recently created ones);
*  a level has *order ties* when the careful phase divided a run of >= 2 equal-size nodes — the order of
   their children in the list, i.e. of the level's keypoints, depends on the addresses.
Counts come from the oracle's restatement (oracle_octree_ties): test infrastructure, CPU only.

usage: python tools/octree_ties.py [--bench-pairs 512] [--procs 8] [--out profiles/octree_ties.json]
"""
import argparse
import json
import sys
from concurrent.futures import ProcessPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _ties_of(args):
    kind, idx, params = args
    from oracle.oracle import OracleExtractor
    from pyorbslam_amd import synth
    ex = OracleExtractor(**params)
    if kind == "bench":
        L, R = synth.make_pair(idx)
        return [ex.octree_ties(L), ex.octree_ties(R)]
    if kind == "euroc":
        L, R = synth.make_pair(idx, 752, 480)
        return [ex.octree_ties(L), ex.octree_ties(R)]
    if kind == "c3":
        import seq_harness as H
        seq = synth.StereoSequence(H.SEQ["seed"], H.SEQ["width"], H.SEQ["height"], H.SEQ["speed"])
        return [ex.octree_ties(im) for im in seq.frame(idx)]
    raise ValueError(kind)


def summarise(levels: np.ndarray) -> dict:
    """levels: (images, nlevels, 5) of oracle_octree_ties."""
    n_img, n_lv = levels.shape[:2]
    st, runs, careful = levels[..., 0], levels[..., 1], levels[..., 2]
    return {
        "images": int(n_img), "levels": int(n_img * n_lv),
        "levels_with_careful_phase": int((careful > 0).sum()),
        "levels_straddled": int(st.sum()),
        "frac_levels_straddled": round(float(st.mean()), 4),
        "levels_with_order_ties": int((runs > 0).sum()),
        "frac_levels_with_order_ties": round(float((runs > 0).mean()), 4),
        "images_with_a_straddle": int((st.sum(axis=1) > 0).sum()),
        "images_address_dependent_in_any_way": int(((st + runs).sum(axis=1) > 0).sum()),
        "straddle_frac_per_level": [round(float(v), 4) for v in st.mean(axis=0)],
        "straddled_run_nodes_mean": round(float(levels[..., 3][st > 0].mean()), 2) if st.any() else 0.0,
        "straddled_run_divided_mean": round(float(levels[..., 4][st > 0].mean()), 2) if st.any() else 0.0,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bench-pairs", type=int, default=512)
    ap.add_argument("--euroc-pairs", type=int, default=64)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "octree_ties.json"))
    a = ap.parse_args()
    from oracle.oracle import OracleExtractor
    from PIL import Image
    import seq_harness as H
    kitti = dict(nfeatures=2000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    euroc = dict(kitti, nfeatures=1000)
    out = {"what": __doc__.split("\n\n")[0], "source": "oracle/orb_oracle.cpp oracle_octree_ties (restates "
           "ORBextractor.cpp:539-762 with creation-order ties)"}
    jobs = {"bench_kitti_512pairs": [("bench", p, kitti) for p in range(a.bench_pairs)],
            "c3_sequence_96frames": [("c3", k, kitti) for k in range(H.SEQ["n_frames"])],
            "c5_euroc_pairs": [("euroc", p, euroc) for p in range(a.euroc_pairs)]}
    with ProcessPoolExecutor(a.procs) as ex:
        for name, js in jobs.items():
            res = np.array([t for r in ex.map(_ties_of, js, chunksize=4) for t in r])
            out[name] = summarise(res)
            print(name, out[name], flush=True)
    img = np.array(Image.open(ROOT / "tests" / "golden" / "kitti06-436.png").convert("L"))
    t = OracleExtractor(**kitti).octree_ties(img)
    out["kitti06_436_png"] = {**summarise(t[None]), "per_level": t.tolist()}
    from test_gpu_paths import _stress_images
    from pyorbslam_amd import synth
    stress = dict(_stress_images())
    stress["noise"] = np.random.default_rng(5).integers(0, 256, (376, 1241), dtype=np.uint8)
    out["stress_images"] = {k: {**summarise(OracleExtractor(**kitti).octree_ties(v)[None]),
                                "per_level": OracleExtractor(**kitti).octree_ties(v).tolist()} for k, v in stress.items()}
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
