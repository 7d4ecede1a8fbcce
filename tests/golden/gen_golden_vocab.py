"""Generate BoW vocabulary goldens from the REFERENCE pyDBoW (build container only).

Imports /root/reference/pyDBoW read-only, loads seeded synthetic vocabularies (tests/vocab_synth.py)
through TemplatedVocabulary.load_from_text_file and records TemplatedVocabulary.transform outputs as
fixtures: the tree arrays, the query descriptors, and per (case, levels_up) the BoW vector (sorted word
ids + float64 weights) and the FeatureVector (sorted node ids + feature-index lists).  Nothing here
runs on the GPU box.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_vocab.py
"""
from __future__ import annotations

import sys
import tempfile
from pathlib import Path

import numpy as np

sys.dont_write_bytecode = True
ROOT = Path(__file__).resolve().parents[2]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, "/root/reference")

import vocab_synth as VS  # noqa: E402
from pyDBoW.TemplatedVocabulary import TemplatedVocabulary  # noqa: E402

# (name, tree kwargs, query seed, n queries, levels_up values)
CASES = [
    ("k5L3", dict(seed=1, k=5, L=3), 11, 300, (2, 4)),            # System.py:38 configuration
    ("k10L4_ragged", dict(seed=2, k=10, L=4, p_stop=0.25, p_dup=0.1, p_zero=0.1, order="dfs"), 12, 600, (1, 2, 4)),
    ("k20L2_ties", dict(seed=3, k=20, L=2, p_dup=0.4, p_zero=0.05), 13, 300, (1, 3)),
]


def main():
    for name, kw, qseed, nq, lups in CASES:
        tree = VS.make_tree(**kw)
        q = VS.query_descriptors(tree, qseed, nq)
        with tempfile.TemporaryDirectory() as td:
            path = Path(td) / "voc.txt"
            VS.write_text(tree, path)
            voc = TemplatedVocabulary()
            assert voc.load_from_text_file(str(path))
        out = dict(parent=tree["parent"], is_leaf=tree["is_leaf"], desc=tree["desc"], weight=tree["weight"],
                   k=tree["k"], L=tree["L"], queries=q, size=len(voc.words), levels_up=np.array(lups, np.int32))
        for lu in lups:
            bv, fv = voc.transform(q, lu)
            out[f"bv_word_{lu}"] = np.array(list(bv.keys()), np.int64)
            out[f"bv_w_{lu}"] = np.array(list(bv.values()), np.float64)
            out[f"fv_node_{lu}"] = np.array(list(fv.keys()), np.int64)
            out[f"fv_len_{lu}"] = np.array([len(v) for v in fv.values()], np.int64)
            out[f"fv_idx_{lu}"] = np.array([i for v in fv.values() for i in v], np.int64)
            out[f"bv_type_{lu}"] = type(bv).__name__
            print(name, "levels_up", lu, "words", len(bv), "nodes", len(fv))
        np.savez_compressed(GOLD / f"vocab_{name}.npz", **out)
    # header outside the accepted ranges: load_from_text_file prints and returns False
    with tempfile.TemporaryDirectory() as td:
        path = Path(td) / "bad.txt"
        VS.write_text(VS.make_tree(seed=4, k=3, L=2), path, k=21)
        voc = TemplatedVocabulary()
        print("reject header ->", voc.load_from_text_file(str(path)), "k", voc.k, "L", voc.L)


if __name__ == "__main__":
    main()
