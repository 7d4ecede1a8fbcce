"""TEST INFRASTRUCTURE ONLY — CPU restatement of pyDBoW's vocabulary descent and BoW/feature-vector
assembly (TemplatedVocabulary.py:108-160, BowVector.py:8-35, FeatureVector.py:8-17), with a numpy
popcount table.  Pinned by tests/golden/vocab_*.npz (made by running the reference pyDBoW).  Only
tests/ and bench.py's cpu_baseline leg may use it; the product (pyorbslam_amd.vocabulary) never does.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

_POP8 = np.array([bin(i).count("1") for i in range(256)], np.int32)


class VocabOracle:
    def __init__(self, parent, is_leaf, desc, weight, L):
        parent = np.asarray(parent)
        n = len(parent)
        self.children = [[] for _ in range(n)]
        for i in range(1, n):
            self.children[int(parent[i])].append(i)
        self.child_arr = [np.array(c, np.int64) for c in self.children]
        self.desc = np.asarray(desc, np.uint8)
        self.weight = np.asarray(weight, np.float64)
        self.word = np.zeros(n, np.int64)
        w = 0
        for i in range(1, n):
            if is_leaf[i] > 0:
                self.word[i] = w
                w += 1
        self.L = L

    def descend(self, q, nid_level):
        """(word id, node at depth nid_level or -1, weight) of one descriptor: at each node the child at
        the smallest Hamming distance, the first one on ties (TemplatedVocabulary.py:143-150)."""
        node, level, nid = 0, 0, -1
        while self.children[node]:
            ch = self.child_arr[node]
            d = _POP8[np.bitwise_xor(self.desc[ch], q)].sum(axis=1)
            node = int(ch[int(np.argmin(d))])  # argmin returns the first minimum
            level += 1
            if level == nid_level:
                nid = node
        return int(self.word[node]), nid, float(self.weight[node])

    def transform(self, features, levels_up=4):
        words: dict = {}
        feats: dict = {}
        nid = 0
        for i in range(len(features)):
            wid, n, w = self.descend(features[i], self.L - levels_up)
            if n >= 0:
                nid = n
            if w > 0:
                words[wid] = words[wid] + w if wid in words else w
                feats.setdefault(nid, []).append(i)
        if not words:
            return {}, {}
        bv = OrderedDict(sorted(words.items()))
        s = 0
        for v in bv.values():
            s = s + v
        if s > 0:
            for key in list(bv):
                bv[key] = bv[key] / s
        return bv, OrderedDict(sorted(feats.items()))
