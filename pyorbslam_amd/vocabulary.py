"""Drop-in for pyDBoW.TemplatedVocabulary's loader and transform (pyDBoW/TemplatedVocabulary.py:23-160).

The reference descends the vocabulary tree one descriptor at a time in Python, with a per-byte popcount
per child (FORB.distance, FORB.py:30-32): ~10 us x k x L per feature, ~1 s per 2000-feature frame on
ORBvoc (k=10, L=6).  Here the text file is parsed natively (orbfe_vocab_load_text), the tree is laid
out child-run-contiguous in HBM, and every descriptor of a frame (or of many frames) descends in one
k_vocab_descend launch (pyorbslam_amd/csrc/orbfe_vocab.hip).  The host keeps only what is inherently
sequential: threading the previous feature's node id through descents that stop above the node level,
and accumulating the BoW weights in feature order so every float sum matches the reference's.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np

from . import _lib
from ._lib import ORBFE_EFORMAT, ORBFE_EREJECT, VocabInfo, call, check, lib, ptr


class TemplatedVocabulary:
    def __init__(self, k=10, L=5, weighting="TF_IDF", scoring="L1_NORM"):
        self.k = k
        self.L = L
        self.weighting = weighting
        self.scoring = scoring
        self._h = None

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h is not None and _lib._lib is not None:
            _lib._lib.orbfe_vocab_destroy(h)

    # TemplatedVocabulary.py:43-81
    def load_from_text_file(self, filename) -> bool:
        with open(filename, "r") as f:  # same exception as the reference for a missing file
            header = f.readline().strip().split()
        # the reference assigns k and L before validating the header (TemplatedVocabulary.py:46-53)
        self.k, self.L = int(header[0]), int(header[1])
        h = C.c_void_p()
        rc = lib().orbfe_vocab_load_text(str(filename).encode(), C.byref(h))
        if rc == ORBFE_EREJECT:
            print("Vocabulary loading failure: Invalid parameters in file!")
            return False
        if rc == ORBFE_EFORMAT:
            raise ValueError(lib().orbfe_last_error().decode(errors="replace"))
        check("orbfe_vocab_load_text", rc)
        self._replace(h)
        info = self.info()
        self.scoring, self.weighting = info.scoring, info.weighting
        return True

    def from_arrays(self, parent, is_leaf, desc, weight):
        """Install a tree given as per-node arrays (node 0 = root), e.g. one built in memory."""
        parent = np.ascontiguousarray(parent, np.int32)
        n = len(parent)
        leaf = np.ascontiguousarray(is_leaf, np.uint8)
        d = np.ascontiguousarray(desc, np.uint8).reshape(n, 32)
        w = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        call("orbfe_vocab_create", int(self.k), int(self.L), 0, 0, n, ptr(parent), ptr(leaf), ptr(d), ptr(w),
             C.byref(h))
        self._replace(h)
        return self

    def _replace(self, h):
        old, self._h = self._h, h
        if old is not None:
            lib().orbfe_vocab_destroy(old)

    def _handle(self):
        if self._h is None:  # an unloaded vocabulary is the bare root (TemplatedVocabulary.py:36)
            h = C.c_void_p()
            call("orbfe_vocab_create", int(self.k), int(self.L), 0, 0, 1, None, None, None, None, C.byref(h))
            self._h = h
        return self._h

    def info(self) -> VocabInfo:
        out = VocabInfo()
        call("orbfe_vocab_get_info", self._handle(), C.byref(out))
        return out

    def node_arrays(self) -> dict:
        n = int(self.info().n_nodes)
        a = dict(parent=np.zeros(n, np.int32), is_leaf=np.zeros(n, np.uint8), desc=np.zeros((n, 32), np.uint8),
                 weight=np.zeros(n, np.float64), word_id=np.zeros(n, np.int32))
        call("orbfe_vocab_get_nodes", self._handle(), *(ptr(a[k]) for k in ("parent", "is_leaf", "desc", "weight",
                                                                            "word_id")))
        return a

    # TemplatedVocabulary.py:96-97
    def size(self) -> int:
        return 0 if self._h is None else int(self.info().n_words)

    def descend(self, features, levels_up=4):
        """Raw per-descriptor (word id, node id at depth L - levels_up or -1, weight): one launch."""
        q = np.ascontiguousarray(features, np.uint8).reshape(-1, 32)
        n = len(q)
        word = np.zeros(n, np.int32)
        node = np.zeros(n, np.int32)
        w = np.zeros(n, np.float64)
        if n:
            call("orbfe_vocab_transform", self._handle(), ptr(q), n, int(self.L - levels_up), ptr(word), ptr(node),
                 ptr(w))
        return word, node, w

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        call("orbfe_vocab_last_ms", self._handle(), C.byref(ms))
        return float(ms.value)

    @staticmethod
    def _assemble(word, node, w):
        """BowVector + FeatureVector of one frame from its raw descents (TemplatedVocabulary.py:108-129;
        BowVector.py:8-35; FeatureVector.py:8-17)."""
        n = len(word)
        if n == 0:
            return {}, {}
        # a descent that stops above the node level keeps the previous feature's node id (initially 0)
        src = np.maximum.accumulate(np.where(node >= 0, np.arange(n), -1))
        nid = np.where(src >= 0, node[np.maximum(src, 0)], 0)
        keep = np.flatnonzero(w > 0)
        if len(keep) == 0:
            return {}, {}
        acc: dict = {}
        feats: dict = {}
        for i, wid, nd, wt in zip(keep.tolist(), word[keep].tolist(), nid[keep].tolist(), w[keep].tolist()):
            acc[wid] = acc[wid] + wt if wid in acc else wt
            feats.setdefault(nd, []).append(i)
        bv = OrderedDict(sorted(acc.items()))
        total = sum(bv.values())
        if total > 0:
            for key in bv:
                bv[key] /= total
        return bv, OrderedDict(sorted(feats.items()))

    # TemplatedVocabulary.py:108-129
    def transform(self, features, levels_up=4):
        return self._assemble(*self.descend(features, levels_up))

    def transform_many(self, frames, levels_up=4):
        """transform() of several frames with ONE kernel launch over all their descriptors."""
        frames = [np.ascontiguousarray(f, np.uint8).reshape(-1, 32) for f in frames]
        if not frames:
            return []
        word, node, w = self.descend(np.concatenate(frames), levels_up)
        out, o = [], 0
        for f in frames:
            out.append(self._assemble(word[o:o + len(f)], node[o:o + len(f)], w[o:o + len(f)]))
            o += len(f)
        return out

    # TemplatedVocabulary.py:131-160
    def transform_feature(self, feature, nid, levels_up):
        word, node, w = self.descend(np.asarray(feature).reshape(1, 32), levels_up)
        if nid is not None and node[0] >= 0:
            nid = int(node[0])
        return int(word[0]), nid, float(w[0])
