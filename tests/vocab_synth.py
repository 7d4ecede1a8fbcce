"""Seeded synthetic vocabulary trees in the reference's text format (TemplatedVocabulary.py:43-81).

ORBvoc.txt is not in the container, so vocabulary goldens use generated trees.  The
shapes exercise what the descent and the transform depend on: ragged depth (descents that stop above
the node level, so the previous feature's node id is carried), zero-weight leaves (skipped), duplicate
children (first-minimum ties) and depth-first node numbering (a node's children are not adjacent ids).
"""
from __future__ import annotations

import numpy as np


def make_tree(seed: int, k: int, L: int, p_stop: float = 0.0, p_dup: float = 0.0, p_zero: float = 0.0,
              order: str = "bfs") -> dict:
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, leaf, desc, weight = [0], [0], [np.zeros(32, np.uint8)], [0.0]

    def add(par, depth, d):
        nid = len(parent)
        is_leaf = depth == L or (depth >= 1 and rng.random() < p_stop)
        parent.append(par)
        leaf.append(1 if is_leaf else 0)
        desc.append(d)
        w = 0.0 if (not is_leaf or rng.random() < p_zero) else float(rng.uniform(0.05, 6.0))
        weight.append(w)
        return nid, is_leaf

    def children_desc(base):
        out = []
        for _ in range(k):
            if out and rng.random() < p_dup:
                out.append(out[int(rng.integers(0, len(out)))].copy())
            else:
                flip = rng.integers(0, 256, 32, dtype=np.uint8) & rng.integers(0, 256, 32, dtype=np.uint8)
                out.append(base ^ flip)
        return out

    root_base = rng.integers(0, 256, 32, dtype=np.uint8)
    if order == "bfs":
        frontier = [(0, 0, root_base)]
        while frontier:
            nxt = []
            for par, depth, base in frontier:
                for d in children_desc(base):
                    nid, is_leaf = add(par, depth + 1, d)
                    if not is_leaf:
                        nxt.append((nid, depth + 1, d))
            frontier = nxt
    else:  # depth-first numbering
        def rec(par, depth, base):
            for d in children_desc(base):
                nid, is_leaf = add(par, depth + 1, d)
                if not is_leaf:
                    rec(nid, depth + 1, d)
        rec(0, 0, root_base)
    return dict(k=k, L=L, parent=np.array(parent, np.int32), is_leaf=np.array(leaf, np.uint8),
                desc=np.stack(desc).astype(np.uint8), weight=np.array(weight, np.float64))


def write_text(tree: dict, path, n1: int = 0, n2: int = 0, k=None, L=None) -> None:
    """The ORBvoc text layout: header `k L scoring weighting`, then one line per node after the root:
    `parent is_leaf d0 .. d31 weight` (weights written with repr, so they round-trip exactly)."""
    k = tree["k"] if k is None else k
    L = tree["L"] if L is None else L
    with open(path, "w") as f:
        f.write(f"{k} {L} {n1} {n2}\n")
        for i in range(1, len(tree["parent"])):
            d = " ".join(str(int(b)) for b in tree["desc"][i])
            f.write(f"{int(tree['parent'][i])} {int(tree['is_leaf'][i])} {d} {float(tree['weight'][i])!r}\n")


def query_descriptors(tree: dict, seed: int, n: int) -> np.ndarray:
    """Uniform noise, perturbed node descriptors and exact node copies (distance-0 ties)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    nodes = len(tree["parent"])
    a = rng.integers(0, 256, (n // 3, 32), dtype=np.uint8)
    pick = rng.integers(1, nodes, n // 3)
    noise = (rng.integers(0, 256, (n // 3, 32), dtype=np.uint8) & rng.integers(0, 256, (n // 3, 32), dtype=np.uint8)
             & rng.integers(0, 256, (n // 3, 32), dtype=np.uint8))
    b = tree["desc"][pick] ^ noise
    c = tree["desc"][rng.integers(1, nodes, n - 2 * (n // 3))]
    q = np.concatenate([a, b, c])
    return q[rng.permutation(len(q))]


def make_full_tree(seed: int, k: int = 10, L: int = 6, p_zero: float = 0.02) -> dict:
    """A complete k-ary tree of depth L numbered breadth-first (ORBvoc's k=10, L=6 shape: 1 111 111
    nodes), built level by level with numpy; children descriptors are parent ^ (random & random)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    parent, desc = [np.zeros(1, np.int64)], [rng.integers(0, 256, (1, 32), dtype=np.uint8)]
    first = 0
    for depth in range(1, L + 1):
        prev = desc[-1]
        par = np.repeat(np.arange(len(prev)) + first, k)
        flip = rng.integers(0, 256, (len(par), 32), dtype=np.uint8) & rng.integers(0, 256, (len(par), 32),
                                                                                  dtype=np.uint8)
        desc.append(np.repeat(prev, k, axis=0) ^ flip)
        parent.append(par)
        first += len(prev)
    n_leaf = k ** L
    n = sum(len(p) for p in parent)
    weight = np.zeros(n)
    w = rng.uniform(0.05, 6.0, n_leaf)
    w[rng.random(n_leaf) < p_zero] = 0.0
    weight[n - n_leaf:] = w
    leaf = np.zeros(n, np.uint8)
    leaf[n - n_leaf:] = 1
    return dict(k=k, L=L, parent=np.concatenate(parent).astype(np.int32), is_leaf=leaf,
                desc=np.concatenate(desc), weight=weight)
