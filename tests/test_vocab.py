"""BoW vocabulary (pyDBoW.TemplatedVocabulary drop-in): oracle and native loader on CPU, the gfx950
descent against the reference's own transform outputs (tests/golden/vocab_*.npz, made by
tests/golden/gen_golden_vocab.py from the reference pyDBoW)."""
import ctypes as C

import numpy as np
import pytest

from conftest import GOLDEN
import vocab_synth as VS
from oracle.vocab_oracle import VocabOracle

CASES = ["k5L3", "k10L4_ragged", "k20L2_ties"]


def load(case):
    return np.load(GOLDEN / f"vocab_{case}.npz", allow_pickle=False)


def golden_outputs(z, lu):
    bv = dict(zip(z[f"bv_word_{lu}"].tolist(), z[f"bv_w_{lu}"].tolist()))
    idx = z[f"fv_idx_{lu}"].tolist()
    off = np.concatenate([[0], np.cumsum(z[f"fv_len_{lu}"])]).tolist()
    fv = {n: idx[off[j]:off[j + 1]] for j, n in enumerate(z[f"fv_node_{lu}"].tolist())}
    return bv, fv


def same(got, want_bv, want_fv):
    bv, fv = got
    # exact float equality (same accumulation order as the reference) and the same key order
    assert list(bv.items()) == list(want_bv.items())
    assert list(fv.items()) == list(want_fv.items())


def tree_of(z):
    return dict(k=int(z["k"]), L=int(z["L"]), parent=z["parent"], is_leaf=z["is_leaf"], desc=z["desc"],
                weight=z["weight"])


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    z = load(case)
    o = VocabOracle(z["parent"], z["is_leaf"], z["desc"], z["weight"], int(z["L"]))
    for lu in z["levels_up"].tolist():
        same(o.transform(z["queries"], lu), *golden_outputs(z, lu))


@pytest.mark.parametrize("case", CASES)
def test_native_loader_roundtrip(case, tmp_path):
    """orbfe_vocab_load_text (host-only, no GPU) reproduces the tree the reference loads."""
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    z = load(case)
    path = tmp_path / "voc.txt"
    VS.write_text(tree_of(z), path, n1=2, n2=1)
    v = TemplatedVocabulary()
    assert v.load_from_text_file(path) is True
    assert (v.k, v.L, v.scoring, v.weighting) == (int(z["k"]), int(z["L"]), 2, 1)
    a = v.node_arrays()
    assert np.array_equal(a["parent"], z["parent"])
    assert np.array_equal(a["is_leaf"], z["is_leaf"])
    assert np.array_equal(a["desc"][1:], z["desc"][1:])
    assert np.array_equal(a["weight"], z["weight"])  # repr -> strtod round trip is exact
    assert v.size() == int(z["size"])
    o = VocabOracle(z["parent"], z["is_leaf"], z["desc"], z["weight"], int(z["L"]))
    assert np.array_equal(a["word_id"], o.word)


def test_loader_rejects_header_like_reference(tmp_path, capsys):
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    path = tmp_path / "bad.txt"
    VS.write_text(VS.make_tree(seed=4, k=3, L=2), path, k=21)
    v = TemplatedVocabulary()
    assert v.load_from_text_file(path) is False
    assert "Invalid parameters" in capsys.readouterr().out
    assert (v.k, v.L) == (21, 2) and v.size() == 0  # header assigned before the check, nodes untouched


def test_loader_format_errors(tmp_path):
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    path = tmp_path / "v.txt"
    VS.write_text(VS.make_tree(seed=5, k=3, L=2), path)
    lines = path.read_text().splitlines()
    for bad in (lines[1].rsplit(" ", 1)[0],                  # missing field
                "99 1 " + lines[1].split(" ", 2)[2],          # parent not yet defined
                " ".join(lines[1].split()[:2] + ["300"] + lines[1].split()[3:])):  # byte out of range
        path.write_text("\n".join([lines[0], bad] + lines[2:]) + "\n")
        with pytest.raises(ValueError):
            TemplatedVocabulary().load_from_text_file(path)
    with pytest.raises(FileNotFoundError):
        TemplatedVocabulary().load_from_text_file(tmp_path / "missing.txt")


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_transform_gpu_golden(case, tmp_path):
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    z = load(case)
    path = tmp_path / "voc.txt"
    VS.write_text(tree_of(z), path)
    v = TemplatedVocabulary()
    assert v.load_from_text_file(path)
    for lu in z["levels_up"].tolist():
        got = v.transform(z["queries"], lu)
        same(got, *golden_outputs(z, lu))
        assert type(got[0]).__name__ == str(z[f"bv_type_{lu}"])


@pytest.mark.gpu
def test_transform_many_and_feature():
    """One launch over several frames == per-frame transform; transform_feature threads nid."""
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    z = load("k10L4_ragged")
    v = TemplatedVocabulary(k=int(z["k"]), L=int(z["L"])).from_arrays(z["parent"], z["is_leaf"], z["desc"],
                                                                      z["weight"])
    q = z["queries"]
    frames = [q[:100], q[100:101], q[101:101], q[101:450], q[450:]]
    many = v.transform_many(frames, 1)
    for f, got in zip(frames, many):
        want = v.transform(f, 1)
        assert list(got[0].items()) == list(want[0].items()) and list(got[1].items()) == list(want[1].items())
    o = VocabOracle(z["parent"], z["is_leaf"], z["desc"], z["weight"], int(z["L"]))
    nid = 0
    for i in range(60):
        w, nid_new, wt = v.transform_feature(q[i], nid, 1)
        ow, on, owt = o.descend(q[i], int(z["L"]) - 1)
        assert (w, wt) == (ow, owt)
        assert nid_new == (on if on >= 0 else nid)
        nid = nid_new
    assert v.transform_feature(q[0], None, 1)[1] is None
    assert v.transform(np.zeros((0, 32), np.uint8)) == ({}, {})


@pytest.mark.gpu
def test_transform_orbvoc_sized_tree():
    """k=10, L=6 (ORBvoc's shape, ~1.1 M nodes): descent of 3000 descriptors vs the oracle."""
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    t = VS.make_full_tree(seed=7, k=10, L=6)
    v = TemplatedVocabulary(k=10, L=6).from_arrays(t["parent"], t["is_leaf"], t["desc"], t["weight"])
    assert v.info().n_nodes == len(t["parent"]) and v.info().depth == 6
    q = VS.query_descriptors(t, 8, 3000)
    word, node, w = v.descend(q, 4)
    o = VocabOracle(t["parent"], t["is_leaf"], t["desc"], t["weight"], 6)
    for i in range(0, 3000, 7):
        assert (int(word[i]), int(node[i]), float(w[i])) == o.descend(q[i], 2), i


@pytest.mark.gpu
def test_transform_device_entry_point():
    import torch
    from pyorbslam_amd._lib import call
    from pyorbslam_amd.vocabulary import TemplatedVocabulary
    z = load("k5L3")
    v = TemplatedVocabulary(k=5, L=3).from_arrays(z["parent"], z["is_leaf"], z["desc"], z["weight"])
    q = torch.from_numpy(z["queries"]).cuda()
    n = q.shape[0]
    word = torch.zeros(n, dtype=torch.int32, device="cuda")
    node = torch.zeros(n, dtype=torch.int32, device="cuda")
    w = torch.zeros(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    call("orbfe_vocab_transform_device", v._handle(), C.c_void_p(q.data_ptr()), n, 1, C.c_void_p(word.data_ptr()),
         C.c_void_p(node.data_ptr()), C.c_void_p(w.data_ptr()), C.c_void_p(s.cuda_stream))
    s.synchronize()
    hw, hn, hwt = v.descend(z["queries"], 2)
    assert np.array_equal(word.cpu().numpy(), hw) and np.array_equal(node.cpu().numpy(), hn)
    assert np.array_equal(w.cpu().numpy(), hwt)
