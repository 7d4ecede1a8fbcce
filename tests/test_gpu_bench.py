"""The bench's N > 1 path on the GPU box: `bench.py --gpus 2` started as a fresh
process goes through its own launcher (torch.distributed.run child, two ranks sharing the one GPU with the
gloo backend, ORBFE_DIST_BACKEND=gloo), and its JSON line must report two ranks, a clean parity sample and
correct gathered records for the weak-scaling step and for C4."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_two_ranks_through_the_launcher():
    env = dict(os.environ, ORBFE_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--pairs", "8", "--steps", "3", "--warmup", "1",
           "--cpu-sample", "0", "--no-c3", "--roofline-steps", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["total_pairs_per_step"] == 16
    assert out["parity_failures"] == 0 and out["overflow"] == 0 and out["parity_checked_pairs"] == 16
    assert out["with_gather"]["record_check"] is True
    assert out["with_gather"]["pairs_gathered"] == 16
    # every gathered record unpacked on rank 0 and checked against its sender's digest
    assert out["with_gather"]["records_verified"] == 16
    assert out["c4_strong"]["with_gather"]["record_check"] is True
    assert out["c4_strong"]["with_gather"]["records_verified"] == 64
    assert out["c4_strong"]["pairs_per_gpu"] == 32
    assert out["host_fed"]["record_check"] is True


def test_c4_eight_ranks_through_the_launcher():
    """C4's real 8-way shape end to end — `bench.py --gpus 8 --total-pairs 64` through its own
    launcher, 8 ranks sharing the one GPU with gloo: the 8-rank shard plan (8 pairs each), the 8-sender
    rank-0 buffer, the compact unpack of 64 records, parity of every rank's pairs."""
    env = dict(os.environ, ORBFE_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--total-pairs", "64", "--pairs", "8", "--steps", "3",
           "--warmup", "1", "--cpu-sample", "0", "--no-c3", "--no-host-fed", "--roofline-steps", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["scaling"] == "strong"
    assert out["config"]["total_pairs_per_step"] == 64 and out["config"]["pairs_per_step_per_gpu"] == 8
    assert out["parity_failures"] == 0 and out["overflow"] == 0 and out["parity_checked_pairs"] == 64
    g = out["c4_strong"]["with_gather"]
    assert g["record_check"] is True and g["pairs_gathered"] == 64
    assert g["records_verified"] == 64 and g["padded_rows_zero"] == 0
    assert out["with_gather"]["record_check"] is True and out["with_gather"]["records_verified"] == 64
    assert out["with_gather"]["bytes_to_rank0"] == 64 * g["record_bytes"]
