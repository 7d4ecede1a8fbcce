"""bench.py's launcher and argument logic on the CPU: `--gpus N` either starts N ranks
or fails loudly, a torch.distributed environment that disagrees with --gpus exits non-zero, and the C4 /
strong-scaling shard plan covers every pair once."""
import json
import os
import subprocess
import sys
import types

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def run_bench(args, env_extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True, text=True,
                          timeout=300)


def test_world_size_mismatch_exits_2():
    r = run_bench(["--gpus", "4", "--cpu-sample", "0"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_gpus_without_enough_devices_fails_loudly():
    # this container has no GPU: `--gpus 2` must not fall back to one rank
    r = run_bench(["--gpus", "2", "--cpu-sample", "0"], {})
    assert r.returncode == 2
    assert "needs 2 GPUs" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_launcher_starts_n_ranks(monkeypatch):
    import torch
    seen = {}

    def fake_run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return types.SimpleNamespace(returncode=0)

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--total-pairs", "64"])
    args = types.SimpleNamespace(gpus=8)
    assert bench.launch_ranks(args) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--total-pairs", "64"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_check_world(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.check_world(types.SimpleNamespace(gpus=1)) == (1, 0, 0)
    assert bench.check_world(types.SimpleNamespace(gpus=2)) is None
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert bench.check_world(types.SimpleNamespace(gpus=8)) == (8, 3, 3)
    with pytest.raises(SystemExit):
        bench.check_world(types.SimpleNamespace(gpus=1))


@pytest.mark.parametrize("total", [64, 65, 7, 1])
def test_strong_scaling_shards(total):
    for world in (1, 2, 4, 8):
        spans = [bench.shard(total, world, r) for r in range(world)]
        assert sum(c for _, c in spans) == total
        assert [s for s, _ in spans] == [sum(c for _, c in spans[:r]) for r in range(world)]


def test_stamped_lookup(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "x.json").write_text(json.dumps({"w": {"detect": 1.0}, "w_meta": {"build_id": "abc"}}))
    v, src = bench.stamped("x.json", "w", "abc")
    assert v == {"detect": 1.0} and "abc" in src
    v, src = bench.stamped("x.json", "w", "def")
    assert v is None and "dropped" in src
    v, src = bench.stamped("x.json", "other", "abc")
    assert v is None
