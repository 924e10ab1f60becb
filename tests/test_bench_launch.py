"""CPU tests of bench.py's own rank launcher (`python bench.py --gpus N` with no external launcher):
the parent starts N rank processes with the torch.distributed.run environment and never initialises the
GPU itself; a failing rank ends the others."""
from __future__ import annotations

import json
import sys
from types import SimpleNamespace

import pytest
import torch

import bench


def _no_gpu(monkeypatch):
    def boom(*a, **k):
        raise AssertionError("the launching parent initialised the GPU")

    monkeypatch.setattr(torch.cuda, "_lazy_init", boom)
    monkeypatch.setattr(torch.cuda, "set_device", boom)
    monkeypatch.setattr(torch.cuda, "current_stream", boom)
    monkeypatch.setattr(torch.cuda, "is_available", boom)


def test_spawn_ranks_environment(monkeypatch, tmp_path):
    _no_gpu(monkeypatch)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("OUT", str(tmp_path / "rank"))
    keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "DGE_AMD_BENCH_SPAWNED",
            "HSA_ENABLE_IPC_MODE_LEGACY")
    code = ("import json, os; open(os.environ['OUT'] + os.environ['RANK'], 'w').write(json.dumps("
            f"{{k: os.environ.get(k) for k in {keys!r}}}))")
    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    rc = bench.spawn_ranks(SimpleNamespace(gpus=3), argv=[], child_cmd=[sys.executable, "-c", code])
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{r}").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and {e["DGE_AMD_BENCH_SPAWNED"] for e in envs} == {"1"}
    assert {e["HSA_ENABLE_IPC_MODE_LEGACY"] for e in envs} == {"0"}  # (kept for RCCL's dmabuf IPC)


def test_spawn_ranks_failure_ends_the_others(monkeypatch):
    _no_gpu(monkeypatch)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(7) if r == 1 else time.sleep(120)"
    import time

    t0 = time.time()
    rc = bench.spawn_ranks(SimpleNamespace(gpus=3), argv=[], child_cmd=[sys.executable, "-c", code])
    assert rc == 7 and time.time() - t0 < 60


def test_main_spawns_before_touching_the_gpu(monkeypatch):
    _no_gpu(monkeypatch)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    def fake_spawn(args, argv=None, child_cmd=None):
        seen["gpus"] = args.gpus
        return 0

    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and seen["gpus"] == 8
