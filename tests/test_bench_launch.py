"""bench.py --gpus N started as a plain process spawns its own N ranks.

The driver runs `python3 bench.py --gpus N ...`; the rank processes must come
from a fresh child `torch.distributed.run`, started before anything touches
the GPU (CPU only: the child command is captured, never run)."""
import subprocess
import sys
import types
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _args(gpus, workload="jacobi3d_1024"):
    return types.SimpleNamespace(gpus=gpus, workload=workload)


def test_child_argv_is_torchrun_with_the_same_arguments():
    seen = {}

    def fake_run(cmd, env=None):
        import torch
        seen["cmd"], seen["env"] = cmd, env
        # nothing on the GPU before the ranks start (no HIP context in the parent)
        seen["initialised"] = torch.cuda.is_initialized()
        return subprocess.CompletedProcess(cmd, 7)

    argv = ["--gpus", "8", "--steps", "3", "--warmup", "1"]
    rc = bench.spawn_ranks(_args(8), argv, run=fake_run, device_count=8)
    assert rc == 7  # the child's exit code is forwarded
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") and int(c.split("=")[1]) > 0 for c in cmd)
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == argv
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert seen["initialised"] is False


def test_refuses_when_too_few_devices():
    with pytest.raises(SystemExit, match="only 2 GPU"):
        bench.spawn_ranks(_args(4), ["--gpus", "4"], run=lambda *a, **k: None, device_count=2)


def test_refuses_single_gpu_workloads():
    with pytest.raises(SystemExit, match="single-GPU"):
        bench.spawn_ranks(_args(2, "cavity2d_128"), [], run=lambda *a, **k: None, device_count=8)


def test_main_spawns_only_without_world_size(monkeypatch):
    calls = []
    monkeypatch.setattr(bench, "spawn_ranks", lambda a, argv: calls.append(argv) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [["--gpus", "2", "--steps", "1"]]
