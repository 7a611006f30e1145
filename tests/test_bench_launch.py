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


def test_shared_gpu_needs_one_device_and_copy_engines():
    seen = {}

    def fake_run(cmd, env=None):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 0)

    a = types.SimpleNamespace(gpus=2, workload="jacobi3d_512", shared_gpu=True, transport="ce")
    argv = ["--gpus", "2", "--shared-gpu", "--workload", "jacobi3d_512"]
    assert bench.spawn_ranks(a, argv, run=fake_run, device_count=1) == 0
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-len(argv):] == argv
    a.transport = "rccl"
    with pytest.raises(SystemExit, match="copy-engine"):
        bench.spawn_ranks(a, argv, run=fake_run, device_count=1)


def _gather_worker(rank, world, port, sizes, q):
    import os
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        mine = torch.full((sizes[rank], 3, 4), float(rank + 1))
        parts = [torch.empty((n, 3, 4)) for n in sizes]
        got = bench.gather_planes(dist, parts, mine, rank, dev)
        t = torch.tensor([float(rank), 2.0 * rank], dtype=torch.float64, device=bench.coll_device(dist, dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put((rank, [float(p.mean()) for p in got], [p.shape[0] for p in got], t.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [(3, 3), (4, 3, 3)])
def test_gather_planes_on_gloo(sizes):
    """The collectives of bench.py's N-rank path (verify_slabs' gathers of the
    owned planes, equal and uneven counts, and the timing max) on gloo, as the
    --shared-gpu rehearsal runs them."""
    import torch.multiprocessing as mp
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench._free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, list(sizes), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, means, counts, tmax in res:
        assert means == [float(r + 1) for r in range(world)]
        assert counts == list(sizes)
        assert tmax == [float(world - 1), 2.0 * (world - 1)]
