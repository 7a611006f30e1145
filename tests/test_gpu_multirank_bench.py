"""bench.py's N-rank path, end to end, on a one-GPU lease (--shared-gpu).

`python bench.py --gpus 2 --shared-gpu ...` runs as a fresh child process: it
spawns its two ranks (torch.distributed.run), puts both on device 0, joins a
gloo process group, attaches the copy-engine transport (IPC-mapped neighbour
ghosts, the N-GPU default), runs verify_slabs / verify_slabs_rbgs against the
single-GPU solve, the timed slab solves, the max-over-ranks timing and rank
0's JSON line: exactly the code the driver's `bench.py --gpus 8` runs, minus
RCCL (which refuses two ranks on one device).  The timing is meaningless on a
shared device; the parity flag and the line's shape are what is checked.
Reference: the Jacobi branch v5.py:336-346 (slab-decomposed) and
the red-black GS v5.py:202-226 in 3-D (BASELINE configs 4-5)."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.gpu


def _run(args, timeout=420):
    cmd = [sys.executable, "-u", str(ROOT / "bench.py"), "--gpus", "2", "--shared-gpu", "--no-cpu-baseline"] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=str(ROOT))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-6000:]
    return json.loads(lines[0]), out


@pytest.mark.timeout(480)
def test_bench_two_ranks_shared_gpu_jacobi():
    d, out = _run(["--workload", "jacobi3d_512", "--steps", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["steps"] == 2
    assert d["config"]["halo"].startswith("copy engines"), d["config"]
    assert d["config"]["multi_gpu_parity"].startswith("bit-exact"), (d["config"], out[-3000:])
    assert "shared_gpu" in d["config"]
    assert d["value"] > 0 and d["roofline"]["avg_launch_ms"] > 0


@pytest.mark.timeout(480)
def test_bench_two_ranks_shared_gpu_jacobi_1024():
    """The default workload at two ranks: 2.2 GB slab arrays, past what
    hipIpcOpenMemHandle maps (2 GiB; it never returned, r06), so the ghosts
    arrive through the ranks' landing buffers."""
    d, out = _run(["--steps", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2 and d["config"]["grid"] == [1024, 1024, 1024]
    assert d["config"]["halo"].startswith("copy engines"), d["config"]
    assert d["config"]["multi_gpu_parity"].startswith("bit-exact"), (d["config"], out[-3000:])


@pytest.mark.timeout(480)
def test_bench_two_ranks_shared_gpu_rbgs():
    d, out = _run(["--workload", "rbgs3d_1024", "--grid", "128,128,128", "--steps", "2", "--warmup", "1"])
    assert d["n_gpus"] == 2
    assert d["config"]["grid"] == [128, 128, 128]
    assert d["config"]["halo"].startswith("copy engines"), d["config"]
    assert d["config"]["multi_gpu_parity"].startswith("bit-exact"), (d["config"], out[-3000:])
    assert d["config"]["iterations_done_last_step"] >= 1
