"""Multi-rank slab decomposition on CPU (gloo, world_size 2 and 3).

Each rank owns SlabPlan(nz, R, rank)'s planes plus ghosts, sweeps its update
range with the CPU oracle (the checker stands in for the GPU sweep), and swaps
ghost planes with torch.distributed send/recv in exactly the pattern the RCCL
driver (cfd_slab_jacobi3d_f32) uses: SlabPlan.exchanges() / receives().  The
gathered result must be bit-identical to the single-domain solve.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgpath  # noqa: E402  (spawned ranks re-import this module)

_pkgpath.load()
from cfd_simulations_amd.slab import SlabPlan  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, nz, ny, nx, iters, out_dir):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    import _pkgpath
    _pkgpath.load()
    import oracle
    from cfd_simulations_amd.slab import SlabPlan as Plan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(42)
        div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
        p = Plan(nz, world, rank)
        dloc = p.scatter(div)
        phi = np.zeros_like(dloc)
        zb, ze = p.z_update_begin, p.z_update_end
        for _ in range(iters):
            new = phi.copy()
            if ze > zb:
                # one sweep of planes [zb, ze): the oracle on the sub-block with
                # planes zb-1 and ze as held boundaries
                new[zb - 1:ze + 1] = oracle.jacobi3d(dloc[zb - 1:ze + 1], phi[zb - 1:ze + 1], h=0.05,
                                                     dt=np.float32(2e-3), iters=1)
            reqs = []
            for send_plane, peer, _ in p.exchanges():
                reqs.append(dist.isend(torch.from_numpy(new[send_plane].copy()), dst=peer))
            bufs = []
            for ghost, peer in p.receives():
                t = torch.empty((ny, nx), dtype=torch.float32)
                reqs.append(dist.irecv(t, src=peer))
                bufs.append((ghost, t))
            for r in reqs:
                r.wait()
            for ghost, t in bufs:
                new[ghost] = t.numpy()
            phi = new
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), phi[1:p.nz_local + 1])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz", [(2, 17), (3, 20)])
def test_slab_decomposition_gloo_bitexact(tmp_path, world, nz):
    import oracle
    ny, nx, iters = 9, 12, 5
    mp.spawn(_worker, args=(world, _free_port(), nz, ny, nx, iters, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    rng = np.random.default_rng(42)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(2e-3), iters=iters)
    assert np.array_equal(got, ref)


def test_slab_plan_partition():
    for nz in (7, 64, 1024):
        for R in (1, 2, 3, 4, 8):
            if nz < R:
                continue
            plans = [SlabPlan(nz, R, r) for r in range(R)]
            assert plans[0].z_lo == 0 and plans[-1].z_hi == nz
            for a, b in zip(plans, plans[1:]):
                assert a.z_hi == b.z_lo
            sizes = [p.nz_local for p in plans]
            assert max(sizes) - min(sizes) <= 1
            # update ranges cover exactly the interior planes 1..nz-2
            upd = []
            for p in plans:
                upd += [p.z_lo - 1 + k for k in range(p.z_update_begin, p.z_update_end)]
            assert upd == list(range(1, nz - 1))
            # each send lands in the peer's matching ghost
            for p in plans:
                for send, peer, recv in p.exchanges():
                    q = plans[peer]
                    assert p.z_lo - 1 + send == q.z_lo - 1 + recv
                    assert (recv, p.rank) in q.receives()


def test_slab_plan_1024_on_8():
    p = SlabPlan(1024, 8, 3)
    assert (p.z_lo, p.z_hi, p.nz_local) == (384, 512, 128)
    assert p.exchanges() == [(1, 2, 129), (128, 4, 0)]
    assert p.receives() == [(0, 2), (129, 4)]
    assert (p.z_update_begin, p.z_update_end) == (1, 129)
    p0 = SlabPlan(1024, 8, 0)
    assert (p0.z_update_begin, p0.z_update_end, p0.lo_peer) == (2, 129, -1)
    p7 = SlabPlan(1024, 8, 7)
    assert (p7.z_update_begin, p7.z_update_end, p7.hi_peer) == (1, 128, -1)
