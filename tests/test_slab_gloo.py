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


def _worker(rank, world, port, nz, ny, nx, iters, ghost, out_dir):
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
        p = Plan(nz, world, rank, ghost)
        dloc = p.scatter(div)
        phi = np.zeros_like(dloc)
        zb, ze = p.z_update_begin, p.z_update_end
        fixed_lo, fixed_hi = p.z_lo == 0, p.z_hi == nz

        def sweep(a, lo, hi):
            # one sweep of planes [lo, hi): the oracle on the sub-block with
            # planes lo-1 and hi held
            out = a.copy()
            if hi > lo:
                out[lo - 1:hi + 1] = oracle.jacobi3d(dloc[lo - 1:hi + 1], a[lo - 1:hi + 1], h=0.05,
                                                     dt=np.float32(2e-3), iters=1)
            return out

        done = 0
        while done < iters:
            # a fused pass of k = min(ghost, remaining) levels (as
            # cfd_slab_jacobi3d_f32): level j on the owned range widened by
            # k - j inner ghost planes (never past a global Dirichlet plane)
            k = min(ghost, iters - done)
            lev = phi
            for j in range(1, k + 1):
                w = k - j
                lev = sweep(lev, zb if fixed_lo else zb - w, ze if fixed_hi else ze + w)
            new = phi.copy()
            new[zb:ze] = lev[zb:ze]
            done += k
            reqs, bufs = [], []
            for first, count, peer, _ in p.exchanges():
                reqs.append(dist.isend(torch.from_numpy(new[first:first + count].copy()), dst=peer))
            for first, count, peer in p.receives():
                t = torch.empty((count, ny, nx), dtype=torch.float32)
                reqs.append(dist.irecv(t, src=peer))
                bufs.append((first, count, t))
            for r in reqs:
                r.wait()
            for first, count, t in bufs:
                new[first:first + count] = t.numpy()
            phi = new
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), phi[p.owned()])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,ghost,iters", [(2, 17, 1, 5), (3, 20, 1, 5), (2, 17, 2, 6),
                                                  (3, 21, 2, 7), (3, 8, 2, 4), (2, 19, 3, 8),
                                                  (3, 22, 4, 9), (3, 12, 4, 6)])
def test_slab_decomposition_gloo_bitexact(tmp_path, world, nz, ghost, iters):
    import oracle
    ny, nx = 9, 12
    mp.spawn(_worker, args=(world, _free_port(), nz, ny, nx, iters, ghost, str(tmp_path)), nprocs=world,
             join=True)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    rng = np.random.default_rng(42)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(2e-3), iters=iters)
    assert np.array_equal(got, ref)


def _colour_pass(phi, div, c, lo, hi, zoff, k):
    """Red-black colour c over local planes [lo, hi) with GLOBAL parity
    (zoff = global index of local plane 0), numpy float32: the cells of one
    colour only read the other colour, so the vectorised pass equals the
    serial one.  Returns (new phi, max|change|)."""
    cx, cy, cz, cd, dt_inv = k
    out = phi.copy()
    if hi <= lo:
        return out, np.float32(0)
    z = np.arange(lo, hi)[:, None, None] + zoff
    y = np.arange(1, phi.shape[1] - 1)[None, :, None]
    x = np.arange(1, phi.shape[2] - 1)[None, None, :]
    sel = ((z + y + x + 1 + c) % 2) == 0
    C = phi[lo:hi, 1:-1, 1:-1]
    rhs = -div[lo:hi, 1:-1, 1:-1] * dt_inv
    a = cx * (phi[lo:hi, 1:-1, 2:] + phi[lo:hi, 1:-1, :-2])
    b = cy * (phi[lo:hi, 2:, 1:-1] + phi[lo:hi, :-2, 1:-1])
    e = cz * (phi[lo + 1:hi + 1, 1:-1, 1:-1] + phi[lo - 1:hi - 1, 1:-1, 1:-1])
    new = (((a + b) + e) - rhs) * cd
    out[lo:hi, 1:-1, 1:-1] = np.where(sel, new, C)
    ch = np.abs(new - C)[sel]
    return out, (ch.max() if ch.size else np.float32(0))


def _rbgs_worker(rank, world, port, nz, ny, nx, iters, tol, ghost, out_dir):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    import _pkgpath
    _pkgpath.load()
    from cfd_simulations_amd.slab import SlabPlan as Plan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dx, dy, dz, dt = 0.05, 0.06, 0.07, np.float32(1e-2)
        # constants as cfd_rbgs3d_f32 / the oracle round them (v5.py:205-210)
        i2 = (1.0 / dx ** 2, 1.0 / dy ** 2, 1.0 / dz ** 2)
        k = tuple(np.float32(v) for v in i2) + (np.float32(1.0 / (2.0 * sum(i2))),
                                                np.float32(1.0) / dt)
        rng = np.random.default_rng(21)
        div = rng.standard_normal((nz, ny, nx)).astype(np.float32) * np.float32(1e-3)
        p = Plan(nz, world, rank, ghost)
        dloc = p.scatter(div)
        phi = np.zeros_like(dloc)
        zb, ze, zoff = p.z_update_begin, p.z_update_end, p.z_lo - ghost
        fixed_lo, fixed_hi = int(p.z_lo == 0), int(p.z_hi == nz)

        def exchange(a):
            reqs, bufs = [], []
            for first, count, peer, _ in p.exchanges():
                reqs.append(dist.isend(torch.from_numpy(a[first:first + count].copy()), dst=peer))
            for first, count, peer in p.receives():
                t = torch.empty((count, ny, nx), dtype=torch.float32)
                reqs.append(dist.irecv(t, src=peer))
                bufs.append((first, count, t))
            for r in reqs:
                r.wait()
            for first, count, t in bufs:
                a[first:first + count] = t.numpy()

        done = iters
        for it in range(iters):
            if ghost == 2:
                # the fused pass: colour 0 also on the inner ghost planes
                # (recomputed, as cfd_rbgs3d_pass_f32 does), colour 1 on the
                # owned planes, then one 2-plane exchange
                l1, m0 = _colour_pass(phi, dloc, 0, zb - 1 + fixed_lo, ze + 1 - fixed_hi, zoff, k)
                l1o, m0o = _colour_pass(phi, dloc, 0, zb, ze, zoff, k)  # owned part of the max
                l2, m1 = _colour_pass(l1, dloc, 1, zb, ze, zoff, k)
                phi = phi.copy()
                phi[zb:ze] = l2[zb:ze]
                exchange(phi)
                m = max(m0o, m1)
            else:
                phi, m0 = _colour_pass(phi, dloc, 0, zb, ze, zoff, k)
                exchange(phi)
                phi, m1 = _colour_pass(phi, dloc, 1, zb, ze, zoff, k)
                exchange(phi)
                m = max(m0, m1)
            t = torch.tensor([float(m)], dtype=torch.float32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the per-iteration ncclAllReduce(max)
            if t.item() < tol:
                done = it + 1
                break
        np.save(os.path.join(out_dir, f"rank{rank}.npy"), phi[p.owned()])
        np.save(os.path.join(out_dir, f"done{rank}.npy"), np.array([done]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nz,ghost,iters,tol", [(2, 17, 1, 6, 0.0), (3, 20, 2, 7, 0.0),
                                                      (2, 18, 2, 300, 2e-5), (3, 19, 1, 300, 2e-5)])
def test_slab_rbgs_gloo_bitexact(tmp_path, world, nz, ghost, iters, tol):
    """Distributed red-black GS: global colours + a global max per iteration
    reproduce the single-domain oracle bit-for-bit, stop iteration included."""
    import oracle
    ny, nx = 10, 12
    mp.spawn(_rbgs_worker, args=(world, _free_port(), nz, ny, nx, iters, tol, ghost, str(tmp_path)),
             nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    dones = {int(np.load(tmp_path / f"done{r}.npy")[0]) for r in range(world)}
    rng = np.random.default_rng(21)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=0.05, dy=0.06, dz=0.07, dt=np.float32(1e-2), iters=iters, tol=tol)
    assert dones == {n_ref}
    if tol > 0:
        assert 1 < n_ref < iters
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ghost", [1, 2, 3, 4])
def test_slab_plan_partition(ghost):
    for nz in (7, 64, 1024):
        for R in (1, 2, 3, 4, 8):
            if nz < R * ghost:
                continue
            plans = [SlabPlan(nz, R, r, ghost) for r in range(R)]
            assert plans[0].z_lo == 0 and plans[-1].z_hi == nz
            for a, b in zip(plans, plans[1:]):
                assert a.z_hi == b.z_lo
            sizes = [p.nz_local for p in plans]
            assert max(sizes) - min(sizes) <= 1
            # update ranges cover exactly the interior planes 1..nz-2
            upd = []
            for p in plans:
                upd += [p.z_lo - ghost + k for k in range(p.z_update_begin, p.z_update_end)]
            assert upd == list(range(1, nz - 1))
            # each send lands in the peer's matching ghost planes
            for p in plans:
                for first, count, peer, recv in p.exchanges():
                    q = plans[peer]
                    assert count == ghost
                    assert p.z_lo - ghost + first == q.z_lo - ghost + recv
                    assert (recv, count, p.rank) in q.receives()
                    # the sent planes are owned by p
                    assert p.owned().start <= first and first + count <= p.owned().stop


def test_slab_plan_1024_on_8():
    p = SlabPlan(1024, 8, 3)
    assert (p.z_lo, p.z_hi, p.nz_local) == (384, 512, 128)
    assert p.exchanges() == [(1, 1, 2, 129), (128, 1, 4, 0)]
    assert p.receives() == [(0, 1, 2), (129, 1, 4)]
    assert (p.z_update_begin, p.z_update_end) == (1, 129)
    p0 = SlabPlan(1024, 8, 0)
    assert (p0.z_update_begin, p0.z_update_end, p0.lo_peer) == (2, 129, -1)
    p7 = SlabPlan(1024, 8, 7)
    assert (p7.z_update_begin, p7.z_update_end, p7.hi_peer) == (1, 128, -1)
    q = SlabPlan(1024, 8, 3, ghost=2)
    assert q.nz_total == 132 and q.owned() == slice(2, 130)
    assert q.exchanges() == [(2, 2, 2, 130), (128, 2, 4, 0)]
    assert q.receives() == [(0, 2, 2), (130, 2, 4)]
    q0 = SlabPlan(1024, 8, 0, ghost=2)
    assert (q0.z_update_begin, q0.z_update_end) == (3, 130)
