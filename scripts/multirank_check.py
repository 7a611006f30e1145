#!/usr/bin/env python3
"""Multi-rank slab check on whatever GPUs are present.

    python -m torch.distributed.run --nproc-per-node R --master-addr 127.0.0.1 \
        --master-port 29533 scripts/multirank_check.py [--share-gpu] [--transport ce|rccl]

Every rank solves its slab with cfd_slab_jacobi3d_f32 / _zero_f32 and
cfd_slab_rbgs3d_f32 (overlap on and off, 1- to 4-deep ghosts, early GS stops)
over the chosen transport: copy engines (IPC-mapped neighbour buffers, the
default) or RCCL.  Rank 0 gathers the owned planes over gloo and compares them
bitwise with the CPU oracle's single-domain solve.  With --share-gpu all ranks
use device 0: separate processes on one GPU, which the copy-engine transport
supports (RCCL refuses several ranks on one device).
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402

_pkgpath.load()
import oracle  # noqa: E402
from cfd_simulations_amd import slab as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share-gpu", action="store_true")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--transport", default="ce", choices=["ce", "rccl"])
    ap.add_argument("--quick", action="store_true", help="fewer cases")
    ap.add_argument("--repeat", type=int, default=1, help="run the whole case list this many times")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(0 if a.share_gpu else local)
    dist.init_process_group("gloo")
    n = a.size
    nz, ny, nx = n, n - 6, n + 8
    rng = np.random.default_rng(77)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    comm = S.make_comm(rank, world, a.transport)
    ok = True

    def gather(owned, planes):
        mine = torch.from_numpy(owned.cpu().numpy().copy())
        parts = [torch.empty((p, ny, nx)) for p in planes]
        dist.all_gather(parts, mine)
        return torch.cat(parts).numpy()

    def report(tag, same):
        nonlocal ok
        ok &= same
        if rank == 0:
            print(f"world={world} {a.transport} {tag}: {'bit-exact' if same else 'MISMATCH'}", flush=True)

    try:
        for _ in range(a.repeat):
            run_cases(a, S, comm, rank, world, nz, ny, nx, div, rng, gather, report)
        if hasattr(comm, "status"):
            comm.status()
    finally:
        comm.close()
        dist.destroy_process_group()
    if rank == 0:
        print("MULTIRANK", "OK" if ok else "FAIL", flush=True)
        sys.exit(0 if ok else 1)


def run_cases(a, S, comm, rank, world, nz, ny, nx, div, rng, gather, report):
    if True:
        ghosts = (1, 3) if a.quick else (1, 2, 3, 4)
        for ghost in ghosts:
            planes = [S.SlabPlan(nz, world, r, ghost).nz_local for r in range(world)]
            for overlap in (False, True):
                for iters in (6, 7):
                    for zero in (False, True):
                        plan = S.SlabPlan(nz, world, rank, ghost=ghost)
                        sj = S.SlabJacobi3D(plan, ny, nx, 0.05, np.float32(1e-3), comm)
                        sj.div.copy_(torch.from_numpy(plan.scatter(div)).cuda())
                        if not zero:  # a nonzero start: the general driver with the initial exchange
                            sj.phi.fill_(0.0)
                        sj.solve(iters, overlap=overlap, zero_phi=zero)
                        torch.cuda.synchronize()
                        got = gather(sj.owned(), planes)
                        if rank == 0:
                            ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(1e-3), iters=iters)
                            same = np.array_equal(got, ref)
                        else:
                            same = True
                        report(f"jacobi ghost={ghost} overlap={overlap} iters={iters} zero={zero}", same)
        # red-black GS: global colours, the global stop rule
        gdiv = (rng.standard_normal((nz, ny, nx)) * 1e-3).astype(np.float32)
        gcases = [(2, 0.0, 9), (4, 2e-5, 300)] if a.quick else \
            [(1, 0.0, 9), (2, 0.0, 9), (2, 2e-5, 300), (4, 0.0, 9), (4, 2e-5, 300), (4, 1.5e-5, 300)]
        for ghost, tol, iters in gcases:
            planes = [S.SlabPlan(nz, world, r, ghost).nz_local for r in range(world)]
            for overlap in (False, True):
                plan = S.SlabPlan(nz, world, rank, ghost=ghost)
                sg = S.SlabRBGS3D(plan, ny, nx, 0.05, 0.05, 0.05, np.float32(1e-2), comm)
                sg.div.copy_(torch.from_numpy(plan.scatter(gdiv)).cuda())
                sg.solve(iters, tolerance=tol, overlap=overlap)
                torch.cuda.synchronize()
                cnt = int(sg.iters_done.cpu()[0])
                got = gather(sg.owned(), planes)
                counts = [None] * world
                dist.all_gather_object(counts, cnt)
                if rank == 0:
                    ref, n_ref = oracle.rbgs3d(gdiv, dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2),
                                               iters=iters, tol=tol)
                    same = np.array_equal(got, ref) and counts == [n_ref] * world
                else:
                    same = True
                report(f"rbgs ghost={ghost} overlap={overlap} tol={tol} iters={iters} count={cnt}", same)


if __name__ == "__main__":
    main()
