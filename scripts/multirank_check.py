#!/usr/bin/env python3
"""Multi-rank RCCL slab check on whatever GPUs are present.

    python -m torch.distributed.run --nproc-per-node R --master-addr 127.0.0.1 \
        --master-port 29533 scripts/multirank_check.py [--share-gpu]

Every rank solves its slab with cfd_slab_jacobi3d_f32 (RCCL halo exchange,
overlap on and off, 1- and 2-deep ghosts).  Rank 0 gathers the owned planes
over gloo and compares them bitwise with the CPU oracle's single-domain solve.
With --share-gpu all ranks use device 0 (a rehearsal on a one-GPU box, if
RCCL accepts several ranks on one device).
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
    ap.add_argument("--n", type=int, default=64)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(0 if a.share_gpu else local)
    dist.init_process_group("gloo")
    n = a.n
    nz, ny, nx = n, n - 6, n + 8
    rng = np.random.default_rng(77)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    comm = S.RcclComm(rank, world)
    ok = True
    try:
        for ghost in (1, 2, 3, 4):
            for overlap in (False, True):
                for iters in (6, 7):
                    plan = S.SlabPlan(nz, world, rank, ghost=ghost)
                    sj = S.SlabJacobi3D(plan, ny, nx, 0.05, np.float32(1e-3), comm)
                    sj.div.copy_(torch.from_numpy(plan.scatter(div)).cuda())
                    sj.solve(iters, overlap=overlap)
                    torch.cuda.synchronize()
                    mine = torch.from_numpy(sj.owned().cpu().numpy().copy())
                    parts = [torch.empty((S.SlabPlan(nz, world, r, ghost).nz_local, ny, nx)) for r in range(world)]
                    dist.all_gather(parts, mine)
                    if rank == 0:
                        got = torch.cat(parts).numpy()
                        ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(1e-3), iters=iters)
                        same = np.array_equal(got, ref)
                        ok &= same
                        print(f"world={world} ghost={ghost} overlap={overlap} iters={iters}: "
                              f"{'bit-exact' if same else 'MISMATCH'}", flush=True)
    finally:
        comm.close()
        dist.destroy_process_group()
    if rank == 0:
        print("MULTIRANK", "OK" if ok else "FAIL", flush=True)
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
