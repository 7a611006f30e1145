#!/usr/bin/env python3
"""Rehearsal of the N-rank slab solve on ONE GPU (N host threads, the
in-process slab group of cfd_comm_init_local): every rank runs the real
cfd_slab_jacobi3d_f32 / cfd_slab_rbgs3d_f32 driver on its share of the grid,
with device copies in place of the RCCL send/recv pairs.

All ranks share one GPU, so the aggregate rate printed here is the decomposed
job's *compute* efficiency (ghost recompute, boundary-first launches, launch
gaps) relative to the single-domain solve, without the xGMI links:
    predicted N-GPU rate ~ N x (aggregate rate here) when the exchange hides.

    python scripts/slab_rehearsal.py [--ranks 8] [--workload jacobi|rbgs] [--n 1024]

--rccl-self (alias --self) instead times ONE middle rank of an R-rank job in
isolation: a one-rank comm peered with itself, so the pass sequence is the
real one (boundary planes, the exchange beside the interior launch, the GS
max-reduce) with local copies for the xGMI transfers.  --transport ce (the
default): the copy engines write the boundary planes into the rank's own
ghost planes at ~58 GB/s per direction (about one xGMI link's rate) and the
sync kernel waits for them; --transport rccl: RCCL send/recv kernels on the
reserved CUs.  Its result is not a solve (timing only).
"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402

_pkgpath.load()
from cfd_simulations_amd import slab as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--workload", default="jacobi", choices=["jacobi", "rbgs"])
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--nz", type=int, default=0)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--rccl-self", "--self", dest="rccl_self", action="store_true")
    ap.add_argument("--transport", default="ce", choices=["ce", "rccl"])
    ap.add_argument("--comm-priority", type=int, default=1, help="1: high-priority comm stream")
    ap.add_argument("--prefetch", type=int, default=0, help="cfd_set_jacobi3d_prefetch (0 auto, 1 DMA, 2 regs)")
    ap.add_argument("--ghost", type=int, default=0, help="Jacobi ghost planes (0: the sweeps per pass)")
    ap.add_argument("--tb", type=int, default=0,
                    help="--self red-black GS: 0 or 4 = two iterations per pass (4-deep ghosts), 2 = one")
    a = ap.parse_args()
    if a.rccl_self:
        return rccl_self(a)
    R, n = a.ranks, a.n
    nz = a.nz or n
    dev = torch.device("cuda", 0)
    gs = a.workload == "rbgs"
    h = 1.0 / (n - 1)
    dt = np.float32(5e-5)
    comms = S.LocalComm.group(R)
    sol = []
    for r in range(R):
        plan = S.SlabPlan(nz, R, r, ghost=2 if gs else 3)
        if gs:
            s = S.SlabRBGS3D(plan, n, n, h, h, h, dt, comms[r], device=dev)
        else:
            s = S.SlabJacobi3D(plan, n, n, h, dt, comms[r], device=dev)
        g = torch.Generator(device=dev).manual_seed(1234 + r)
        s.div.copy_(torch.randn(s.div.shape, generator=g, device=dev))
        sol.append(s)
    streams = [torch.cuda.Stream(device=dev) for _ in range(R)]
    torch.cuda.synchronize()
    bar = threading.Barrier(R)
    times = [0.0] * R
    errs = [None] * R

    def work(r):
        try:
            with torch.cuda.stream(streams[r]):
                for step in range(a.steps + 1):  # first step is the warm-up
                    bar.wait()
                    t0 = time.perf_counter()
                    if gs:
                        sol[r].solve(a.iters, tolerance=1e-8, overlap=not a.no_overlap)
                    else:
                        sol[r].solve(a.iters, overlap=not a.no_overlap)
                    streams[r].synchronize()
                    bar.wait()
                    if step:
                        times[r] += time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e
            bar.abort()

    th = [threading.Thread(target=work, args=(r,)) for r in range(R)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    torch.cuda.synchronize()
    for c in comms:
        c.close()
    if any(errs):
        raise SystemExit(f"rank errors: {errs}")
    t = max(times) / a.steps
    cells = (nz - 2) * (n - 2) * (n - 2) * a.iters
    print(json.dumps({"workload": a.workload, "ranks_on_one_gpu": R, "grid": [nz, n, n], "iters": a.iters,
                      "overlap": not a.no_overlap, "ms_per_solve": round(t * 1e3, 3),
                      "aggregate_gcells": round(cells / t / 1e9, 1)}))


def rccl_self(a):
    from cfd_simulations_amd._lib import call, lib, ptr
    dev = torch.device("cuda", 0)
    n, R = a.n, a.ranks
    nz = a.nz or n
    gs = a.workload == "rbgs"
    if a.tb:
        call("cfd_set_jacobi3d_blocking", a.tb, 0, 0)  # GS: rbgs3d_iters_per_pass(): 2 at 4, else 1
    # Jacobi: ghosts as deep as the sweeps per pass (bench.py's plan at N > 1;
    # --ghost overrides, and a pass then fuses min(levels, ghost) sweeps)
    G = (4 if a.tb in (0, 4) else 2) if gs else (a.ghost or int(lib().cfd_get_jacobi3d_levels()))
    nzl = nz // R
    shape = (nzl + 2 * G, n, n)
    h = 1.0 / (n - 1)
    dt = np.float32(5e-5)
    comm = S.make_comm(0, 1, a.transport)
    call("cfd_set_jacobi3d_prefetch", a.prefetch)
    g = torch.Generator(device=dev).manual_seed(1234)
    div = torch.randn(shape, generator=g, device=dev) * 1e-3
    phi, tmp = torch.zeros_like(div), torch.zeros_like(div)
    rhs = torch.empty_like(div)
    if a.transport == "ce":
        comm.attach(phi, tmp)
    cs = torch.cuda.Stream(device=dev, priority=-1 if a.comm_priority else 0)
    ws = torch.empty(int(lib().cfd_rbgs_workspace_bytes(a.iters)), dtype=torch.uint8, device=dev)
    done = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def solve():
        if gs:
            phi.zero_()
            call("cfd_slab_rbgs3d_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), None, nzl, G, n, n, 0, 0,
                 G, nzl + G, 100, h, h, h, float(dt), a.iters, 1e-30, ptr(ws), ptr(done),
                 int(not a.no_overlap), s, cs.cuda_stream)
        else:
            # phi = zeros inside the solve, as SlabJacobi3D.solve does
            call("cfd_slab_jacobi3d_zero_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), ptr(rhs), nzl, G,
                 n, n, 0, 0, G, nzl + G, h, float(dt), a.iters, int(not a.no_overlap), s, cs.cuda_stream)

    solve()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        solve()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / a.steps
    if a.transport == "ce":
        comm.status()  # raises if a sync kernel timed out
    comm.close()
    cells = nzl * (n - 2) * (n - 2) * a.iters
    print(json.dumps({"workload": a.workload, "mode": f"{a.transport}-self (one middle rank of R)", "ranks": R,
                      "grid": [nz, n, n], "nz_local": nzl, "ghost": G, "iters": a.iters,
                      "overlap": not a.no_overlap, "prefetch": a.prefetch,
                      "comm_priority": a.comm_priority, "ms_per_solve": round(t * 1e3, 3),
                      "rank_gcells": round(cells / t / 1e9, 1),
                      "predicted_job_gcells": round(R * cells / t / 1e9, 1)}))


if __name__ == "__main__":
    main()
