#!/usr/bin/env python3
"""Benchmark: Gcell-updates/s of the pressure-Poisson solve on MI355X.

Default workload (north_star, BASELINE.json): 7-point Jacobi on a 1024^3 fp32
grid, one "step" = one pressure solve = zero-fill phi + ITERS (200) Jacobi
sweeps, inputs resident in HBM.  N GPUs: z-slab decomposition with the halo
exchange overlapped with the interior pass -- copy engines writing into the
neighbours' IPC-mapped ghost planes (default; --transport rccl: RCCL
send/recv); strong scaling (the grid is fixed, each rank owns 1024/N planes).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts
the N ranks itself: a child `torch.distributed.run --nproc-per-node N` of the
same arguments, launched before anything touches the GPU; its exit code is
forwarded (spawn_ranks).

Rank 0 prints ONE JSON line.  `value` = all ranks' interior cell-updates / the
max-over-ranks wall time of the K timed steps.  `roofline` prices one launch
of the dominant kernel -- a temporally blocked pass that fuses several sweeps
-- at the 12 algorithmic bytes per fp32 cell (24 per fp64) the pass moves
(read phi, read rhs, write phi'), using HIP events recorded on the solve's own
stream around its launches.  `cpu_baseline` times the NumPy restatement of the
reference's Jacobi branch (oracle/, bit-exact to v5.py:336-346) on a bounded
sample of the same grid, on this host, at N=1 only.

`--workload cavity2d_128` is config 1: the whole projection step of the
lid-driven cavity (128^2, Re = 100, 500 Jacobi sweeps per pressure solve) per
step; `value` counts the pressure cell-updates over the step's wall time, and
the CPU baseline is the same step on the host (oracle.OracleCavitySolver with
the reference's NumPy Jacobi form).

`--workload rbgs3d_1024` is config 5: red-black Gauss-Seidel (the 3-D
generalisation of v5.py:202-226) on the 1024^3 grid, one step = zero-fill +
200 iterations at the reference's tolerance 1e-8 (stop rule evaluated on device
every iteration; one cell-update per cell per iteration).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Gcell-updates/s on pressure-Poisson Jacobi; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (shape, dtype, iters per step, bytes per cell-update)
    "jacobi3d_1024": ((1024, 1024, 1024), "f32", 200, 12),
    "jacobi3d_512": ((512, 512, 512), "f32", 200, 12),
    # config 4: 1024 (x) x 1024 (y) x 512 (z) channel, z-slabs (64 planes per GPU at N=8)
    "jacobi3d_channel": ((512, 1024, 1024), "f32", 200, 12),
    "jacobi2d_8192_f64": ((8192, 8192), "f64", 1000, 24),
    "rbgs3d_1024": ((1024, 1024, 1024), "f32", 200, 12),
    # config 1: lid-driven cavity 128^2, Re = 100, 500 Jacobi sweeps per pressure
    # solve; one step = one LidDrivenCavitySolver.time_step() (v5.py:375-441)
    "cavity2d_128": ((128, 128), "f32", 500, 12),
    # the second north-star kernel: the fused advection-diffusion predictor
    # (v5.py:388-403, kernels :127-176) over an 8192^2 SUPG field, scalar
    # nu_eff (LES off), tau written: one step = one cfd_predictor2d call;
    # 20 B per cell (u, v read; u*, v*, tau written), 40 B in float64
    "predictor2d_8192": ((8192, 8192), "f32", 1, 20),
    "predictor2d_8192_f64": ((8192, 8192), "f64", 1, 40),
}
GS_TOL = 1e-8  # OptimizedTurbulentConfig.pressure_tolerance (v5.py)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="jacobi3d_1024", choices=sorted(WORKLOADS))
    ap.add_argument("--iters", type=int, default=0, help="Jacobi sweeps per step (0 = workload default)")
    ap.add_argument("--variant", type=int, default=0, help="3-D kernel: 0 auto, 1 LDS, 2 cache")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--zchunk", type=int, default=0)
    ap.add_argument("--tb", type=int, default=0, help="sweeps fused per HBM pass: 0 auto, 1 off, 2..4")
    ap.add_argument("--tb-rows", type=int, default=0)
    ap.add_argument("--tb-zchunk", type=int, default=0)
    ap.add_argument("--tb-prefetch", type=int, default=0, help="planes of prefetch in the blocked kernel")
    ap.add_argument("--j2-staging", type=int, default=-1,
                    help="2-D blocked Jacobi: rows staged ahead through the LDS ring (0 = register march, -1 = library default)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--transport", default="ce", choices=["ce", "rccl"],
                    help="slab halo transport: copy engines over IPC (default) or RCCL send/recv")
    ap.add_argument("--shared-gpu", action="store_true",
                    help="rehearsal of the N-rank path on ONE GPU: every rank on device 0, a gloo "
                         "process group, the copy-engine transport (timing is not a scaling number)")
    ap.add_argument("--grid", default="",
                    help="3-D workloads: override the grid as NZ,NY,NX (e.g. a small rbgs3d rehearsal)")
    ap.add_argument("--no-rhs-ws", action="store_true", help="form the RHS in-register every sweep")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="skip the N>1 parity check")
    ap.add_argument("--force-slab", action="store_true",
                    help="use the RCCL slab path even on one rank (launch under torch.distributed.run)")
    ap.add_argument("--cpu-sample-planes", type=int, default=256)
    ap.add_argument("--sweep-tiles", action="store_true", help="print a tile-size sweep (N=1, 3-D)")
    ap.add_argument("--tau-mode", default="exact", choices=["exact", "fast"],
                    help="predictor workloads: SUPG tau arithmetic (exact: bit-exact glibc powf/pow; "
                         "fast: the compiled reference's fastmath form)")
    return ap.parse_args()


def load_traffic(workload: str, n_gpus: int):
    """HBM bytes per sweep launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950
    correction), or None when no matching profile is committed."""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        e = d.get(workload)
        if e and int(e.get("n_gpus", 1)) == n_gpus:
            return float(e["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def cpu_baseline(shape, iters_total_hint, gs=False):
    """NumPy restatement timed on this host (1 thread: NumPy ufuncs); for the
    red-black GS workload the oracle's C restatement (serial, 1 thread: the
    reference's numba build is not installed here)."""
    import oracle
    if gs:
        sample = (min(shape[0], 128), shape[1], shape[2])
        rng = np.random.default_rng(1234)
        div = rng.standard_normal(sample, dtype=np.float32)
        it = 3
        h = 1.0 / (shape[2] - 1)
        t0 = time.perf_counter()
        oracle.rbgs3d(div, dx=h, dy=h, dz=h, dt=np.float32(5e-5), iters=it, tol=GS_TOL)
        t = time.perf_counter() - t0
        cells = (sample[0] - 2) * (sample[1] - 2) * (sample[2] - 2) * it
        return {"value": cells / t / 1e9, "unit": "Gcell-updates/s", "cores": 1, "kind": "port",
                "sample": f"{sample[0]}x{sample[1]}x{sample[2]} slab of the grid, {it} iterations, "
                          f"oracle_rbgs3d_f32 (C, serial red-black order); {t:.2f} s; host has "
                          f"{os.cpu_count()} logical CPUs, 1 used"}
    if len(shape) == 3:
        nz = min(shape[0], ARGS.cpu_sample_planes)
        sample = (nz, shape[1], shape[2])
        rng = np.random.default_rng(1234)
        div = rng.standard_normal(sample, dtype=np.float32)
        it = 2
        t0 = time.perf_counter()
        oracle.jacobi3d_numpy(div, h=1.0 / (shape[2] - 1), dt=np.float32(5e-5), iters=it)
        t = time.perf_counter() - t0
        cells = (sample[0] - 2) * (sample[1] - 2) * (sample[2] - 2) * it
        desc = f"{sample[0]}x{sample[1]}x{sample[2]} slab of the grid, {it} sweeps, jacobi3d_numpy"
    else:
        ny = min(shape[0], 2048)
        sample = (ny, shape[1])
        rng = np.random.default_rng(1234)
        div = rng.standard_normal(sample)
        it = 6
        t0 = time.perf_counter()
        oracle.jacobi2d_numpy(div, dx=1.0 / (shape[1] - 1), dt=np.float32(5e-5), iters=it)
        t = time.perf_counter() - t0
        cells = (sample[0] - 2) * (sample[1] - 2) * it
        desc = f"{sample[0]}x{sample[1]} rows of the grid, {it} sweeps, jacobi2d_numpy (v5.py:336-346 form)"
    return {"value": cells / t / 1e9, "unit": "Gcell-updates/s", "cores": 1, "kind": "port",
            "sample": desc + f"; {t:.2f} s; host has {os.cpu_count()} logical CPUs, NumPy uses 1"}


def cpu_baseline_all_cores(shape, gs=False):
    """The oracle's OpenMP C restatement (bit-identical to the serial one) on
    every thread OpenMP is given here: OMP_NUM_THREADS, which the GPU box sets
    to its CPU share of 16 (the host's logical CPUs -- 256 on the MI355X node --
    are shared by the node's GPU slots; os.cpu_count() reports them all).  The
    line states both numbers; `cores` is the threads actually used."""
    import oracle
    nz = min(shape[0], 256)
    sample = (nz, shape[1], shape[2])
    rng = np.random.default_rng(1234)
    div = rng.standard_normal(sample, dtype=np.float32)
    h = 1.0 / (shape[2] - 1)
    it = 4
    t0 = time.perf_counter()
    if gs:
        oracle.rbgs3d(div, dx=h, dy=h, dz=h, dt=np.float32(5e-5), iters=it, tol=GS_TOL, mt=True)
        what = "oracle_rbgs3d_f32_mt"
    else:
        oracle.jacobi3d(div, h=h, dt=np.float32(5e-5), iters=it, mt=True)
        what = "oracle_jacobi3d_f32_mt"
    t = time.perf_counter() - t0
    cells = (sample[0] - 2) * (sample[1] - 2) * (sample[2] - 2) * it
    nthr = oracle.threads()
    return {"value": cells / t / 1e9, "unit": "Gcell-updates/s", "cores": nthr, "kind": "port",
            "sample": f"{sample[0]}x{sample[1]}x{sample[2]} slab of the grid, {it} iterations, {what} (C, "
                      f"OpenMP over planes); {t:.2f} s; {nthr} threads = OMP_NUM_THREADS "
                      f"({os.environ.get('OMP_NUM_THREADS', 'unset')}: this job's CPU share) of the host's "
                      f"{os.cpu_count()} logical CPUs"}


def cavity_bench():
    """Config 1 (single GPU): LidDrivenCavitySolver.time_step() repeated; the
    pressure solve is the small-grid 2-D Jacobi kernel (4 sweeps per launch),
    latency-bound at 128^2 (a pass moves 190 KB)."""
    import torch
    import _pkgpath
    _pkgpath.load()
    import oracle
    from cfd_simulations_amd._lib import call, lib
    from cfd_simulations_amd.solver import LidDrivenCavityConfig, LidDrivenCavitySolver
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("the cavity workload (config 1) is single-GPU")
    cfg = LidDrivenCavityConfig()
    g = LidDrivenCavitySolver(cfg)
    for _ in range(ARGS.warmup):
        g.time_step()
    torch.cuda.synchronize()
    call("cfd_timing_enable", 1)
    t0 = time.perf_counter()
    for _ in range(ARGS.steps):
        g.time_step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = ctypes.c_double()
    nsw = ctypes.c_longlong()
    call("cfd_timing_read", ctypes.byref(ms), ctypes.byref(nsw), 1)
    call("cfd_timing_enable", 0)
    ny, nx = cfg.ny, cfg.nx
    cells = (ny - 2) * (nx - 2)
    iters = cfg.pressure_iterations
    # the small-grid solve is ONE persistent launch (jacobi2d_persist, r03) of
    # all the sweeps, moving the grid's 12 B per cell through HBM once; if the
    # library took the launch-per-pass path instead, it reports its depth
    spl_c = ctypes.c_int(0)
    persistent = int(lib().cfd_get_last_jacobi2d_path(ctypes.byref(spl_c))) == 1
    spl = max(int(spl_c.value), 1)
    launch_ms = ms.value / max(nsw.value, 1) * spl
    alg = cells * 12
    achieved = alg / (launch_ms * 1e-3) / 1e9
    out = {
        "metric": METRIC, "value": round(cells * iters * ARGS.steps / elapsed / 1e9, 3),
        "unit": "Gcell-updates/s", "n_gpus": 1, "steps": ARGS.steps, "warmup": ARGS.warmup,
        "ms_per_step": round(elapsed / ARGS.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: lid-driven cavity from rest, lid u = 1 (no dataset)",
        "config": {"workload": "cavity2d_128x128_re100_jacobi500", "grid": [ny, nx], "iters_per_step": iters,
                   "step": "LidDrivenCavitySolver.time_step (predictor, BC, divergence, 500 Jacobi sweeps, "
                           "projection, divergence cleaning, energy)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": ("jacobi2d_persist<MASK, 8> (the whole solve in one launch; latency-bound: 190 KB per solve)"
                                if persistent else f"jacobi2d_small ({spl} sweeps per launch)"),
                     "sweeps_per_launch": spl, "cells_per_launch": cells, "algorithmic_bytes_per_launch": alg,
                     "avg_launch_ms": round(launch_ms, 5)},
        "cpu_baseline": None,
    }
    if not ARGS.no_cpu_baseline:
        o = oracle.OracleCavitySolver(cfg, numpy_jacobi=True)
        n = 0
        t0 = time.perf_counter()
        while n < 10 or (time.perf_counter() - t0 < 5.0 and n < 400):
            o.time_step()
            n += 1
        t = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": cells * iters * n / t / 1e9, "unit": "Gcell-updates/s", "cores": 1,
                               "kind": "port", "ms_per_step": round(t / n * 1e3, 3),
                               "sample": f"{n} steps of OracleCavitySolver(numpy_jacobi=True).time_step() "
                                         f"(the same step, pressure in the reference's NumPy Jacobi form, "
                                         f"v5.py:336-346); {t:.2f} s; NumPy uses 1 of {os.cpu_count()} "
                                         f"logical CPUs"}
    print(json.dumps(out), flush=True)


def predictor_bench():
    """The fused predictor (v5.py:388-403) on the 8192^2 grid of
    OptimizedTurbulentConfig's domain: u, v ~ U(-1, 1) (seeded), SUPG, nu_eff =
    nu + art_visc as a scalar (nu_t == 0 with LES off, v5.py:386-388), tau
    written.  value = cells / s; roofline = algorithmic bytes (20 B per f32
    cell, 40 B per f64) / the launch's HIP-event duration (the library's
    predictor timing channel).  --tau-mode exact|fast picks the SUPG tau
    arithmetic; the CPU-baseline leg also measures the launch's relative
    L-inf against the oracle (exact arithmetic) on the sampled rows."""
    import torch
    import _pkgpath
    _pkgpath.load()
    from cfd_simulations_amd import kernels as K
    from cfd_simulations_amd._lib import call, lib
    from cfd_simulations_amd.solver import OptimizedTurbulentConfig
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("the predictor workload is single-GPU")
    shape, dt_name, _, bpc = WORKLOADS[ARGS.workload]
    ny, nx = shape
    f64 = dt_name == "f64"
    tdt = torch.float64 if f64 else torch.float32
    npt = np.float64 if f64 else np.float32
    cfg = OptimizedTurbulentConfig(nx=nx, ny=ny, memory_efficient=not f64)
    nu_eff = npt(cfg.nu) + npt(cfg.artificial_viscosity)
    dt = np.float32(2e-5)
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.rand(shape, generator=g, device="cuda", dtype=tdt) * 2 - 1
    v = torch.rand(shape, generator=g, device="cuda", dtype=tdt) * 2 - 1
    us, vs, tau = torch.empty_like(u), torch.empty_like(u), torch.empty_like(u)

    def step():
        K.predictor_fused(u, v, cfg.dx, cfg.dy, dt, float(nu_eff), True, us, vs, tau, tau_mode=ARGS.tau_mode)
    for _ in range(max(ARGS.warmup, 1)):
        step()
    torch.cuda.synchronize()
    call("cfd_timing_enable", 1)
    t0 = time.perf_counter()
    for _ in range(ARGS.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = ctypes.c_double()
    nl = ctypes.c_longlong()
    call("cfd_timing_read_channel", 1, ctypes.byref(ms), ctypes.byref(nl), 1)
    call("cfd_timing_enable", 0)
    launch_ms = ms.value / max(nl.value, 1)
    cells = ny * nx
    alg = cells * bpc
    achieved = alg / (launch_ms * 1e-3) / 1e9
    # the kernel that ran, as the library reports it
    mode_c, vec_c = ctypes.c_int(), ctypes.c_int()
    path = int(lib().cfd_get_last_predictor2d_path(ctypes.byref(mode_c), ctypes.byref(vec_c)))
    mode = {0: "exact", 1: "fast"}[mode_c.value]
    T = "double" if f64 else "float"
    kern = (f"k_predictor_rows<{T}, tau {mode}, SUPG, scalar nu, {vec_c.value} cells per lane> (row march)"
            if path == 1 else ("k_predictor64<SUPG>" if f64 else "k_predictor<SUPG>") + " (one thread per cell)")
    out = {
        "metric": "Gcell-updates/s of the fused advection-diffusion predictor; achieved HBM GB/s vs peak",
        "value": round(cells * ARGS.steps / elapsed / 1e9, 3), "unit": "Gcell-updates/s", "n_gpus": 1,
        "steps": ARGS.steps, "warmup": ARGS.warmup, "ms_per_step": round(elapsed / ARGS.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": dt_name,
        "data": "synthetic: u, v ~ U(-1, 1) seeded, on OptimizedTurbulentConfig's 20 x 4 domain (no dataset)",
        "config": {"workload": f"predictor2d_supg_{ny}x{nx}_{dt_name}", "grid": [ny, nx], "use_supg": True,
                   "nu_eff": "scalar (LES off)", "tau_written": True, "tau_mode": mode,
                   "tau_arithmetic": ("glibc powf/pow restated on device (the reference's NumPy scalar **), "
                                      "bit-exact" if mode == "exact" else
                                      "fastmath: x*x, correctly rounded sqrt, rcp+Newton divisions")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic(ARGS.workload + ("" if mode == "exact" else "_fast"), 1),
                     "kernel": kern, "bytes_per_cell": bpc, "cells_per_launch": cells,
                     "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(launch_ms, 5)},
        "cpu_baseline": None,
    }
    if not ARGS.no_cpu_baseline:
        import oracle
        rows = 512 if f64 else 1024
        hu, hv = u[:rows].cpu().numpy(), v[:rows].cpu().numpy()
        n = 0
        t0 = time.perf_counter()
        while n < 1 or (time.perf_counter() - t0 < 10.0 and n < 20):
            ref = oracle.predictor2d(hu, hv, nu_eff, dx=cfg.dx, dy=cfg.dy, dt=dt, use_supg=True, dtype=npt)
            n += 1
        t = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": rows * nx * n / t / 1e9, "unit": "Gcell-updates/s", "cores": 1,
                               "kind": "port",
                               "sample": f"{rows}x{nx} rows of the grid, {n} calls of oracle.predictor2d (C "
                                         f"restatement of v5.py:127-176, :388-403 with libm "
                                         f"{'pow' if f64 else 'powf'}, {dt_name}, serial); {t:.2f} s; host has "
                                         f"{os.cpu_count()} logical CPUs, 1 used"}
        # accuracy of the timed launch on the sampled rows (their interior:
        # row rows-1 is a boundary row of the sample), vs the exact oracle
        torch.cuda.synchronize()
        err = {}
        for k, t_ in (("u_star", us), ("v_star", vs), ("tau", tau)):
            a_ = t_[1:rows - 1].cpu().numpy().astype(np.float64)
            b_ = ref[k][1:rows - 1].astype(np.float64)
            err[k] = float(np.abs(a_ - b_).max() / max(np.abs(b_).max(), 1e-300))
        out["config"]["rel_linf_vs_exact_oracle"] = err
    print(json.dumps(out), flush=True)


SINGLE_GPU_WORKLOADS = ("cavity2d_128", "jacobi2d_8192_f64", "predictor2d_8192", "predictor2d_8192_f64")


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_launch_cmd(argv, n, port):
    """The child command that starts N ranks of this script on one node (one
    process per GPU, rendezvous on 127.0.0.1): the same bench.py arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py")] + list(argv)


def spawn_ranks(args, argv, run=None, device_count=None):
    """`bench.py --gpus N` (N > 1) started as a plain process: start the N
    ranks ourselves as a child `torch.distributed.run` and return its exit
    code.  Nothing here touches the GPU (counting devices does not initialise
    HIP on this image); the child is a fresh process, never an exec."""
    import subprocess
    n = args.gpus
    if args.workload in SINGLE_GPU_WORKLOADS:
        raise SystemExit(f"--workload {args.workload} is single-GPU; --gpus {n} applies to the 3-D slab workloads")
    if device_count is None:
        import torch
        device_count = torch.cuda.device_count()
    need = 1 if getattr(args, "shared_gpu", False) else n
    if device_count < need:
        raise SystemExit(f"--gpus {n}: only {device_count} GPU(s) visible on this node")
    if getattr(args, "shared_gpu", False) and args.transport != "ce":
        raise SystemExit("--shared-gpu runs the copy-engine transport (RCCL refuses two ranks on one device)")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    cmd = rank_launch_cmd(argv, n, _free_port())
    print(f"bench.py: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return (run or subprocess.run)(cmd, env=env).returncode


T_START = time.perf_counter()


def main():
    global ARGS
    ARGS = parse()
    if ARGS.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(ARGS, sys.argv[1:]))
    if ARGS.workload == "cavity2d_128":
        return cavity_bench()
    if ARGS.workload.startswith("predictor2d"):
        return predictor_bench()
    import torch
    import torch.distributed as dist
    import _pkgpath
    _pkgpath.load()
    from cfd_simulations_amd import kernels as K
    from cfd_simulations_amd import slab as S
    from cfd_simulations_amd._lib import call, lib

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != ARGS.gpus:
        print(f"WARNING: --gpus {ARGS.gpus} but WORLD_SIZE={world}: running {world} rank(s)", file=sys.stderr)
    if ARGS.shared_gpu and ARGS.transport != "ce":
        raise SystemExit("--shared-gpu runs the copy-engine transport (RCCL refuses two ranks on one device)")
    # --shared-gpu: every rank on device 0 (the rehearsal of the N-rank path on
    # a one-GPU lease); otherwise one GPU per rank
    local_dev = 0 if ARGS.shared_gpu else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    use_slab = world > 1 or ARGS.force_slab
    if use_slab and ARGS.shared_gpu:
        # RCCL refuses two ranks on one device: the process group (IPC blob
        # exchange, verification gathers, the timing max) runs on gloo
        dist.init_process_group("gloo")
    elif use_slab:
        # bound RCCL's send/recv kernel to 16 blocks: the overlapped slab
        # drivers confine the exchange to 16 reserved CUs (slab.hip,
        # partition_streams), where up to 48 such blocks fit at once
        os.environ.setdefault("NCCL_MAX_P2P_NCHANNELS", "16")
        dist.init_process_group("nccl", device_id=dev)

    def progress(what):
        # N-rank runs: a line per phase on stderr (a long silent phase reads as a hang)
        if use_slab:
            print(f"bench.py rank {rank}/{world}: {what} ({time.perf_counter() - T_START:.1f} s)",
                  file=sys.stderr, flush=True)

    shape, dt_name, iters_default, bpc = WORKLOADS[ARGS.workload]
    if ARGS.grid:
        grid = tuple(int(x) for x in ARGS.grid.split(","))
        if len(shape) != 3 or len(grid) != 3 or min(grid) < 8:
            raise SystemExit("--grid NZ,NY,NX applies to the 3-D workloads (each extent >= 8)")
        shape = grid
    iters = ARGS.iters or iters_default
    call("cfd_set_jacobi3d_config", ARGS.variant, ARGS.waves, ARGS.zchunk)
    if len(shape) == 3:
        call("cfd_set_jacobi3d_blocking", ARGS.tb, ARGS.tb_rows, ARGS.tb_zchunk)
        call("cfd_set_jacobi3d_prefetch", ARGS.tb_prefetch)
    else:
        call("cfd_set_jacobi2d_blocking", ARGS.tb)
        if ARGS.j2_staging >= 0:
            call("cfd_set_jacobi2d_staging", ARGS.j2_staging)
    dt = np.float32(5e-5)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)

    gs = ARGS.workload.startswith("rbgs")
    gs_done = None
    if gs:
        nz, ny, nx = shape
        h = 1.0 / (nx - 1)
        # two GS iterations per slab pass (the default; --tb 2/3: one) need 4-deep ghosts
        plan = S.SlabPlan(nz, world, rank, ghost=1 if ARGS.tb == 1 else (2 if ARGS.tb in (2, 3) else 4))
        if not use_slab:
            div = torch.randn(shape, generator=g, device=dev, dtype=torch.float32)
            phi = torch.zeros_like(div)
            tmp = torch.zeros_like(div)
            gs_ws = torch.empty(int(lib().cfd_rbgs_workspace_bytes(iters)), dtype=torch.uint8, device=dev)
            gs_done = torch.zeros(1, dtype=torch.int32, device=dev)

            def step():
                phi.zero_()
                K.solve_pressure_gauss_seidel3d(phi, div, h, h, h, dt, None, iters, GS_TOL, workspace=gs_ws,
                                                iters_done=gs_done, phi_tmp=tmp)
        else:
            progress("attaching the slab transport")
            comm = make_comm(S, rank, world)
            progress(f"transport up ({TRANSPORT}); allocating the {plan.nz_total}-plane slab")
            sj = S.SlabRBGS3D(plan, ny, nx, h, h, h, dt, comm, device=dev)
            sj.div.copy_(torch.randn(sj.div.shape, generator=g, device=dev, dtype=torch.float32))
            gs_done = sj.iters_done

            def step():
                sj.solve(iters, tolerance=GS_TOL, overlap=not ARGS.no_overlap)
        cells_all = (nz - 2) * (ny - 2) * (nx - 2) * iters
        cells_rank = (plan.z_update_end - plan.z_update_begin) * (ny - 2) * (nx - 2)
        workload = f"rbgs3d_7pt_{nz}x{ny}x{nx}_f32"
        dtype = "f32"
    elif len(shape) == 3:
        nz, ny, nx = shape
        h = 1.0 / (nx - 1)
        # slab ghosts: as deep as the sweeps per pass (r05 per-rank rehearsal at
        # R = 8: 4-deep ghosts / 4 sweeps per slab pass 20.0 ms per 200-sweep
        # solve against 23.0 with 3-deep ones; r03, before the r05 tall-tile
        # work, 3-deep ones had been the faster)
        levels = int(lib().cfd_get_jacobi3d_levels())
        plan = S.SlabPlan(nz, world, rank, ghost=1 if ARGS.tb == 1 else levels)
        if not use_slab:
            div = torch.randn(shape, generator=g, device=dev, dtype=torch.float32)
            phi = torch.zeros_like(div)
            tmp = torch.zeros_like(div)
            rhs = None if ARGS.no_rhs_ws else torch.empty_like(div)

            def step():
                if rhs is None:
                    phi.zero_()
                    K.solve_pressure_jacobi3d(phi, div, h, dt, None, iters, phi_tmp=tmp, rhs_ws=None)
                else:
                    # phi = zeros + the sweeps (v5.py:337-346) in one call: the first
                    # pass starts from the zeros and forms the RHS workspace
                    K.solve_pressure_jacobi3d_zero(phi, div, h, dt, iters, phi_tmp=tmp, rhs_ws=rhs)
        else:
            progress("attaching the slab transport")
            comm = make_comm(S, rank, world)
            progress(f"transport up ({TRANSPORT}); allocating the {plan.nz_total}-plane slab")
            sj = S.SlabJacobi3D(plan, ny, nx, h, dt, comm, device=dev, rhs_workspace=not ARGS.no_rhs_ws)
            sj.div.copy_(torch.randn(sj.div.shape, generator=g, device=dev, dtype=torch.float32))
            progress("slab allocated and attached")

            def step():
                sj.solve(iters, overlap=not ARGS.no_overlap)
        cells_all = (nz - 2) * (ny - 2) * (nx - 2) * iters
        cells_rank = (plan.z_update_end - plan.z_update_begin) * (ny - 2) * (nx - 2)
        workload = f"jacobi3d_7pt_{nz}x{ny}x{nx}_f32"
        dtype = "f32"
    else:
        if world > 1:
            raise SystemExit("the 2-D workload is single-GPU (config 2); use jacobi3d_1024 for N>1")
        ny, nx = shape
        div = torch.randn(shape, generator=g, device=dev, dtype=torch.float64)
        phi = torch.zeros_like(div)
        tmp = torch.zeros_like(div)
        rhs = None if ARGS.no_rhs_ws else torch.empty_like(div)
        h = 1.0 / (nx - 1)

        def step():
            phi.zero_()
            K.solve_pressure_jacobi(phi, div, h, dt, None, iters, phi_tmp=tmp, rhs_ws=rhs)
        cells_all = (ny - 2) * (nx - 2) * iters
        cells_rank = (ny - 2) * (nx - 2)
        workload = f"jacobi2d_5pt_{ny}x{nx}_f64"
        dtype = "f64"

    def barrier():
        if use_slab:
            dist.barrier()

    verified = None
    if use_slab and len(shape) == 3 and not ARGS.no_verify:
        progress("verifying the slab solve against the one-GPU solve")
        verified = (verify_slabs_rbgs if gs else verify_slabs)(S, K, dist, comm, world, rank, dev)
        progress(f"verification {'bit-exact' if verified else 'MISMATCH'}")

    if ARGS.sweep_tiles and world == 1 and len(shape) == 3 and not gs:
        tile_sweep(K, call, div, phi, tmp, h, dt, bpc, cells_rank, rhs)

    for w in range(ARGS.warmup):
        step()
        if use_slab:  # (untimed) one line per warm-up step of an N-rank run
            torch.cuda.synchronize()
            progress(f"warm-up step {w + 1}/{ARGS.warmup} done")
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    call("cfd_timing_enable", 1)
    t0 = time.perf_counter()
    for _ in range(ARGS.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    progress("timed steps done")
    ms = ctypes.c_double()
    nsw = ctypes.c_longlong()
    call("cfd_timing_read", ctypes.byref(ms), ctypes.byref(nsw), 1)
    call("cfd_timing_enable", 0)
    sweep_ms = ms.value / max(nsw.value, 1)

    if use_slab:
        t = torch.tensor([elapsed, sweep_ms], dtype=torch.float64, device=coll_device(dist, dev))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, sweep_ms_max = float(t[0]), float(t[1])
    else:
        sweep_ms_max = sweep_ms

    value = cells_all * ARGS.steps / elapsed / 1e9
    # roofline of the dominant kernel, per launch.  A temporally blocked launch
    # (jacobi3d_tbr<K>) performs K sweeps in one HBM pass: 12 B of algorithmic
    # traffic per cell per launch = 12/K B per cell-update.
    blocked = ARGS.tb != 1 and (iters >= 2 or gs)
    levels = int(lib().cfd_get_jacobi3d_levels() if len(shape) == 3 else lib().cfd_get_jacobi2d_levels())
    # sweeps per launch: K Jacobi sweeps per blocked pass; the GS timing
    # counts iterations, and a fused GS pass is one (two with --tb 4)
    if not gs:
        # (a slab pass fuses min(levels, ghost) sweeps)
        spl = (min(levels, plan.ghost) if use_slab and len(shape) == 3 else levels) if blocked else 1
    elif use_slab:  # slab passes: two iterations with 4-deep ghosts, else one
        spl = 2 if blocked and plan.ghost == 4 else 1
    elif ARGS.tb_rows in (5, 13):  # the tuned 2-level GS kernel: one iteration per pass
        spl = 1
    else:  # single GPU: half-sweeps per pass (--tb, or the library's auto: 4 = two iterations)
        spl = int(lib().cfd_get_rbgs3d_levels()) / 2 if blocked else 1
    launch_ms = sweep_ms * spl
    alg_bytes = cells_rank * bpc  # one pass moves bpc bytes per cell whatever it fuses
    achieved = alg_bytes / (launch_ms * 1e-3) / 1e9
    traffic = None if ARGS.grid else load_traffic(ARGS.workload, world)
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Gcell-updates/s",
        "n_gpus": world,
        "steps": ARGS.steps,
        "warmup": ARGS.warmup,
        "ms_per_step": round(elapsed / ARGS.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic (div ~ N(0,1), seeded; phi zero-filled each step like v5.py:337)",
        "config": {"workload": workload, "grid": list(shape), "iters_per_step": iters,
                   "decomposition": "z-slab" if len(shape) == 3 else "none",
                   "halo": ((TRANSPORT_NAMES[TRANSPORT] + (", overlapped" if not ARGS.no_overlap else ""))
                            if use_slab else "none"),
                   "kernel_variant": ARGS.variant, "waves": ARGS.waves, "zchunk": ARGS.zchunk,
                   "temporal_blocking": ARGS.tb, "tb_rows": ARGS.tb_rows,
                   "rhs_workspace": not ARGS.no_rhs_ws},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": (f"jacobi3d_tbr<{int(2 * spl)}, MODE_RBGS>" if blocked else "rbgs3d_color x2") if gs
                     else (blocked_kernel_name(levels, ARGS.tb_rows) if blocked
                           else "jacobi3d_march") if len(shape) == 3
                     else (f"jacobi2d_tbk<{levels}>" if blocked else "jacobi2d_march"),
                     "sweeps_per_launch": spl, "bytes_per_cell_update": bpc / spl,
                     "cells_per_launch": cells_rank, "algorithmic_bytes_per_launch": alg_bytes,
                     "avg_launch_ms": round(launch_ms, 4),
                     "max_rank_avg_launch_ms": round(sweep_ms_max * spl, 4)},
        "cpu_baseline": None,
    }
    if gs:
        out["metric"] = METRIC.replace("Jacobi", "red-black Gauss-Seidel")
        out["config"]["tolerance"] = GS_TOL
        out["config"]["iterations_done_last_step"] = int(gs_done.item())
        out["roofline"]["bytes_per_cell_update"] = bpc / spl if blocked else 2 * bpc
    if ARGS.shared_gpu and use_slab:
        out["config"]["shared_gpu"] = (f"rehearsal: {world} ranks (processes) on device 0, gloo process group; "
                                       f"the timing is not a scaling number")
    if verified is not None:
        out["config"]["multi_gpu_parity"] = (("bit-exact vs 1-GPU solve (96^3, 9 its + early stop, both ghost depths)"
                                              if gs else
                                              "bit-exact vs 1-GPU solve (96^3, ghost depths 1-4)")
                                             if verified else "MISMATCH")
    if rank == 0 and world == 1 and not ARGS.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(shape, iters, gs)
        if len(shape) == 3:
            out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(shape, gs)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_slab and len(shape) == 3:
        if hasattr(comm, "status"):
            comm.status()  # raises if a neighbour wait expired during the run
        comm.close()
    if use_slab:
        dist.destroy_process_group()


TRANSPORT = None
TRANSPORT_NAMES = {"ce": "copy engines (SDMA into IPC-mapped neighbour ghosts)", "rccl": "rccl send/recv"}


def make_comm(S, rank, world):
    """The slab comm of --transport; a copy-engine comm that cannot map its
    peers' buffers (no IPC between these GPUs) falls back to RCCL, and the
    JSON line's config.halo says which one ran."""
    global TRANSPORT
    if ARGS.transport == "ce":
        import torch
        comm = None
        try:  # collective: every rank raises if any rank fails to map its peers
            comm = S.CopyEngineComm(rank, world)
            probe = torch.zeros((2, 4096), dtype=torch.float32, device="cuda")
            comm.attach(probe[0], probe[1])
            TRANSPORT = "ce"
            return comm
        except Exception as e:  # noqa: BLE001 -- reported, then RCCL
            if comm is not None:
                comm.close()
            if ARGS.shared_gpu:
                raise
            print(f"WARNING: copy-engine transport unavailable ({e}); using RCCL", file=sys.stderr)
    TRANSPORT = "rccl"
    return S.RcclComm(rank, world)


def blocked_kernel_name(levels, rows):
    """The kernel cfd_jacobi3d_f32 dispatches for (levels, rows) -- mirrors
    jacobi3d_blocked_pass in poisson3d.hip (the tall-tile kernel for 2..4)."""
    if rows == 0:
        return f"jacobi3d_tbr<{levels}> (tile shape by the launcher's cost model)"
    return f"jacobi3d_tbr<{levels}> ({rows}-row tiles)"


def verify_slabs(S, K, dist, comm, world, rank, dev):
    """Multi-GPU parity on a small grid before timing: every rank solves its
    slab through RCCL, rank 0 solves the whole grid on its own GPU, and the
    gathered owned planes must match bit-for-bit."""
    import torch
    nz, ny, nx = 96, 90, 104
    g = torch.Generator(device=dev).manual_seed(99)
    div = torch.randn((nz, ny, nx), generator=g, device=dev, dtype=torch.float32)  # same on every rank
    ok = True
    for ghost, iters in ((1, 7), (2, 8), (3, 8), (4, 10)):
        plan = S.SlabPlan(nz, world, rank, ghost=ghost)
        sj = S.SlabJacobi3D(plan, ny, nx, 0.03, np.float32(1e-3), comm, device=dev)
        lo = plan.z_lo - ghost
        for k in range(plan.nz_total):
            if 0 <= lo + k < nz:
                sj.div[k].copy_(div[lo + k])
        sj.solve(iters, overlap=True)
        mine = sj.owned().contiguous()
        sizes = [S.SlabPlan(nz, world, r, ghost=ghost).nz_local for r in range(world)]
        parts = [torch.empty((n, ny, nx), dtype=torch.float32, device=dev) for n in sizes]
        parts = gather_planes(dist, parts, mine, rank, dev)
        if rank == 0:
            ref = torch.zeros_like(div)
            K.solve_pressure_jacobi3d(ref, div, 0.03, np.float32(1e-3), None, iters)
            ok &= bool(torch.equal(torch.cat(parts), ref))
    flag = torch.tensor([1 if ok else 0], device=coll_device(dist, dev))
    dist.broadcast(flag, src=0)
    if not bool(flag.item()) and rank == 0:
        print("WARNING: multi-GPU slab result differs from the single-GPU solve", file=sys.stderr)
    return bool(flag.item())


def verify_slabs_rbgs(S, K, dist, comm, world, rank, dev):
    """verify_slabs for the distributed red-black GS: both ghost depths, a
    fixed count and an early stop (global max|change| < tol)."""
    import torch
    nz, ny, nx = 96, 90, 104
    g = torch.Generator(device=dev).manual_seed(98)
    div = torch.randn((nz, ny, nx), generator=g, device=dev, dtype=torch.float32) * 1e-3
    ok = True
    for ghost, iters, tol in ((1, 9, 0.0), (2, 9, 0.0), (2, 400, 2e-5), (4, 400, 1.5e-5)):
        plan = S.SlabPlan(nz, world, rank, ghost=ghost)
        sg = S.SlabRBGS3D(plan, ny, nx, 0.05, 0.05, 0.05, np.float32(1e-2), comm, device=dev)
        lo = plan.z_lo - ghost
        for k in range(plan.nz_total):
            if 0 <= lo + k < nz:
                sg.div[k].copy_(div[lo + k])
        sg.solve(iters, tolerance=tol, overlap=True)
        mine = sg.owned().contiguous()
        sizes = [S.SlabPlan(nz, world, r, ghost=ghost).nz_local for r in range(world)]
        parts = [torch.empty((n, ny, nx), dtype=torch.float32, device=dev) for n in sizes]
        parts = gather_planes(dist, parts, mine, rank, dev)
        n_mine = int(sg.iters_done.item())
        if rank == 0:
            ref = torch.zeros_like(div)
            done = torch.zeros(1, dtype=torch.int32, device=dev)
            K.solve_pressure_gauss_seidel3d(ref, div, 0.05, 0.05, 0.05, np.float32(1e-2), None, iters, tol,
                                            iters_done=done)
            ok &= bool(torch.equal(torch.cat(parts), ref)) and n_mine == int(done.item())
    flag = torch.tensor([1 if ok else 0], device=coll_device(dist, dev))
    dist.broadcast(flag, src=0)
    if not bool(flag.item()) and rank == 0:
        print("WARNING: multi-GPU RB-GS result differs from the single-GPU solve", file=sys.stderr)
    return bool(flag.item())


def coll_device(dist, dev):
    """Where a tensor of a torch.distributed collective lives: the GPU under
    RCCL, the host under gloo (the --shared-gpu rehearsal)."""
    import torch
    return dev if dist.get_backend() == "nccl" else torch.device("cpu")


def gather_planes(dist, parts, mine, rank, dev):
    """All-gather every rank's owned planes into `parts` (rank order), equal or
    uneven counts, on the process group's device; returns them on `dev`."""
    cd = coll_device(dist, dev)
    mine = mine.to(cd)
    parts = [p.to(cd) for p in parts]
    if len({p.shape for p in parts}) == 1:
        dist.all_gather(parts, mine)
    else:
        for r, p in enumerate(parts):
            if r == rank:
                p.copy_(mine)
            dist.broadcast(p, src=r)
    return [p.to(dev) for p in parts]


def tile_sweep(K, call, div, phi, tmp, h, dt, bpc, cells, rhs=None):
    """Config 3: time every tile on this grid: the single-sweep kernel's
    (variant, waves, zchunk) and the tall-tile kernels' (levels, output rows,
    zchunk); 2 levels is the tall-tile kernel too (the older 2-level kernels
    are gone from the library)."""
    import torch
    res = []
    call("cfd_set_jacobi3d_blocking", 1, 0, 0)
    for variant in (1, 2):
        for waves in (1, 2, 4, 8, 16):
            for zchunk in (0, 64, 128):
                call("cfd_set_jacobi3d_config", variant, waves, zchunk)
                phi.zero_()
                K.solve_pressure_jacobi3d(phi, div, h, dt, None, 4, phi_tmp=tmp, rhs_ws=rhs)
                torch.cuda.synchronize()
                call("cfd_timing_enable", 1)
                K.solve_pressure_jacobi3d(phi, div, h, dt, None, 20, phi_tmp=tmp, rhs_ws=rhs)
                ms = ctypes.c_double()
                n = ctypes.c_longlong()
                call("cfd_timing_read", ctypes.byref(ms), ctypes.byref(n), 1)
                call("cfd_timing_enable", 0)
                per = ms.value / n.value
                res.append({"variant": variant, "waves": waves, "zchunk": zchunk, "ms": round(per, 4),
                            "GBps": round(cells * bpc / per / 1e6, 1)})
                print(json.dumps({"tile": res[-1]}), file=sys.stderr, flush=True)
    call("cfd_set_jacobi3d_config", ARGS.variant, ARGS.waves, ARGS.zchunk)
    # the tall-tile kernels (the default family): levels per pass x output rows
    # per tile (the shape) x z-chunk (0: the launcher's cost model)
    call("cfd_set_jacobi3d_prefetch", 0)
    for lv, rows in [(2, 16), (2, 18), (2, 20), (2, 28), (3, 16), (3, 18), (3, 17), (4, 16), (4, 14), (4, 15)]:
        for zchunk in (0, 64, 128, 256, 512):
            call("cfd_set_jacobi3d_blocking", lv, rows, zchunk)
            phi.zero_()
            K.solve_pressure_jacobi3d(phi, div, h, dt, None, 12, phi_tmp=tmp, rhs_ws=rhs)
            torch.cuda.synchronize()
            call("cfd_timing_enable", 1)
            K.solve_pressure_jacobi3d(phi, div, h, dt, None, 24, phi_tmp=tmp, rhs_ws=rhs)
            ms = ctypes.c_double()
            n = ctypes.c_longlong()
            call("cfd_timing_read", ctypes.byref(ms), ctypes.byref(n), 1)
            call("cfd_timing_enable", 0)
            per = ms.value / n.value
            shape = [ctypes.c_int() for _ in range(4)]
            call("cfd_get_last_tbr_shape", *[ctypes.byref(v) for v in shape])
            shape = [v.value for v in shape]
            res.append({"tbr_levels": lv, "tb_rows": rows, "zchunk": zchunk,
                        "shape": {"levels": shape[0], "row_waves": shape[1], "rows_per_wave": shape[2],
                                  "zchunk": shape[3]},
                        "ms_per_sweep": round(per, 4), "ms_per_pass": round(per * lv, 4),
                        "GBps_pass": round(cells * 12 / (lv * per) / 1e6, 1),
                        "Gcell_per_s": round(cells / per / 1e6, 1)})
            print(json.dumps({"tile": res[-1]}), file=sys.stderr, flush=True)
    call("cfd_set_jacobi3d_blocking", ARGS.tb, ARGS.tb_rows, ARGS.tb_zchunk)
    call("cfd_set_jacobi3d_prefetch", ARGS.tb_prefetch)
    return res


if __name__ == "__main__":
    main()
