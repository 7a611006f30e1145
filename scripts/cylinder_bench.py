#!/usr/bin/env python3
"""End-to-end rate of the v5 cylinder solver's time_step() on one GPU.

    python scripts/cylinder_bench.py [--nx 600 --ny 180] [--steps 20] [--jacobi]

The reference's own configuration (OptimizedTurbulentConfig defaults,
v5.py:41-94): 600 x 180 grid, Re 600, SUPG predictor, 1500 red-black GS
iterations per step at tolerance 1e-8 (in fp32 the stop never fires, so all
1500 run).  Prints one JSON line: steps/s, ms per step, the pressure solve's
share, and the GS cell-update rate inside it, plus a ``cpu_baseline``: the same
step on this host's CPU (oracle.OracleSolver.time_step, the C restatement that
tests/test_oracle_golden.py pins bit-for-bit to the reference's own time_step
outputs; the reference's numba build is absent here) from the same initial
state -- the red-black GS serially (1 thread) and with the rows of each colour
over all OpenMP threads (the reference's prange structure); the Jacobi branch
in the reference's own NumPy form (1 thread, NumPy is single-threaded).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402

_pkgpath.load()
from cfd_simulations_amd.solver import OptimizedTurbulentConfig, OptimizedTurbulentSolver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=600)
    ap.add_argument("--ny", type=int, default=180)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--jacobi", action="store_true", help="use_fast_pressure=False (NumPy-branch Jacobi)")
    ap.add_argument("--levels", type=int, default=0, help="cfd_set_jacobi2d_blocking (0 auto)")
    ap.add_argument("--cpu-steps", type=int, default=3, help="CPU-baseline steps per form (0: none)")
    ap.add_argument("--coop-launch", action="store_true",
                    help="persistent solves as cooperative launches (cfd_set_persistent_launch(1, 0)); "
                         "the library default since r05 is a plain launch")
    ap.add_argument("--pred-rows", type=int, default=0, help="cfd_set_predictor2d_config(0, rows, 0) (0 auto)")
    a = ap.parse_args()
    from cfd_simulations_amd._lib import call
    if a.pred_rows:
        call("cfd_set_predictor2d_config", 0, a.pred_rows, 0)
    call("cfd_set_jacobi2d_blocking", a.levels)
    if a.coop_launch:
        call("cfd_set_persistent_launch", 1, 0)
    cfg = OptimizedTurbulentConfig(nx=a.nx, ny=a.ny, use_fast_pressure=not a.jacobi)
    s = OptimizedTurbulentSolver(cfg)
    for _ in range(a.warmup):
        s.time_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s.time_step()
    torch.cuda.synchronize()
    t_step = (time.perf_counter() - t0) / a.steps
    # the pressure solve alone, same state
    div = s.div_u_star.clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s.solve_pressure_fast(div)
    torch.cuda.synchronize()
    t_p = (time.perf_counter() - t0) / a.steps
    it = cfg.pressure_iterations
    cells = (a.ny - 2) * (a.nx - 2) * it
    out = {"workload": f"cylinder_v5_{a.nx}x{a.ny}", "pressure": "jacobi" if a.jacobi else "rbgs",
           "levels": a.levels, "persistent_launch": "cooperative" if a.coop_launch else "plain",
           "pressure_iterations": it, "steps_per_s": round(1.0 / t_step, 2),
           "ms_per_step": round(t_step * 1e3, 3), "pressure_ms": round(t_p * 1e3, 3),
           "pressure_share": round(t_p / t_step, 3),
           "pressure_us_per_iteration": round(t_p / it * 1e6, 2),
           "pressure_gcell_updates_s": round(cells / t_p / 1e9, 2),
           "u_finite": bool(torch.isfinite(s.u).all().item()),
           "energy_last": float(np.float64(s.energy_history[-1][1]))}
    if a.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_steps, t_step)
    print(json.dumps(out), flush=True)


def cpu_baseline(cfg, steps, gpu_step_s):
    """The same time_step on the host: oracle.OracleSolver from the solver's
    initial state (host_grid / host_masks / host_potential_flow), warm-up step
    excluded; ms per step for each form, and the GPU speed-up over it."""
    import oracle
    from cfd_simulations_amd.solver import host_grid, host_masks, host_potential_flow
    _, y, X, Y = host_grid(cfg)
    dist, cyl, ibm = host_masks(cfg, X, Y)
    u, v = host_potential_flow(cfg, X, Y, dist, ibm)
    forms = ([("rbgs_serial_c", 1, False), ("rbgs_openmp_c", oracle.threads(), True)] if cfg.use_fast_pressure
             else [("jacobi_numpy", 1, False)])
    res = []
    for name, cores, mt in forms:
        sol = oracle.OracleSolver(cfg, u, v, cyl, ibm, y)
        sol.mt = mt
        sol.numpy_jacobi = not cfg.use_fast_pressure  # the reference's own Jacobi form (v5.py:336-346)
        sol.time_step()
        t0 = time.perf_counter()
        for _ in range(steps):
            sol.time_step()
        t = (time.perf_counter() - t0) / steps
        res.append({"form": name, "cores": cores, "ms_per_step": round(t * 1e3, 2),
                    "steps_per_s": round(1.0 / t, 3), "gpu_speedup": round(t / gpu_step_s, 1),
                    "kind": "port", "sample": f"{steps} time_steps after one warm-up step, same config"})
    return res


if __name__ == "__main__":
    main()
