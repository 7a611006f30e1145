#!/usr/bin/env python3
"""Fixed cost of one persistent small-grid Jacobi solve (jacobi2d_persist) on
the v5 cylinder grid: ms per solve against the sweep count; the intercept of
the linear fit is the launch's cost outside its blocks.

    python scripts/j2_overhead.py [--ni 10 --mode 2]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402

_pkgpath.load()
from cfd_simulations_amd import kernels as K  # noqa: E402
from cfd_simulations_amd._lib import call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ni", type=int, default=10)
    ap.add_argument("--mode", type=int, default=2)
    a = ap.parse_args()
    call("cfd_set_small2d_jacobi_persistent", a.mode, a.ni)
    rng = np.random.default_rng(3)
    ny, nx = 180, 600
    div = torch.from_numpy(rng.standard_normal((ny, nx)).astype(np.float32)).cuda()
    mask = torch.from_numpy(rng.random((ny, nx)) < 0.03).cuda()
    phi = torch.zeros_like(div)
    out = {}
    for iters in (a.ni * 2 + 1, 101, 301, 751, 1500):
        solve = lambda: K.solve_pressure_jacobi(phi, div, 20.0 / (nx - 1), np.float32(5e-5), mask, iters, zero_start=True)  # noqa: E731
        for _ in range(3):
            solve()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            solve()
        e1.record()
        torch.cuda.synchronize()
        out[iters] = e0.elapsed_time(e1) / 20
    x = np.array(list(out)), np.array(list(out.values()))
    slope, icpt = np.polyfit(x[0], x[1], 1)
    print(json.dumps({"ni": a.ni, "mode": a.mode, "ms_per_solve": {k: round(v, 4) for k, v in out.items()},
                      "us_per_sweep_fit": round(slope * 1e3, 4), "fixed_us_fit": round(icpt * 1e3, 2)}), flush=True)
    call("cfd_reset_tuning")


if __name__ == "__main__":
    main()
