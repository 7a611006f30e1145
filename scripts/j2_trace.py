#!/usr/bin/env python3
"""Per-block phases of the persistent small-grid Jacobi (jacobi2d_persist) on
the v5 cylinder grid: median over tiles and blocks of the kernel's 100 MHz
timestamps (cfd_set_small2d_gs_trace): block period, halo wait (poll of the
neighbours' granules), levels (NI sweeps with their LDS exchanges), publish.

    python scripts/j2_trace.py [--ny 180 --nx 600 --iters 1500 --ni 8 --mode 2]
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
    ap.add_argument("--ny", type=int, default=180)
    ap.add_argument("--nx", type=int, default=600)
    ap.add_argument("--iters", type=int, default=1500)
    ap.add_argument("--ni", type=int, default=8)
    ap.add_argument("--mode", type=int, default=2, help="2: two sweeps per LDS exchange, 3: one")
    a = ap.parse_args()
    call("cfd_set_small2d_jacobi_persistent", a.mode, a.ni)
    rng = np.random.default_rng(3)
    div = torch.from_numpy(rng.standard_normal((a.ny, a.nx)).astype(np.float32)).cuda()
    mask = torch.from_numpy(rng.random((a.ny, a.nx)) < 0.03).cuda()
    phi = torch.zeros_like(div)
    dx = 20.0 / (a.nx - 1)
    solve = lambda: K.solve_pressure_jacobi(phi, div, dx, np.float32(5e-5), mask, a.iters, zero_start=True)  # noqa: E731
    for _ in range(3):
        solve()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        solve()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out_rows, sout = 32 - 2 * a.ni, 64 - 2 * a.ni
    ntiles = -(-a.nx // sout) * -(-(a.ny - 2) // out_rows)
    nb = -(-a.iters // a.ni)
    buf = torch.zeros((nb + 1) * ntiles * 4, dtype=torch.int64, device="cuda")
    call("cfd_set_small2d_gs_trace", buf.data_ptr(), buf.numel() * 8)
    solve()
    torch.cuda.synchronize()
    call("cfd_set_small2d_gs_trace", None, 0)
    t = buf.cpu().numpy().reshape(nb + 1, ntiles, 4).astype(np.float64) * 0.01  # us
    ends = t[nb]  # per tile: kernel entry, loop start, loop end, exit
    t = t[:nb]
    full = t
    t = t[2:nb - 1]
    q = lambda x: round(float(np.median(x)), 3)  # noqa: E731
    per = np.diff(t[:, :, 0], axis=0)
    pct = lambda x: [round(float(v), 3) for v in np.percentile(x, [10, 50, 90, 99, 99.9])]  # noqa: E731
    print(json.dumps({"ny": a.ny, "nx": a.nx, "iters": a.iters, "ni": a.ni, "mode": a.mode, "tiles": ntiles,
                      "ms_per_solve": round(ms, 4), "us_per_sweep": round(ms * 1e3 / a.iters, 3),
                      "period": q(np.diff(t[:, :, 0], axis=0)), "halo_wait": q(t[:, :, 1] - t[:, :, 0]),
                      "levels": q(t[:, :, 2] - t[:, :, 1]), "publish": q(t[:, :, 3] - t[:, :, 2]),
                      "gap_to_next": q(t[1:, :, 0] - t[:-1, :, 3]),
                      "start_skew_p50": q(t[:, :, 0].max(axis=1) - t[:, :, 0].min(axis=1)),
                      # the whole launch (first block start to last publish) and the mean period
                      "span_us": round(float(full[-1, :, 3].max() - full[0, :, 0].min()), 1),
                      "first_block_us": round(float(full[1, :, 0].max() - full[0, :, 0].min()), 2),
                      "mean_period": round(float((t[-1, :, 0] - t[0, :, 0]).mean() / (t.shape[0] - 1)), 3),
                      "period_pct_10_50_90_99_999": pct(per),
                      "halo_wait_pct": pct(t[:, :, 1] - t[:, :, 0]),
                      "levels_pct": pct(t[:, :, 2] - t[:, :, 1]),
                      # entry spread (dispatch), prologue, loop, epilogue of the launch
                      "entry_spread_us": round(float(ends[:, 0].max() - ends[:, 0].min()), 2),
                      "prologue_us_max": round(float((ends[:, 1] - ends[:, 0]).max()), 2),
                      "loop_us": round(float(ends[:, 2].max() - ends[:, 1].min()), 1),
                      "epilogue_us_max": round(float((ends[:, 3] - ends[:, 2]).max()), 2),
                      "kernel_us": round(float(ends[:, 3].max() - ends[:, 0].min()), 1)}), flush=True)
    call("cfd_reset_tuning")


if __name__ == "__main__":
    main()
