#!/usr/bin/env python3
"""Per-wave step timeline of the 3-D tall-tile kernel (cfd_set_tbr_trace):
one 1024^3 solve (Jacobi, or --gs red-black GS), workgroup 0, z-steps 200..263.
Prints, per wave, the median cycles from step entry to its arrival at each
barrier and how long it then waits there; the last wave to arrive at a
barrier sets the step's length."""
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
from cfd_simulations_amd._lib import call, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gs", action="store_true")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--tb", type=int, default=0)
    args = ap.parse_args()
    n = args.n
    dev = torch.device("cuda", 0)
    div = torch.randn((n, n, n), device=dev, dtype=torch.float32)
    phi = torch.zeros_like(div)
    tmp = torch.zeros_like(div)
    call("cfd_set_jacobi3d_blocking", args.tb, 0, 0)
    buf = torch.zeros(16 * 64 * 5, dtype=torch.int64, device=dev)
    h, dt = 1.0 / (n - 1), np.float32(5e-5)
    ws = torch.empty(int(lib().cfd_rbgs_workspace_bytes(12)), dtype=torch.uint8, device=dev)

    def solve():
        if args.gs:
            K.solve_pressure_gauss_seidel3d(phi, div, h, h, h, dt, None, 12, 0.0, workspace=ws, phi_tmp=tmp)
        else:
            rhs = torch.empty_like(div)
            K.solve_pressure_jacobi3d_zero(phi, div, h, dt, 12, phi_tmp=tmp, rhs_ws=rhs)
    solve()
    torch.cuda.synchronize()
    call("cfd_set_tbr_trace", buf.data_ptr(), buf.numel() * 8)
    solve()
    torch.cuda.synchronize()
    call("cfd_set_tbr_trace", None, 0)
    t = buf.cpu().numpy().reshape(16, 64, 5).astype(np.float64)
    waves = [w for w in range(16) if (t[w] > 0).all()]
    t = t[waves]
    t0 = t[:, :, 0].min(axis=0)  # per step: the earliest wave's entry
    rel = t - t0[None, :, None]
    step_len = np.diff(t0)
    out = {"gs": args.gs, "waves": len(waves), "median_step_cycles": float(np.median(step_len))}
    per = []
    for i, w in enumerate(waves):
        per.append({"wave": w, "arrive_b1": float(np.median(rel[i, :, 1])), "wait_b1": float(np.median(rel[i, :, 2] - rel[i, :, 1])),
                    "arrive_b2": float(np.median(rel[i, :, 3])), "wait_b2": float(np.median(rel[i, :, 4] - rel[i, :, 3])),
                    "last_at_b1": int((rel[i, :, 1] == rel[:, :, 1].max(axis=0)).sum()),
                    "last_at_b2": int((rel[i, :, 3] == rel[:, :, 3].max(axis=0)).sum())})
    out["per_wave"] = per
    print(json.dumps(out))
    call("cfd_reset_tuning")


if __name__ == "__main__":
    main()
