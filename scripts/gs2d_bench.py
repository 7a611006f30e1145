#!/usr/bin/env python3
"""Time the small-grid 2-D red-black GS solve (the v5 cylinder's 600 x 180
pressure solve, 1500 iterations) by iterations per block, persistent or
launch-per-block, with and without the stop test.  One JSON line per case.

  python scripts/gs2d_bench.py [--ny 180 --nx 600 --iters 1500 --reps 20]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ni", default="2,3,4")
    ap.add_argument("--modes", default="2,3,1",
                    help="cfd_set_small2d_gs_persistent modes (2 on, 3 on with one exchange per level, 1 off)")
    ap.add_argument("--tols", default="1e-8,0")
    ap.add_argument("--trace", action="store_true",
                    help="also record the persistent kernel's per-block timestamps and print phase medians")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    div = torch.from_numpy(rng.standard_normal((args.ny, args.nx)).astype(np.float32) * np.float32(1e-3)).to(dev)
    mask = torch.from_numpy(rng.random((args.ny, args.nx)) < 0.03).to(dev)
    phi = torch.zeros_like(div)
    tmp = torch.empty_like(div)
    done = torch.zeros(1, dtype=torch.int32, device=dev)
    for mode in [int(m) for m in args.modes.split(",")]:
        for ni in [int(n) for n in args.ni.split(",")]:
            for tol in [float(t) for t in args.tols.split(",")]:
                call("cfd_set_small2d_gs_iters", ni, 2)
                call("cfd_set_small2d_gs_persistent", mode)

                def solve():
                    phi.zero_()
                    K.solve_pressure_gauss_seidel_fast(phi, div, 0.05, 0.05, np.float32(1e-2), mask, args.iters,
                                                       tol, iters_done=done, phi_tmp=tmp)
                for _ in range(3):
                    solve()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    solve()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                out = {"ny": args.ny, "nx": args.nx, "iters": args.iters, "ni": ni,
                       "persistent": mode >= 2, "exchange_per_level": mode == 3, "tol": tol, "done": int(done.item()),
                       "ms_per_solve": round(ms, 4), "us_per_iteration": round(ms * 1e3 / args.iters, 3)}
                if args.trace and mode >= 2:
                    out["trace_us"] = trace_phases(solve, args, ni)
                print(json.dumps(out), flush=True)
    call("cfd_reset_tuning")


def trace_phases(solve, args, ni):
    """Median per-block phase durations (us) over tiles and blocks, from the
    kernel's 100 MHz timestamps: e0 block start, e1 halo in (wave 0), e2 tile
    ready (after the first barrier), e3 levels done."""
    L = 2 * ni
    out_rows, sout = 32 - 2 * L, 64 - 2 * L
    ntiles = -(-args.nx // sout) * -(-(args.ny - 2) // out_rows)
    nb = -(-args.iters // ni)
    buf = torch.zeros((nb + 1) * ntiles * 4, dtype=torch.int64, device="cuda")
    call("cfd_set_small2d_gs_trace", buf.data_ptr(), buf.numel() * 8)
    solve()
    torch.cuda.synchronize()
    call("cfd_set_small2d_gs_trace", None, 0)
    t = buf.cpu().numpy().reshape(nb + 1, ntiles, 4).astype(np.float64) * 0.01  # us
    ends = t[nb]  # per tile: kernel entry, loop start, loop end, exit
    t = t[:nb]
    done = t[:, :, 3] > 0
    blocks = int(done.all(axis=1).sum())
    t = t[2:blocks]
    q = lambda x: round(float(np.median(x)), 3)  # noqa: E731
    return {"blocks": blocks, "period": q(np.diff(t[:, :, 0], axis=0)), "halo_wait": q(t[:, :, 1] - t[:, :, 0]),
            "tile_ready": q(t[:, :, 2] - t[:, :, 1]), "levels": q(t[:, :, 3] - t[:, :, 2]),
            "publish_gap": q(t[1:, :, 0] - t[:-1, :, 3]),
            "start_skew_p50": q(t[:, :, 0].max(axis=1) - t[:, :, 0].min(axis=1)),
            "mean_period": round(float((t[-1, :, 0] - t[0, :, 0]).mean() / (t.shape[0] - 1)), 3),
            "entry_spread": round(float(ends[:, 0].max() - ends[:, 0].min()), 2),
            "prologue_max": round(float((ends[:, 1] - ends[:, 0]).max()), 2),
            "loop": round(float(ends[:, 2].max() - ends[:, 1].min()), 1),
            "epilogue_max": round(float((ends[:, 3] - ends[:, 2]).max()), 2),
            "kernel": round(float(ends[:, 3].max() - ends[:, 0].min()), 1)}


if __name__ == "__main__":
    main()
