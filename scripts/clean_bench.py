"""Time clean_divergence_fast (v5.py:240-256) alone: the serial lexicographic
phi sweep dominates it.  Prints one JSON line per shape with microseconds per
call (two iterations: 5 launches on the skewed layout, k_lex_gs_skew).
A/B: CFD_LEX_SKEW_WAVES=1..4 sets the waves per band."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkgpath  # noqa: E402

_pkgpath.load()
from cfd_simulations_amd import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="180x600,1026x1026")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    for sh in a.shapes.split(","):
        ny, nx = (int(t) for t in sh.split("x"))
        g = torch.Generator(device="cpu").manual_seed(1)
        u0 = (torch.rand(ny, nx, generator=g) * 2 - 1).cuda()
        v0 = (torch.rand(ny, nx, generator=g) * 2 - 1).cuda()
        dx, dy = 20.0 / (nx - 1), 6.0 / (ny - 1)
        u, v = u0.clone(), v0.clone()
        for _ in range(3):
            K.clean_divergence_fast(u, v, dx, dy, iterations=2)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            K.clean_divergence_fast(u, v, dx, dy, iterations=2)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(json.dumps({"shape": [ny, nx], "us_per_call": round(us, 2),
                          "waves": os.environ.get("CFD_LEX_SKEW_WAVES", "4"),
                          "finite": bool(torch.isfinite(u).all())}), flush=True)


if __name__ == "__main__":
    main()
