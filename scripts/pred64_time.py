#!/usr/bin/env python3
"""Times the fp64 fused predictor on 8192^2, SUPG and upwind (the memory-side
reference), 20 launches each."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402
_pkgpath.load()
from cfd_simulations_amd import kernels as K  # noqa: E402

n = 8192
g = torch.Generator(device="cuda").manual_seed(3)
u = torch.rand((n, n), device="cuda", generator=g, dtype=torch.float64) * 2 - 1
v = torch.rand((n, n), device="cuda", generator=g, dtype=torch.float64) * 2 - 1
us, vs, tau = torch.empty_like(u), torch.empty_like(u), torch.empty_like(u)
for supg in (True, False):
    for _ in range(3):
        K.predictor_fused(u, v, 20.0 / (n - 1), 4.0 / (n - 1), 2e-5, 1.0 / 600, supg, u_star=us, v_star=vs, tau=tau)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.predictor_fused(u, v, 20.0 / (n - 1), 4.0 / (n - 1), 2e-5, 1.0 / 600, supg, u_star=us, v_star=vs, tau=tau)
    e1.record()
    torch.cuda.synchronize()
    print(f"f64 predictor 8192^2 supg={supg}: {e0.elapsed_time(e1) / 20:.4f} ms", flush=True)
