#!/usr/bin/env python3
"""Measurement aid: with a library built -DCFD_PRED_COUNT (CFDSIM_LIB), the
number of cells the predictor row march queued for the exact path, per
cells-per-lane setting, on the bench's 8192^2 inputs."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgpath  # noqa: E402
_pkgpath.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cfd_simulations_amd import kernels as K  # noqa: E402
from cfd_simulations_amd._lib import call, lib  # noqa: E402
from cfd_simulations_amd.solver import OptimizedTurbulentConfig  # noqa: E402
n = 8192
cfg = OptimizedTurbulentConfig(nx=n, ny=n)
g = torch.Generator(device="cuda").manual_seed(3)
u = torch.rand((n, n), generator=g, device="cuda") * 2 - 1
v = torch.rand((n, n), generator=g, device="cuda") * 2 - 1
nu = float(np.float32(cfg.nu) + np.float32(cfg.artificial_viscosity))
import ctypes  # noqa: E402
f = lib().cfd_debug_pred_count
f.restype = ctypes.c_ulonglong
f.argtypes = [ctypes.c_int]
for vec in (1, 2, 4):
    call("cfd_set_predictor2d_config", 2, 16, vec)
    f(1)
    K.predictor_fused(u, v, cfg.dx, cfg.dy, np.float32(2e-5), nu, True)
    q = f(1)
    print(f"vec {vec}: queued {q} of {n * n} cells = {q / (n * n) * 100:.3f} %")
