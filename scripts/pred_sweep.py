#!/usr/bin/env python3
"""Predictor tuning map (tuning aid): ms per cfd_predictor2d_f32 call on an
8192^2 grid for kernel variant x rows per chunk x SUPG/upwind x tau on/off x
scalar/array nu_eff; one JSON line per configuration."""
import ctypes
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import _pkgpath  # noqa: E402

_pkgpath.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cfd_simulations_amd import kernels as K  # noqa: E402
from cfd_simulations_amd._lib import call  # noqa: E402

ny = nx = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
g = torch.Generator(device="cuda").manual_seed(3)
u = torch.rand((ny, nx), generator=g, device="cuda") * 2 - 1
v = torch.rand((ny, nx), generator=g, device="cuda") * 2 - 1
us, vs, tau = torch.empty_like(u), torch.empty_like(u), torch.empty_like(u)
nua = torch.full((ny, nx), 0.0026667, device="cuda")
dx = dy = 20.0 / (nx - 1)
dt = np.float32(2e-5)
for variant, rows, vec in [(1, 0, 0), (2, 0, 4), (2, 16, 4), (2, 32, 4), (2, 0, 2), (2, 16, 2), (2, 32, 2),
                          (2, 0, 1), (2, 16, 1), (2, 32, 1), (2, 64, 1)]:
    for supg in (True, False):
        for with_tau in ((True, False) if supg else (False,)):
            for nu in (0.0026667, nua):
                call("cfd_set_predictor2d_config", variant, rows, vec)
                for _ in range(3):
                    K.predictor_fused(u, v, dx, dy, dt, nu, supg, us, vs, tau if with_tau else None)
                torch.cuda.synchronize()
                call("cfd_timing_enable", 1)
                for _ in range(10):
                    K.predictor_fused(u, v, dx, dy, dt, nu, supg, us, vs, tau if with_tau else None)
                ms = ctypes.c_double()
                n = ctypes.c_longlong()
                call("cfd_timing_read", ctypes.byref(ms), ctypes.byref(n), 1)
                call("cfd_timing_enable", 0)
                per = ms.value / n.value
                nb = (8 + 8 + (4 if with_tau else 0) + (4 if not isinstance(nu, float) else 0)) * ny * nx
                print(json.dumps({"variant": variant, "rows": rows, "vec": vec, "supg": supg, "tau": with_tau,
                                  "nu_array": not isinstance(nu, float), "ms": round(per, 4),
                                  "GBps": round(nb / per / 1e6, 1)}), flush=True)
