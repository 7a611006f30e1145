#!/usr/bin/env python3
"""Debug helper: the clean_divergence phi sweep on the device against the
oracle, printing where the first differences are."""
import sys
from pathlib import Path
import numpy as np
import torch
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import _pkgpath  # noqa: E402
_pkgpath.load()
import oracle  # noqa: E402
from cfd_simulations_amd import kernels as K  # noqa: E402

for ny, nx in [(3, 50), (66, 30), (130, 17), (128, 128), (180, 600), (515, 9)]:
    for its in (1, 2):
        rng = np.random.default_rng(ny * 1000 + nx)
        u0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
        v0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
        dx, dy = 20.0 / (nx - 1), 6.0 / (ny - 1)
        cu, cv = oracle.clean_divergence2d(u0, v0, dx=dx, dy=dy, iterations=its)
        u, v = torch.from_numpy(u0).cuda(), torch.from_numpy(v0).cuda()
        K.clean_divergence_fast(u, v, dx, dy, iterations=its)
        gu = u.cpu().numpy()
        bad = np.argwhere(gu != cu)
        print(ny, nx, its, "mismatches", len(bad), bad[:8].tolist(), flush=True)
