"""cfd_simulations_amd -- MI355X-native drop-in for the pressure-Poisson /
predictor hot path of Santhosh-Sathyamurthy/cfd-simulations' cylinder solver
(python/flow_over_cylinder (Fischer)/v5.py).

Layers:
  csrc/        hand-written gfx950 HIP kernels + the C ABI (include/cfdsim.h),
               built into libcfdsim.so in this directory
  _lib.py      ctypes binding of that ABI (no fallback if the library is absent)
  kernels.py   reference-named kernel functions (the @njit drop-ins)
  solver.py    OptimizedTurbulentConfig / OptimizedTurbulentSolver drop-ins
  slab.py      multi-GPU slab decomposition with RCCL halo exchange

Importing the package does not load the HIP library; the first kernel call
does (and raises if libcfdsim.so was not built).
"""
from __future__ import annotations

__version__ = "0.1.0"

from .solver import (OptimizedTurbulentConfig, OptimizedTurbulentSolver,  # noqa: F401
                     monitor_simulation_health, host_grid, host_masks, host_potential_flow)
from .slab import SlabPlan  # noqa: F401
from . import kernels  # noqa: F401
