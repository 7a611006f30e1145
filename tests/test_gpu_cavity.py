"""BASELINE config 1 on the GPU: the lid-driven cavity (128 x 128, Re = 100,
500 Jacobi iterations per pressure solve) through LidDrivenCavitySolver --
the v5 time step with cavity walls -- against the CPU path of the same step
(oracle.OracleCavitySolver).  Bar: BIT-EXACT fields and dt every step (the
projection step reassociates nothing); the mean kinetic energy to 1e-6
relative (float64 device sum vs NumPy's float32 pairwise sum).
"""
import numpy as np
import pytest
import torch

import oracle
from cfd_simulations_amd._lib import call
from cfd_simulations_amd.solver import LidDrivenCavityConfig, LidDrivenCavitySolver

pytestmark = pytest.mark.gpu


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.mark.parametrize("kw", [{}, {"use_supg": False}, {"use_fast_pressure": True, "pressure_iterations": 300},
                                {"nx": 96, "ny": 72, "pressure_iterations": 120}])
def test_cavity_steps_bitexact(kw):
    call("cfd_reset_tuning")
    c = LidDrivenCavityConfig(log_diagnostics=True, **kw)
    g = LidDrivenCavitySolver(c)
    o = oracle.OracleCavitySolver(c)
    for k in range(4):
        assert g.time_step() == o.time_step()
        for f in ("u", "v", "phi", "u_star", "v_star", "div_u_star"):
            assert np.array_equal(host(getattr(g, f)), getattr(o, f)), (f, k)
        d = g.diagnostics
        for key in ("pre_div_max", "grad_max", "post_div_max", "vorticity_max"):
            assert np.float32(d[key]) == o.diagnostics[key], (key, k)
    e = np.array([v for _, v in g.energy_history])
    assert np.allclose(e, [v for _, v in o.energy_history], rtol=1e-6, atol=0)
    u = host(g.u)
    assert (u[-1] == np.float32(c.lid_velocity)).all() and (u[:-1, [0, -1]] == 0).all()
