"""The fused predictor (v5.py:388-403; kernels :112-176) on the GPU, bit-exact
against the oracle's C restatement (oracle.predictor2d, pinned to the
reference's own outputs by tests/test_oracle_golden.py):

* the bench workload at full size: 8192^2, SUPG, scalar nu_eff, tau written
  (the row-march kernel k_predictor_rows the bench times), and the same grid
  through every kernel variant (row march vs one thread per cell, SUPG and
  upwind, array and scalar nu_eff), which must agree bit for bit;
* ragged shapes (nx not a multiple of the 256-column segment, tiny grids,
  nx % 4 != 0 falling back to the per-cell kernel), chunk lengths down to one
  row (every row a chunk boundary);
* inputs that force the exact-path powf off its fast path: squares and roots
  near a float rounding midpoint, zeros, subnormals, huge values, inf, NaN.
"""
import numpy as np
import pytest
import torch

import oracle
from cfd_simulations_amd import kernels as K
from cfd_simulations_amd._lib import call
from cfd_simulations_amd.solver import OptimizedTurbulentConfig

pytestmark = pytest.mark.gpu
DEV = "cuda"
SQ_WIN, SQRT_WIN = 952545, 931768  # libm_powf.hpp kPowfSqWin / kPowfSqrtWin


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


@pytest.fixture(autouse=True)
def _reset_tuning():
    call("cfd_reset_tuning")
    yield
    call("cfd_reset_tuning")


def _cfg(ny, nx):
    c = OptimizedTurbulentConfig(nx=nx, ny=ny)
    return c, np.float32(c.nu) + np.float32(c.artificial_viscosity)


def _check(u, v, nu, c, dt, supg, nu_array, ref=None):
    ny, nx = u.shape
    nu_in = np.full((ny, nx), nu, np.float32) if nu_array else float(nu)
    ref = ref or oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=dt, use_supg=supg)
    us, vs, tau = K.predictor_fused(dev(u), dev(v), c.dx, c.dy, dt, dev(nu_in) if nu_array else nu_in, supg)
    assert np.array_equal(host(us), ref["u_star"], equal_nan=True)
    assert np.array_equal(host(vs), ref["v_star"], equal_nan=True)
    if supg:
        assert np.array_equal(host(tau), ref["tau"], equal_nan=True)
    return ref


def test_predictor_8192_bench_workload_bitexact():
    """The bench's predictor2d_8192 step (row march, SUPG, scalar nu_eff, tau
    written) against the oracle at full size."""
    ny = nx = 8192
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(3)
    u = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    v = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    _check(u, v, nu, c, np.float32(2e-5), True, False)


def test_predictor_8192_variants_agree():
    """Row march (1, 2 and 4 cells per lane) and one thread per cell, SUPG /
    upwind, array / scalar nu: the same bits at 8192^2."""
    ny = nx = 8192
    c, nu = _cfg(ny, nx)
    g = torch.Generator(device=DEV).manual_seed(11)
    u = torch.rand((ny, nx), generator=g, device=DEV) * 4 - 2
    v = torch.rand((ny, nx), generator=g, device=DEV) * 4 - 2
    nua = torch.full((ny, nx), float(nu), device=DEV)
    dt = np.float32(2e-5)
    for supg in (True, False):
        for nu_in in (float(nu), nua):
            outs = []
            for variant, vec in ((1, 0), (2, 4), (2, 2), (2, 1)):
                call("cfd_set_predictor2d_config", variant, 0, vec)
                outs.append([None if t is None else t.clone()
                             for t in K.predictor_fused(u, v, c.dx, c.dy, dt, nu_in, supg)])
            for o in outs[1:]:
                for a, b in zip(outs[0], o):
                    if a is not None:
                        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(40, 56), (180, 600), (37, 260), (5, 4), (3, 8), (64, 1028), (9, 58), (33, 2)])
@pytest.mark.parametrize("rows", [0, 1, 3])
@pytest.mark.parametrize("vec", [0, 1, 2, 4])
@pytest.mark.parametrize("supg,nu_array", [(True, False), (True, True), (False, True)])
def test_predictor_shapes_bitexact(shape, rows, vec, supg, nu_array):
    ny, nx = shape
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(ny * 1000 + nx)
    u = rng.uniform(-1.5, 1.5, shape).astype(np.float32)
    v = rng.uniform(-1.5, 1.5, shape).astype(np.float32)
    call("cfd_set_predictor2d_config", 0, rows, vec)
    _check(u, v, nu, c, np.float32(2e-5), supg, nu_array)


def _near_midpoint(rng, n):
    """float32 values whose exact square lies within twice the fast-path
    window of a float rounding midpoint."""
    x = rng.uniform(0.01, 4.0, n * 400).astype(np.float32)
    d = x.astype(np.float64) ** 2
    lo = (d.view(np.uint64) & np.uint64((1 << 29) - 1)).astype(np.int64) - (1 << 28)
    sel = x[np.abs(lo) < 2 * SQ_WIN]
    assert sel.size >= n
    return sel[:n]


def _near_midpoint_roots(rng, n):
    """float32 pairs (u, v) whose |V| = (f32(u^2) + f32(v^2))**0.5 lies within
    twice the fast-path window of a float rounding midpoint."""
    u = rng.uniform(-2.0, 2.0, n * 400).astype(np.float32)
    v = rng.uniform(-2.0, 2.0, n * 400).astype(np.float32)
    s = (u.astype(np.float64) ** 2).astype(np.float32) + (v.astype(np.float64) ** 2).astype(np.float32)
    d = np.sqrt(s.astype(np.float64))
    lo = (d.view(np.uint64) & np.uint64((1 << 29) - 1)).astype(np.int64) - (1 << 28)
    sel = np.abs(lo) < 2 * SQRT_WIN
    assert sel.sum() >= n
    return u[sel][:n], v[sel][:n]


@pytest.mark.parametrize("density", [1.0, 0.03])
@pytest.mark.parametrize("vec", [1, 2, 4])
def test_predictor_slow_path_and_special_values(density, vec):
    """u, v drawn from values whose squares sit near a rounding midpoint (the
    full glibc powf must run), values whose u^2 + v^2 root does, and zeros,
    subnormals, huge values, inf and NaN scattered over the grid.  density
    1: nearly every cell leaves the fast paths (every pass of the march's
    fallback loops has jobs in most lanes); 0.03: sparse fallbacks."""
    ny, nx = 64, 512
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(5)
    sq = _near_midpoint(rng, ny * nx)
    u = (sq * np.where(rng.random(ny * nx) < 0.5, -1, 1)).astype(np.float32).reshape(ny, nx)
    v = rng.permutation(sq).astype(np.float32).reshape(ny, nx)
    if density < 1.0:  # plain values elsewhere
        plain = rng.random((ny, nx)) >= density
        u[plain] = rng.uniform(-1, 1, plain.sum()).astype(np.float32)
        v[plain] = rng.uniform(-1, 1, plain.sum()).astype(np.float32)
    # a third of the cells: (u, v) pairs whose |V| root is near a midpoint
    ru, rv = _near_midpoint_roots(rng, int(ny * nx * density) // 3)
    idx = rng.choice(ny * nx, ru.size, replace=False)
    vf = v.reshape(-1)
    uf = u.reshape(-1)
    uf[idx] = ru
    vf[idx] = rv
    special = np.array([0.0, -0.0, 1e-45, -3e-39, 1e-20, 3e19, -2e30, np.inf, -np.inf, np.nan], np.float32)
    for k, val in enumerate(special):
        pos = rng.choice(ny * nx, 12, replace=False)
        uf[pos] = val
        vf[rng.choice(ny * nx, 12, replace=False)] = special[(k + 3) % special.size]
    with np.errstate(all="ignore"):
        for supg in (True, False):
            for rows in (0, 2):
                call("cfd_set_predictor2d_config", 2, rows, vec)
                _check(u, v, nu, c, np.float32(2e-5), supg, False)


@pytest.mark.parametrize("vec", [1, 2, 4])
def test_predictor_quiescent_fields_bitexact(vec):
    """Fields at rest or in uniform flow (v5's initial state: u = inflow, v = 0;
    a cavity at rest: u = v = 0) and a quiescent patch inside a moving one:
    the zero inputs go through the fast paths (glibc powf returns +0 for a
    zero base) and must give the oracle's bits, tau = dt / 2 where |V| <= eps."""
    ny, nx = 96, 520
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(17)
    dt = np.float32(2e-5)
    zero = np.zeros((ny, nx), np.float32)
    inflow = np.full((ny, nx), np.float32(c.V_inf), np.float32)
    moving = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    patch = moving.copy()
    patch[20:60, 100:300] = 0.0
    patch[30:40, 150:160] = -0.0
    call("cfd_set_predictor2d_config", 2, 0, vec)
    for u, v in ((zero, zero), (inflow, zero), (patch, zero), (patch, patch[::-1].copy()), (zero, moving)):
        for supg in (True, False):
            _check(u, v, nu, c, dt, supg, False)
