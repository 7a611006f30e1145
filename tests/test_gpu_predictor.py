"""The fused predictor (v5.py:388-403; kernels :112-176) on the GPU, bit-exact
against the oracle's C restatement (oracle.predictor2d, pinned to the
reference's own outputs by tests/test_oracle_golden.py):

* the bench workload at full size: 8192^2, SUPG, scalar nu_eff, tau written
  (the row-march kernel k_predictor_rows the bench times), and the same grid
  through every kernel variant (row march vs one thread per cell, SUPG and
  upwind, array and scalar nu_eff), which must agree bit for bit;
* ragged shapes (nx not a multiple of the 256-column segment, tiny grids,
  nx % 4 != 0 lowering the cells per lane down to 1), chunk lengths down to
  one row (every row a chunk boundary);
* inputs that force the exact-path powf off its fast path: squares and roots
  near a float rounding midpoint, zeros, subnormals, huge values, inf, NaN.
"""
import ctypes
import types

import numpy as np
import pytest
import torch

import oracle
from cfd_simulations_amd import kernels as K
from cfd_simulations_amd._lib import call, lib
from cfd_simulations_amd.solver import OptimizedTurbulentConfig, OptimizedTurbulentSolver
from conftest import rel_linf

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


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("variant", [0, 1])
def test_predictor_without_supg_zeroes_tau(dtype, variant):
    """Without SUPG the predictor fills a given tau with zeros -- the
    reference's np.zeros tau_supg, never assigned without SUPG (v5.py:292) --
    so the solver needs no separate fill; u*, v* are unchanged by it."""
    ny, nx = 37, 260
    c, nu = _cfg(ny, nx)
    g = torch.Generator(device=DEV).manual_seed(5)
    u = (torch.rand((ny, nx), generator=g, device=DEV) * 2 - 1).to(dtype)
    v = (torch.rand((ny, nx), generator=g, device=DEV) * 2 - 1).to(dtype)
    call("cfd_set_predictor2d_config", variant, 0, 0)
    tau = torch.full((ny, nx), float("nan"), dtype=dtype, device=DEV)
    us, vs, t = K.predictor_fused(u, v, c.dx, c.dy, 2e-5, float(nu), False, tau=tau)
    assert t is tau and bool((tau == 0).all())
    us0, vs0, t0 = K.predictor_fused(u, v, c.dx, c.dy, 2e-5, float(nu), False)
    assert t0 is None and torch.equal(us, us0) and torch.equal(vs, vs0)


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


# ---------------------------------------------------------------- tau mode 1
# The tolerance mode (cfd_set_predictor2d_tau_mode(1), Solver supg_tau="fast"):
# the compiled reference's fastmath |V| = sqrt(u*u + v*v) (v5.py:149,
# @njit(fastmath=True)), tau's divisions on v_rcp_f32 + one Newton step.
# Bar: north_star's 1e-6 relative L-infinity (max |a - b| / max |b|) on u*,
# v*, tau, against the exact oracle (the reference's NumPy arithmetic) and
# against the oracle's fastmath form, on finite fields (no fallbacks: an inf
# input may give NaN where the exact mode gives 0).
FAST_TOL = 1e-6


def _fast(u, v, c, dt, nu_in, supg=True):
    return K.predictor_fused(u, v, c.dx, c.dy, dt, nu_in, supg, tau_mode="fast")


def _assert_close(got, ref, tol, what):
    for k in ("u_star", "v_star", "tau"):
        if k in got:
            err = rel_linf(got[k], ref[k])
            assert err <= tol, (what, k, err)


def test_predictor_fast_mode_8192_tolerance():
    """The bench workload in tau mode 1 against the exact oracle and the
    fastmath oracle at full size: within 1e-6 relative L-inf on u*, v*, tau;
    the kernel that ran is the row march in mode 1."""
    ny = nx = 8192
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(3)
    u = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    v = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    dt = np.float32(2e-5)
    us, vs, tau = _fast(dev(u), dev(v), c, dt, float(nu))
    got = {"u_star": host(us), "v_star": host(vs), "tau": host(tau)}
    mode, vec = ctypes.c_int(), ctypes.c_int()
    assert lib().cfd_get_last_predictor2d_path(ctypes.byref(mode), ctypes.byref(vec)) == 1 and mode.value == 1
    _assert_close(got, oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=dt), FAST_TOL, "exact")
    fm = oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=dt, fastmath=True)
    _assert_close(got, fm, FAST_TOL, "fastmath")
    # the square root is the correctly rounded one: tau agrees with the
    # fastmath oracle except where a Newton quotient is an ulp off
    assert np.mean(got["tau"] != fm["tau"]) < 1e-3


def test_predictor_fast_mode_reference_fixture(golden):
    """Tau mode 1 on the reference's own predictor fixture (v5.py's functions
    on seeded inputs, array nu_eff): within 1e-6 of its u*, v*, tau."""
    p = golden("predictor2d_f32_40x56_seed3.npz")
    c = types.SimpleNamespace(dx=float(p["dx"]), dy=float(p["dy"]))
    us, vs, tau = _fast(dev(p["u"]), dev(p["v"]), c, p["dt"], dev(p["nu_eff"]))
    _assert_close({"u_star": host(us), "v_star": host(vs), "tau": host(tau)},
                  {"u_star": p["u_star"], "v_star": p["v_star"], "tau": p["tau"]}, FAST_TOL, "fixture")


@pytest.mark.parametrize("shape", [(40, 56), (180, 600), (37, 260), (5, 4), (64, 1028), (9, 58)])
@pytest.mark.parametrize("vec", [0, 1, 4])
@pytest.mark.parametrize("nu_array", [False, True])
def test_predictor_fast_mode_shapes(shape, vec, nu_array):
    """Tau mode 1 on ragged shapes, every cells-per-lane setting, scalar and
    array nu_eff: within 1e-6 of the exact oracle; the upwind form (no tau)
    is bit-exact whatever the mode."""
    ny, nx = shape
    c, nu = _cfg(ny, nx)
    rng = np.random.default_rng(ny * 7 + nx)
    u = rng.uniform(-1.5, 1.5, shape).astype(np.float32)
    v = rng.uniform(-1.5, 1.5, shape).astype(np.float32)
    v[: ny // 3, : nx // 3] = 0.0  # quiescent patch: |V| <= eps, tau = dt / 2
    u[: ny // 4, : nx // 4] = 0.0
    nu_in = dev(np.full(shape, nu, np.float32)) if nu_array else float(nu)
    dt = np.float32(2e-5)
    call("cfd_set_predictor2d_config", 0, 0, vec)
    us, vs, tau = _fast(dev(u), dev(v), c, dt, nu_in)
    ref = oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=dt)
    _assert_close({"u_star": host(us), "v_star": host(vs), "tau": host(tau)}, ref, FAST_TOL, shape)
    us, vs, _ = _fast(dev(u), dev(v), c, dt, nu_in, supg=False)
    ref = oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=dt, use_supg=False)
    assert np.array_equal(host(us), ref["u_star"]) and np.array_equal(host(vs), ref["v_star"])


# ---------------------------------------------------------------- float64
def test_predictor_f64_8192_bench_workload_bitexact():
    """memory_efficient=False at the bench's 8192^2: the float64 row march
    (k_predictor_rows<double>, glibc pow for every square and root) against
    the oracle's float64 restatement with libm pow, bit for bit; tau mode 1
    within 1e-6 of it (and of the oracle's fastmath form)."""
    ny = nx = 8192
    c = OptimizedTurbulentConfig(nx=nx, ny=ny, memory_efficient=False)
    nu = np.float64(c.nu) + np.float64(c.artificial_viscosity)
    g = torch.Generator(device=DEV).manual_seed(3)
    u = torch.rand((ny, nx), generator=g, device=DEV, dtype=torch.float64) * 2 - 1
    v = torch.rand((ny, nx), generator=g, device=DEV, dtype=torch.float64) * 2 - 1
    dt = np.float32(2e-5)
    hu, hv = host(u), host(v)
    ref = oracle.predictor2d(hu, hv, nu, dx=c.dx, dy=c.dy, dt=float(dt), dtype=np.float64)
    us, vs, tau = K.predictor_fused(u, v, c.dx, c.dy, dt, float(nu), True, tau_mode="exact")
    assert lib().cfd_get_last_predictor2d_path(None, None) == 1
    for k, t in (("u_star", us), ("v_star", vs), ("tau", tau)):
        assert np.array_equal(host(t), ref[k]), k
    us, vs, tau = K.predictor_fused(u, v, c.dx, c.dy, dt, float(nu), True, tau_mode="fast")
    got = {"u_star": host(us), "v_star": host(vs), "tau": host(tau)}
    _assert_close(got, ref, FAST_TOL, "f64 exact")
    fm = oracle.predictor2d(hu, hv, nu, dx=c.dx, dy=c.dy, dt=float(dt), dtype=np.float64, fastmath=True)
    for k in got:  # IEEE divisions and sqrt in float64: the fastmath oracle's bits
        assert np.array_equal(got[k], fm[k]), k


@pytest.mark.parametrize("shape", [(40, 56), (37, 260), (5, 4), (64, 1030), (9, 58), (33, 2)])
@pytest.mark.parametrize("vec", [0, 1])
@pytest.mark.parametrize("supg,nu_array", [(True, False), (True, True), (False, True)])
def test_predictor_f64_shapes_bitexact(shape, vec, supg, nu_array):
    """The float64 row march on ragged shapes (odd nx: one cell per lane),
    chunk boundaries every 1 / 3 rows, special values: the oracle's bits."""
    ny, nx = shape
    c = OptimizedTurbulentConfig(nx=nx, ny=ny, memory_efficient=False)
    nu = np.float64(c.nu) + np.float64(c.artificial_viscosity)
    rng = np.random.default_rng(ny * 31 + nx)
    u = rng.uniform(-1.5, 1.5, shape)
    v = rng.uniform(-1.5, 1.5, shape)
    special = np.array([0.0, -0.0, 5e-324, -1e-310, 1e-160, 1e150, np.inf, -np.inf, np.nan])
    for k, val in enumerate(special):
        if k < u.size:
            u.flat[rng.integers(u.size)] = val
            v.flat[rng.integers(v.size)] = special[(k + 4) % special.size]
    nu_in = dev(np.full(shape, nu)) if nu_array else float(nu)
    dt = np.float32(2e-5)
    with np.errstate(all="ignore"):
        ref = oracle.predictor2d(u, v, nu, dx=c.dx, dy=c.dy, dt=float(dt), use_supg=supg, dtype=np.float64)
    for rows in (0, 1, 3):
        call("cfd_set_predictor2d_config", 2, rows, vec)
        us, vs, tau = K.predictor_fused(dev(u), dev(v), c.dx, c.dy, dt, nu_in, supg, tau_mode="exact")
        assert np.array_equal(host(us), ref["u_star"], equal_nan=True)
        assert np.array_equal(host(vs), ref["v_star"], equal_nan=True)
        if supg:
            assert np.array_equal(host(tau), ref["tau"], equal_nan=True)


@pytest.mark.parametrize("branch", ["gs", "jacobi"])
@pytest.mark.parametrize("memory_efficient", [True, False])
def test_time_step_fast_tau_vs_reference(golden, branch, memory_efficient):
    """Three time_step() calls with supg_tau="fast" against the reference's
    own steps (the exact-arithmetic fixtures): every field within 1e-5
    relative L-inf (SURVEY.md 8c's step tolerance), dt equal."""
    sfx = "" if memory_efficient else "_f64"
    d = golden(f"step_v5_120x36_n3{sfx}_{branch}.npz")
    c = OptimizedTurbulentConfig(nx=120, ny=36, pressure_iterations=200, use_fast_pressure=(branch == "gs"),
                                 memory_efficient=memory_efficient, supg_tau="fast")
    s = OptimizedTurbulentSolver(c)
    for k in range(3):
        dt = s.time_step()
        assert np.float32(dt) == np.float32(d[f"dt{k}"])
        for f, t in (("u", s.u), ("v", s.v), ("phi", s.phi), ("u_star", s.u_star), ("v_star", s.v_star),
                     ("tau", s.tau_supg)):
            err = rel_linf(host(t), d[f"{f}{k + 1}"])
            assert err <= 1e-5, (f, k, err)
    mode = ctypes.c_int()
    assert lib().cfd_get_last_predictor2d_path(ctypes.byref(mode), None) == 1 and mode.value == 1
