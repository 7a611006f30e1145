"""GPU parity: the HIP kernels (called through the C ABI) against the pinned
CPU oracle and the reference-generated fixtures.

Bars (stated per test):
  * Jacobi 2-D/3-D, red-black GS, divergence, gradient, projection,
    clean_divergence, BC/IBM/clip: BIT-EXACT (same op order, no FMA).
  * SUPG predictor and the full time_step (steps 0-2, 1000-1001, 1500-1501):
    BIT-EXACT too -- |V| = (u**2 + v**2) ** 0.5 runs the device copy of glibc's
    powf that NumPy's float32 scalar `**` calls (libm_powf.hpp).
  * The mean kinetic energy is summed in float64 on the device where NumPy
    sums float32 pairwise: relative 1e-6 (the reference prints 3 decimals).
"""
import numpy as np
import pytest
import torch

import oracle
from cfd_simulations_amd import kernels as K
from cfd_simulations_amd import slab as S
from cfd_simulations_amd._lib import call, lib, ptr, stream_handle
from cfd_simulations_amd.solver import OptimizedTurbulentConfig, OptimizedTurbulentSolver

from conftest import ROOT, rel_linf

pytestmark = pytest.mark.gpu

DEV = "cuda"


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


# ------------------------------------------------------------- Jacobi 2-D
@pytest.mark.parametrize("name", ["jacobi2d_f32_128x128_it500_seed1234",
                                  "jacobi2d_f32_128x128_it500_seed1234_mask",
                                  "jacobi2d_f64_128x128_it500_seed1234",
                                  "jacobi2d_f64_128x128_it500_seed1234_mask",
                                  "jacobi2d_f32_40x72_it60_cyl"])
def test_jacobi2d_golden_bitexact(golden, name):
    d = golden(name + ".npz")
    phi = torch.zeros_like(dev(d["div"]))
    K.solve_pressure_jacobi(phi, dev(d["div"]), float(d["dx"]), d["dt"], dev(d["mask"]), int(d["iters"]))
    out = host(phi)
    assert out.dtype == d["phi"].dtype
    assert np.array_equal(out, d["phi"])


@pytest.mark.parametrize("blocking", [0, 1, 2, 3, 4, 5, 6, 8, 10, 12])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape,iters", [((37, 53), 17), ((3, 3), 4), ((130, 260), 31),
                                         ((66, 516), 8), ((2, 9), 3), ((200, 248), 10), ((9, 124), 6),
                                         ((71, 1000), 12), ((300, 124), 9), ((517, 40), 7)])
def test_jacobi2d_random_bitexact(dtype, shape, iters, blocking):
    call("cfd_set_jacobi2d_blocking", blocking)
    rng = np.random.default_rng(11)
    div = rng.standard_normal(shape).astype(dtype)
    phi0 = rng.standard_normal(shape).astype(dtype)  # nonzero edges + initial guess
    mask = rng.random(shape) < 0.1
    ref = oracle.jacobi2d(div, phi0, dx=0.013, dt=np.float32(3e-4), iters=iters, mask=mask)
    phi = dev(phi0)
    K.solve_pressure_jacobi(phi, dev(div), 0.013, np.float32(3e-4), dev(mask), iters)
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("staging", [0, 4, 6])
@pytest.mark.parametrize("blocking", [4, 6, 8])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape,iters,pre", [((37, 53), 17, False), ((130, 260), 31, True), ((9, 124), 6, True),
                                             ((71, 1000), 12, False), ((300, 124), 9, True), ((517, 40), 7, False),
                                             ((4, 600), 8, True), ((1030, 244), 16, True)])
def test_jacobi2d_staged_rows_bitexact(dtype, shape, iters, pre, blocking, staging):
    """Unmasked blocked passes, whose rows come through the per-wave LDS ring
    (jacobi2d_tbd, `staging` rows ahead) or the register march (0): bit-exact
    against the oracle with and without the rhs workspace."""
    call("cfd_set_jacobi2d_blocking", blocking)
    call("cfd_set_jacobi2d_staging", staging)
    try:
        rng = np.random.default_rng(21)
        div = rng.standard_normal(shape).astype(dtype)
        phi0 = rng.standard_normal(shape).astype(dtype)
        ref = oracle.jacobi2d(div, phi0, dx=0.017, dt=np.float32(2e-4), iters=iters)
        phi = dev(phi0)
        K.solve_pressure_jacobi(phi, dev(div), 0.017, np.float32(2e-4), None, iters,
                                rhs_ws=torch.empty_like(phi) if pre else None)
        assert np.array_equal(host(phi), ref)
    finally:
        call("cfd_set_jacobi2d_staging", 0)
        call("cfd_set_jacobi2d_blocking", 0)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_jacobi2d_rhs_workspace_bitexact(dtype):
    """The RHS prologue (rhs_ws) gives the same bits as the in-register RHS."""
    rng = np.random.default_rng(12)
    shape = (70, 132)
    div = rng.standard_normal(shape).astype(dtype)
    mask = rng.random(shape) < 0.05
    ref = oracle.jacobi2d(div, dx=0.011, dt=np.float32(7e-5), iters=9, mask=mask)
    phi = torch.zeros(shape, dtype=torch.float32 if dtype == np.float32 else torch.float64, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 0.011, np.float32(7e-5), dev(mask), 9, rhs_ws=torch.empty_like(phi))
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("tb", [1, 2])
@pytest.mark.parametrize("shape,iters", [((12, 14, 64), 6), ((9, 10, 260), 5), ((7, 9, 13), 3)])
def test_jacobi3d_rhs_workspace_bitexact(shape, iters, tb):
    call("cfd_set_jacobi3d_blocking", tb, 0, 0)
    rng = np.random.default_rng(13)
    div = rng.standard_normal(shape).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.02, dt=np.float32(3e-4), iters=iters)
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi3d(phi, dev(div), 0.02, np.float32(3e-4), None, iters, rhs_ws=torch.empty_like(phi))
    assert np.array_equal(host(phi), ref)


def test_jacobi2d_residual():
    rng = np.random.default_rng(3)
    div = rng.standard_normal((64, 96)).astype(np.float32)
    k_every, iters = 5, 20
    res = torch.zeros(iters // k_every, dtype=torch.float32, device=DEV)
    phi = torch.zeros((64, 96), dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 0.02, np.float32(1e-3), None, iters, resid_every=k_every,
                            resid_out=res)
    got = host(res)
    for k in range(1, iters // k_every + 1):
        a = oracle.jacobi2d(div, dx=0.02, dt=np.float32(1e-3), iters=k * k_every)
        b = oracle.jacobi2d(div, dx=0.02, dt=np.float32(1e-3), iters=k * k_every - 1)
        assert got[k - 1] == np.abs(a - b).max()


@pytest.mark.parametrize("iters", [3, 8])
def test_jacobi2d_8192_f64_full_size(iters):
    """Config 2 at full size (8192^2 fp64): a few sweeps, bit-exact."""
    n = 8192
    rng = np.random.default_rng(1234)
    div = rng.standard_normal((n, n))
    ref = oracle.jacobi2d(div, dx=1.0 / (n - 1), dt=np.float32(5e-5), iters=iters)
    phi = torch.zeros((n, n), dtype=torch.float64, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 1.0 / (n - 1), np.float32(5e-5), None, iters)
    assert np.array_equal(host(phi), ref)


# ------------------------------------------------------------- Jacobi 3-D
J3_CASES = [((10, 12, 16), None), ((9, 11, 13), None), ((34, 40, 260), None),
            ((6, 7, 520), None), ((20, 19, 8), "mask")]


@pytest.mark.parametrize("variant,waves,zchunk", [(0, 0, 0), (1, 1, 0), (1, 2, 3), (1, 4, 5),
                                                  (1, 8, 0), (1, 16, 2), (2, 1, 0), (2, 4, 7),
                                                  (2, 16, 1)])
@pytest.mark.parametrize("shape,masked", J3_CASES)
def test_jacobi3d_bitexact(shape, masked, variant, waves, zchunk):
    call("cfd_set_jacobi3d_config", variant, waves, zchunk)
    rng = np.random.default_rng(sum(shape))
    div = rng.standard_normal(shape).astype(np.float32)
    phi0 = rng.standard_normal(shape).astype(np.float32)
    mask = (rng.random(shape) < 0.15) if masked else None
    ref = oracle.jacobi3d(div, phi0, h=0.05, dt=np.float32(2e-3), iters=5, mask=mask)
    phi = dev(phi0)
    K.solve_pressure_jacobi3d(phi, dev(div), 0.05, np.float32(2e-3), None if mask is None else dev(mask), 5)
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("prefetch", [1, 2])
@pytest.mark.parametrize("rows,zchunk", [(16, 0), (18, 0), (20, 3), (28, 1), (16, 1), (20, 5)])
@pytest.mark.parametrize("shape,iters", [((10, 12, 16), 6), ((9, 11, 20), 7), ((34, 40, 260), 4),
                                         ((6, 7, 520), 5), ((20, 19, 8), 2), ((5, 33, 768), 9),
                                         ((3, 3, 4), 4)])
def test_jacobi3d_temporal_blocking_bitexact(shape, iters, rows, zchunk, prefetch):
    """Two sweeps fused per pass (jacobi3d_tbr<2>, every 2-level tile shape)
    == two single sweeps, bitwise."""
    call("cfd_set_jacobi3d_blocking", 2, rows, zchunk)
    call("cfd_set_jacobi3d_prefetch", prefetch)
    rng = np.random.default_rng(sum(shape) + iters)
    div = rng.standard_normal(shape).astype(np.float32)
    phi0 = rng.standard_normal(shape).astype(np.float32)
    ref = oracle.jacobi3d(div, phi0, h=0.05, dt=np.float32(2e-3), iters=iters)
    phi = dev(phi0)
    K.solve_pressure_jacobi3d(phi, dev(div), 0.05, np.float32(2e-3), None, iters)
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("levels,rows", [(3, 16), (3, 17), (3, 18), (3, 0), (4, 14), (4, 15), (4, 16),
                                         (2, 0)])
@pytest.mark.parametrize("shape,iters", [((9, 10, 12), 7), ((21, 30, 264), 8), ((40, 31, 520), 12),
                                         ((5, 4, 8), 4), ((13, 40, 16), 9), ((12, 47, 264), 8)])
@pytest.mark.parametrize("zchunk", [0, 1, 5])
@pytest.mark.parametrize("prefetch", [1, 2])
def test_jacobi3d_k_levels_bitexact(shape, iters, levels, rows, zchunk, prefetch):
    """K = 2..4 sweeps per HBM pass (jacobi3d_tbr: tall tiles, several rows
    per wave, every tile shape): bit-identical to the
    oracle for tile-edge shapes, several x-segments and y-tiles, z-chunks of
    1..5 planes (march start/end clipping) and remainders (iters % K)."""
    call("cfd_set_jacobi3d_blocking", levels, rows, zchunk)
    call("cfd_set_jacobi3d_prefetch", prefetch)
    rng = np.random.default_rng(31)
    div = rng.standard_normal(shape).astype(np.float32)
    phi0 = rng.standard_normal(shape).astype(np.float32)
    ref = oracle.jacobi3d(div, phi0, h=0.06, dt=np.float32(3e-3), iters=iters)
    phi = dev(phi0)
    for rhs in (None, torch.empty_like(phi)):
        phi.copy_(dev(phi0))
        K.solve_pressure_jacobi3d(phi, dev(div), 0.06, np.float32(3e-3), None, iters, rhs_ws=rhs)
        assert np.array_equal(host(phi), ref)


def test_jacobi3d_residual_matches_oracle():
    rng = np.random.default_rng(8)
    div = rng.standard_normal((18, 20, 64)).astype(np.float32)
    res = torch.zeros(2, dtype=torch.float32, device=DEV)
    phi = torch.zeros_like(dev(div))
    K.solve_pressure_jacobi3d(phi, dev(div), 0.1, np.float32(1e-2), None, 6, resid_every=3, resid_out=res)
    got = host(res)
    for k in (1, 2):
        a = oracle.jacobi3d(div, h=0.1, dt=np.float32(1e-2), iters=3 * k)
        b = oracle.jacobi3d(div, h=0.1, dt=np.float32(1e-2), iters=3 * k - 1)
        assert got[k - 1] == np.abs(a - b).max()


@pytest.mark.parametrize("n", [512, 1024])
def test_jacobi3d_full_size_bitexact(n):
    """Configs 3 and 5 at full size (512^3, 1024^3 fp32): two sweeps vs the oracle."""
    iters = 2
    rng = np.random.default_rng(1234)
    div = rng.standard_normal((n, n, n), dtype=np.float32)
    ref = oracle.jacobi3d(div, h=1.0 / (n - 1), dt=np.float32(5e-5), iters=iters)
    phi = torch.zeros((n, n, n), dtype=torch.float32, device=DEV)
    d = dev(div)
    del div
    K.solve_pressure_jacobi3d(phi, d, 1.0 / (n - 1), np.float32(5e-5), None, iters)
    assert np.array_equal(host(phi), ref)


def test_jacobi3d_variants_agree_at_1024():
    """Every kernel variant and tile gives the same bits (30 sweeps, 1024^3)."""
    n = 1024
    g = torch.Generator(device=DEV).manual_seed(7)
    div = torch.randn((n, n, n), generator=g, device=DEV, dtype=torch.float32)
    outs = []
    for cfgv, tb, *pf in [((1, 4, 0), 1), ((2, 4, 0), 1), ((1, 8, 64), 1), ((2, 16, 0), 1), ((0, 0, 0), 2),
                     ((0, 0, 0), (2, 18, 0)), ((0, 0, 0), (2, 16, 40)), ((0, 0, 0), 3),
                     ((0, 0, 0), 4), ((0, 0, 0), (3, 0, 70)), ((0, 0, 0), (3, 0, 0), 2),
                     ((0, 0, 0), (4, 0, 0), 2), ((0, 0, 0), (3, 18, 0)), ((0, 0, 0), (3, 17, 0)),
                     ((0, 0, 0), (4, 14, 0)), ((0, 0, 0), (4, 15, 0), 1)]:
        call("cfd_set_jacobi3d_config", *cfgv)
        call("cfd_set_jacobi3d_blocking", *(tb if isinstance(tb, tuple) else (tb, 0, 0)))
        call("cfd_set_jacobi3d_prefetch", pf[0] if pf else 0)
        phi = torch.zeros_like(div)
        K.solve_pressure_jacobi3d(phi, div, 1.0 / (n - 1), np.float32(5e-5), None, 30)
        if outs:
            assert torch.equal(phi, outs[0]), (cfgv, tb, pf)
        else:
            outs.append(phi)


# ------------------------------------------------------------- red-black GS
def _gs_fused(on):
    """fused (one out-of-place pass per iteration) or in-place colour passes"""
    call("cfd_set_jacobi2d_blocking", 0 if on else 1)
    call("cfd_set_jacobi3d_blocking", 0 if on else 1, 0, 0)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("name", ["rbgs2d_f32_64x64_it20_seed7", "rbgs2d_f32_64x64_it20_seed7_mask",
                                  "rbgs2d_f32_48x80_it15_aniso", "rbgs2d_f32_24x24_earlyexit"])
def test_rbgs2d_golden_bitexact(golden, name, fused):
    _gs_fused(fused)
    d = golden(name + ".npz")
    phi = torch.zeros_like(dev(d["div"]))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = K.solve_pressure_gauss_seidel_fast(phi, dev(d["div"]), float(d["dx"]), float(d["dy"]), d["dt"],
                                             dev(d["mask"]), int(d["iters"]), float(d["tol"]),
                                             iters_done=done)
    assert out is phi  # in place, same object (v5.py:223,226)
    assert np.array_equal(host(phi), d["phi"])
    n = int(host(done)[0])
    assert n == int(d["iters_done"]) if "iters_done" in d else n == int(d["iters"])


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("shape", [(31, 45), (31, 44), (64, 128), (5, 4), (130, 520), (3, 8), (2050, 2048)])
def test_rbgs2d_random_bitexact(shape, fused):
    """Small grids run the preloaded two-row fused kernel, 2050 x 2048 the row
    march (rbgs2d_tb); both bit-identical to the serial oracle."""
    _gs_fused(fused)
    rng = np.random.default_rng(4)
    div = rng.standard_normal(shape).astype(np.float32)
    phi0 = rng.standard_normal(shape).astype(np.float32)
    mask = rng.random(shape) < 0.1
    ref, n_ref = oracle.rbgs2d(div, phi0, dx=0.03, dy=0.05, dt=np.float32(1e-3), iters=25, tol=1e-8,
                               mask=mask)
    phi = dev(phi0)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.03, 0.05, np.float32(1e-3), dev(mask), 25, 1e-8,
                                       iters_done=done)
    assert np.array_equal(host(phi), ref)
    assert int(host(done)[0]) == n_ref


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("tol", [3e-5, 1.5e-5])  # stops after 17 / 62 iterations
def test_rbgs2d_early_exit_both_parities(fused, tol):
    """The stop iteration decides which ping-pong buffer holds the result
    (decided on device by the finishing kernel)."""
    _gs_fused(fused)
    rng = np.random.default_rng(12)
    div = rng.standard_normal((66, 132)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs2d(div, np.zeros_like(div), dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=400,
                               tol=tol)
    assert 1 < n_ref < 400
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), None, 400, tol,
                                       iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("shape", [(9, 10, 12), (14, 17, 33), (14, 17, 32), (21, 30, 264), (3, 3, 4)])
def test_rbgs3d_random_bitexact(shape, masked, fused):
    _gs_fused(fused)
    rng = np.random.default_rng(6)
    div = rng.standard_normal(shape).astype(np.float32)
    mask = (rng.random(shape) < 0.1) if masked else None
    ref, n_ref = oracle.rbgs3d(div, dx=0.1, dy=0.12, dz=0.09, dt=np.float32(1e-2), iters=9, tol=1e-8,
                               mask=mask)
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel3d(phi, dev(div), 0.1, 0.12, 0.09, np.float32(1e-2),
                                    None if mask is None else dev(mask), 9, 1e-8, iters_done=done)
    assert np.array_equal(host(phi), ref)
    assert int(host(done)[0]) == n_ref


# (blocking steps, rows): tall tiles with one iteration per pass (steps 2; the
# 16- and 20-row shapes explicitly), one and a half (steps 3: passes that end
# inside an iteration), two (steps 4, and 0 = auto)
GS_FUSED = [(2, 16), (2, 20), (0, 0), (2, 0), (3, 0), (4, 0)]


@pytest.mark.parametrize("steps,rows", GS_FUSED)
@pytest.mark.parametrize("zchunk", [0, 3, 1])
@pytest.mark.parametrize("prefetch", [1, 2])
@pytest.mark.parametrize("iters", [7, 8])
def test_rbgs3d_fused_tiles_bitexact(steps, rows, zchunk, prefetch, iters):
    """Tile shapes of the fused passes: both kernels, 1..3 planes per march,
    both prefetch depths, odd / even iteration counts (the result is copied
    back from phi_tmp on the device when it ends there)."""
    call("cfd_set_jacobi3d_blocking", steps, rows, zchunk)
    call("cfd_set_jacobi3d_prefetch", prefetch)
    rng = np.random.default_rng(8)
    div = rng.standard_normal((19, 45, 264)).astype(np.float32)
    ref, n_ref = oracle.rbgs3d(div, dx=0.1, dy=0.1, dz=0.1, dt=np.float32(1e-2), iters=iters, tol=0.0)
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel3d(phi, dev(div), 0.1, 0.1, 0.1, np.float32(1e-2), None, iters, 0.0,
                                    iters_done=done)
    assert n_ref == iters and int(host(done)[0]) == iters
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("steps,rows", GS_FUSED)
@pytest.mark.parametrize("tol", [2e-5, 1.5e-5, 1e-5])  # stops after 6 / 7 / 11 iterations
def test_rbgs3d_early_exit_fused(steps, rows, tol):
    """A stop inside a pass (an odd count at two iterations per pass; any count
    whose 2c half-sweeps end inside a pass of three) is rolled back on the
    device; the count and field match the oracle."""
    call("cfd_set_jacobi3d_blocking", steps, rows, 0)
    rng = np.random.default_rng(13)
    div = rng.standard_normal((24, 26, 40)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2), iters=300, tol=tol)
    assert 1 < n_ref < 300
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel3d(phi, dev(div), 0.05, 0.05, 0.05, np.float32(1e-2), None, 300, tol,
                                    iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


def test_rbgs3d_fused_matches_colour_passes_at_512():
    """Full-size property check (the oracle is too slow here): the fused pass
    and the in-place colour passes agree bitwise, iteration count included."""
    n = 512
    g = torch.Generator(device=DEV).manual_seed(3)
    div = torch.randn((n, n, n), device=DEV, generator=g)
    outs = []
    for steps in (1, 0, 2, 4):
        call("cfd_set_jacobi3d_blocking", steps, 0, 0)
        phi = torch.zeros_like(div)
        done = torch.zeros(1, dtype=torch.int32, device=DEV)
        h = 1.0 / (n - 1)
        K.solve_pressure_gauss_seidel3d(phi, div, h, h, h, np.float32(5e-5), None, 6, 0.0, iters_done=done)
        outs.append((phi, int(host(done)[0])))
    assert all(o[1] == 6 for o in outs)
    assert all(torch.equal(outs[0][0], o[0]) for o in outs[1:])


# ------------------------------------------------------------- predictor & co
def test_predictor_components_vs_reference(golden):
    d = golden("predictor2d_f32_40x56_seed3.npz")
    dx, dy, dt = float(d["dx"]), float(d["dy"]), d["dt"]
    u, v, nu = dev(d["u"]), dev(d["v"]), dev(d["nu_eff"])
    tau = K.compute_supg_stabilization_fast(u, v, dx, dy, dt, nu)
    assert np.array_equal(host(tau), d["tau"])
    # with the reference's own tau the convection is bit-exact
    tref = dev(d["tau"])
    assert np.array_equal(host(K.compute_convection_supg_fast(u, v, u, dx, dy, tref)), d["conv_u"])
    assert np.array_equal(host(K.compute_convection_supg_fast(u, v, v, dx, dy, tref)), d["conv_v"])
    assert np.array_equal(host(K.compute_convection_fast(u, v, u, dx, dy)), d["conv_u_upwind"])
    assert np.array_equal(host(K.compute_convection_fast(u, v, v, dx, dy)), d["conv_v_upwind"])
    assert np.array_equal(host(K.compute_laplacian_fast(u, dx, dy, nu)), d["lap_u"])
    assert np.array_equal(host(K.compute_laplacian_fast(v, dx, dy, float(d["nu_eff"][0, 0]))), d["lap_v"])
    us, vs, t2 = K.predictor_fused(u, v, dx, dy, dt, nu, use_supg=True)
    assert np.array_equal(host(us), d["u_star"]) and np.array_equal(host(vs), d["v_star"])
    assert np.array_equal(host(t2), d["tau"])
    us, vs, _ = K.predictor_fused(u, v, dx, dy, dt, float(d["nu_eff"][0, 0]), use_supg=False)
    assert np.array_equal(host(us), d["u_star_upwind"]) and np.array_equal(host(vs), d["v_star_upwind"])
    div = K.compute_divergence_fast(dev(d["u_star"]), dev(d["v_star"]), dx, dy)
    assert np.array_equal(host(div), d["div"])
    gx, gy = K.compute_gradient_fast(dev(d["u_star"]), dx, dy)
    assert np.array_equal(host(gx), d["grad_x"]) and np.array_equal(host(gy), d["grad_y"])


def test_project_and_clean_divergence_bitexact(golden):
    d = golden("step_v5_120x36_n3_gs.npz")
    c = OptimizedTurbulentConfig(nx=120, ny=36)
    phi, us, vs = d["phi1"], d["u_star1"], d["v_star1"]
    dt = d["dt0"]
    gx, gy = oracle.gradient2d(phi, dx=c.dx, dy=c.dy)
    u_ref, v_ref = us - dt * gx, vs - dt * gy
    u, v = K.project_velocity(dev(phi), dev(us), dev(vs), c.dx, c.dy, dt)
    assert np.array_equal(host(u), u_ref) and np.array_equal(host(v), v_ref)
    cu, cv = oracle.clean_divergence2d(u_ref, v_ref, dx=c.dx, dy=c.dy, iterations=2)
    K.clean_divergence_fast(u, v, c.dx, c.dy, iterations=2)
    assert np.array_equal(host(u), cu) and np.array_equal(host(v), cv)


@pytest.mark.parametrize("ny,nx", [(3, 3), (3, 50), (4, 7), (66, 30), (67, 30), (130, 17), (180, 600),
                                   (194, 33), (258, 70), (322, 51), (323, 20), (36, 1200),
                                   (514, 9), (515, 9), (1030, 40), (1027, 64), (2060, 66), (130, 131),
                                   (70, 1023), (1100, 97), (300, 66), (130, 67),
                                   (200, 50000), (66, 45000)])
def test_clean_divergence_lexicographic_shapes(ny, nx):
    """The serial lexicographic phi sweep of clean_divergence_fast (v5.py:250-253)
    on ragged shapes: one and several waves per band, a band edge inside a wave,
    a single-row last band (row above and below both from memory), several bands;
    one and two iterations.  nx >= 64 takes the diagonal wavefront (bands of up
    to 1024 rows, 16 waves): 1027 and 2060 rows end in a one- and a ten-row band.
    Short, very wide grids (200 x 50000, 66 x 45000) run one wave per band,
    whose launch needs no dynamic LDS (r05 advisor: it asked for more than a CU
    holds and failed)."""
    rng = np.random.default_rng(ny * 1000 + nx)
    u0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    v0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    dx, dy = 20.0 / (nx - 1), 6.0 / (ny - 1)
    cu, cv = oracle.clean_divergence2d(u0, v0, dx=dx, dy=dy, iterations=2)
    u, v = dev(u0), dev(v0)
    K.clean_divergence_fast(u, v, dx, dy, iterations=2)
    assert np.array_equal(host(u), cu) and np.array_equal(host(v), cv)
    cu1, cv1 = oracle.clean_divergence2d(u0, v0, dx=dx, dy=dy, iterations=1)
    u, v = dev(u0), dev(v0)
    K.clean_divergence_fast(u, v, dx, dy, iterations=1)
    assert np.array_equal(host(u), cu1) and np.array_equal(host(v), cv1)


def test_bc_ibm_clip_bitexact(golden):
    d = golden("step_v5_120x36_n3_gs.npz")
    c = OptimizedTurbulentConfig(nx=120, ny=36)
    y = np.linspace(c.y_min, c.y_max, c.ny)
    o = oracle.OracleSolver(c, d["u1"], d["v1"], d["cylinder_mask"], d["ibm_mask"], y)
    for step in (0, 7, 1500):
        o.step = step
        uu, vv = d["u2"].copy(), d["v2"].copy()
        o.apply_boundary_conditions(uu, vv)
        u, v = dev(d["u2"]), dev(d["v2"])
        call("cfd_apply_bc2d_f32", ptr(u), ptr(v), ptr(dev(y)), c.ny, c.nx, float(c.y_max), float(c.V_inf),
             step, stream_handle())
        assert rel_linf(host(u), uu) <= 1e-7 and np.array_equal(host(v), vv)
        fs = min(1.0, step / c.initial_steps)
        o.apply_ibm(uu, vv, fs)
        u, v = dev(uu), dev(vv)
        uu2, vv2 = uu.copy(), vv.copy()
        o.apply_ibm(uu2, vv2, fs)
        K.apply_ibm_fast(u, v, dev(d["ibm_mask"]), fs)
        assert np.array_equal(host(u), uu2) and np.array_equal(host(v), vv2)
    a = np.array([-9, -5, -1, 0, 2, 5, 7, np.nan], np.float32)
    t = dev(a)
    call("cfd_clip_f32", ptr(t), t.numel(), -5.0, 5.0, stream_handle())
    assert np.array_equal(host(t), np.clip(a, -5, 5), equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("ny,nx", [(36, 120), (7, 2), (5, 3), (300, 257)])
def test_fused_step_tails_match_separate_calls(dtype, ny, nx):
    """The solver step's fused tails are the separate calls in the reference's
    order, bit for bit: apply_bc_ibm2d == apply_bc2d then apply_ibm2d (mask
    values on every edge row and column, so the outlet copy's source is itself
    forced), energy_mean_clip2d == energy_mean2d then two clips."""
    sfx = "_f32" if dtype == torch.float32 else "_f64"
    rng = np.random.default_rng(ny * 7 + nx)
    npd = np.float32 if dtype == torch.float32 else np.float64
    u0 = (rng.uniform(-3, 3, (ny, nx))).astype(npd)
    v0 = (rng.uniform(-3, 3, (ny, nx))).astype(npd)
    m = np.where(rng.uniform(size=(ny, nx)) < 0.4, rng.uniform(0, 1, (ny, nx)), 0.0)
    m[:, -2:] = rng.uniform(0.1, 1, (ny, 2))
    m[0, :] = 0.5
    # device inputs stay referenced until the kernels have run (a temporary's
    # block can be reused by the next host-to-device copy)
    yd, md = dev(np.linspace(-2.0, 2.0, ny)), dev(m)
    s = stream_handle()
    for step, mask in ((0, md), (7, md), (1500, None)):
        fs = min(1.0, step / 1000)
        a_u, a_v = dev(u0), dev(v0)
        call("cfd_apply_bc2d" + sfx, ptr(a_u), ptr(a_v), ptr(yd), ny, nx, 2.0, 1.0, step, s)
        if mask is not None:
            call("cfd_apply_ibm2d" + sfx, ptr(a_u), ptr(a_v), ptr(mask), ny * nx, fs, s)
        b_u, b_v = dev(u0), dev(v0)
        call("cfd_apply_bc_ibm2d" + sfx, ptr(b_u), ptr(b_v), ptr(yd), ny, nx, 2.0, 1.0, step,
             ptr(mask) if mask is not None else None, fs, s)
        assert np.array_equal(host(a_u), host(b_u)) and np.array_equal(host(a_v), host(b_v)), step
    u0[0, 0] = np.nan
    e1 = torch.zeros(1, dtype=torch.float64, device="cuda")
    e2 = torch.zeros(1, dtype=torch.float64, device="cuda")
    a_u, a_v = dev(u0), dev(v0)
    call("cfd_energy_mean2d" + sfx, ptr(a_u), ptr(a_v), a_u.numel(), ptr(e1), s)
    call("cfd_clip" + sfx, ptr(a_u), a_u.numel(), -2.0, 2.0, s)
    call("cfd_clip" + sfx, ptr(a_v), a_v.numel(), -2.0, 2.0, s)
    u0[0, 0] = 0.25
    for uu in (u0,):
        b_u, b_v = dev(uu), dev(v0)
        call("cfd_energy_mean_clip2d" + sfx, ptr(b_u), ptr(b_v), b_u.numel(), ptr(e2), -2.0, 2.0, s)
        ref_u = np.clip(uu, -2, 2)
        assert np.array_equal(host(b_u), ref_u) and np.array_equal(host(b_v), host(a_v))
    assert np.isnan(host(e1)[0]) and np.array_equal(host(a_u)[1:], host(b_u)[1:])
    # with the NaN cell replaced the fused energy equals the separate one
    c_u, c_v = dev(u0), dev(v0)
    call("cfd_energy_mean2d" + sfx, ptr(c_u), ptr(c_v), c_u.numel(), ptr(e1), s)
    assert host(e1)[0] == host(e2)[0]


@pytest.mark.parametrize("branch", ["gs", "jacobi"])
def test_time_step_vs_reference(golden, branch):
    """Three OptimizedTurbulentSolver.time_step() calls vs the reference's:
    every field bit-exact, and the logged diagnostics (v5.py:410, 415, 422,
    428) exactly the reference's values."""
    d = golden(f"step_v5_120x36_n3_{branch}.npz")
    g = golden(f"diag_v5_120x36_n3_{branch}.npz")
    c = OptimizedTurbulentConfig(nx=120, ny=36, pressure_iterations=200,
                                 use_fast_pressure=(branch == "gs"), log_diagnostics=True)
    s = OptimizedTurbulentSolver(c)
    assert np.array_equal(host(s.u), d["u0"]) and np.array_equal(host(s.v), d["v0"])
    for k in range(3):
        dt = s.time_step()
        assert np.float32(dt) == d[f"dt{k}"]
        for f, t in (("u", s.u), ("v", s.v), ("phi", s.phi), ("u_star", s.u_star), ("v_star", s.v_star),
                     ("div", s.div_u_star), ("tau", s.tau_supg)):
            assert np.array_equal(host(t), d[f"{f}{k + 1}"]), (f, k)
        diag = s.diagnostics
        for key in ("pre_div_max", "grad_max", "post_div_max", "vorticity_max"):
            assert np.float32(diag[key]) == g[key][k], (key, k)
        assert rel_linf(diag["energy_mean"], g["energy"][k]) <= 1e-6
    e = np.array([v for _, v in s.energy_history])
    assert np.allclose(e, d["energy"], rtol=1e-6, atol=0)


# ------------------------------------------------------------- slabs
def test_slab_sweeps_emulated_on_one_gpu():
    """The slab driver's building block (cfd_jacobi3d_sweep_f32 on local
    arrays with ghost planes) with the SlabPlan exchange list, emulated on
    one GPU for 3 slabs: bit-identical to the single-domain solve."""
    nz, ny, nx, iters, R = 23, 18, 36, 6, 3
    rng = np.random.default_rng(9)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.07, dt=np.float32(4e-3), iters=iters)
    plans = [S.SlabPlan(nz, R, r) for r in range(R)]
    A = [dev(p.scatter(np.zeros_like(div))) for p in plans]
    B = [a.clone() for a in A]
    D = [dev(p.scatter(div)) for p in plans]
    for _ in range(iters):
        for p, a, b, d_ in zip(plans, A, B, D):
            S.sweep_range(a, b, d_, None, p.z_update_begin, p.z_update_end, 0.07, np.float32(4e-3))
        for p, b in zip(plans, B):
            for first, count, peer, recv in p.exchanges():
                B[peer][recv:recv + count].copy_(b[first:first + count])
        A, B = B, A
    got = np.concatenate([host(a)[p.owned()] for p, a in zip(plans, A)])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ghost", [1, 2, 3, 4])
@pytest.mark.parametrize("overlap", [False, True])
def test_slab_rccl_single_rank(overlap, ghost):
    """The RCCL slab driver with a one-rank communicator equals the plain solve."""
    n, iters = 40, 7
    rng = np.random.default_rng(10)
    div = rng.standard_normal((n, n, n + 8)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(1e-3), iters=iters)
    comm = S.RcclComm(0, 1)
    try:
        plan = S.SlabPlan(n, 1, 0, ghost=ghost)
        sj = S.SlabJacobi3D(plan, n, n + 8, 0.05, np.float32(1e-3), comm)
        sj.div.copy_(dev(plan.scatter(div)))
        sj.solve(iters, overlap=overlap)
        assert np.array_equal(host(sj.owned()), ref)
    finally:
        comm.close()


@pytest.mark.parametrize("tol,iters", [(0.0, 7), (2e-5, 300)])
def test_slab_rbgs_passes_emulated_on_one_gpu(tol, iters):
    """The fused RB-GS slab pass (cfd_rbgs3d_pass_f32, global colour offset,
    2-deep ghosts, recomputed inner-ghost colour 0) for 3 slabs on one GPU,
    the per-iteration max combined across slabs like the ncclAllReduce:
    bit-identical to the single-domain oracle, stop iteration included."""
    nz, ny, nx, R = 23, 18, 36, 3
    dx, dy, dz, dt = 0.05, 0.06, 0.07, np.float32(1e-2)
    rng = np.random.default_rng(21)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=dx, dy=dy, dz=dz, dt=dt, iters=iters, tol=tol)
    plans = [S.SlabPlan(nz, R, r, ghost=2) for r in range(R)]
    A = [dev(p.scatter(np.zeros_like(div))) for p in plans]
    B = [a.clone() for a in A]
    D = [dev(p.scatter(div)) for p in plans]
    need = int(lib().cfd_rbgs_workspace_bytes(iters))
    W = [torch.zeros(need, dtype=torch.uint8, device=DEV) for _ in plans]
    done = [torch.zeros(1, dtype=torch.int32, device=DEV) for _ in plans]
    s = stream_handle()
    for w, dn in zip(W, done):
        call("cfd_rbgs_init", ptr(w), iters, tol, ptr(dn), s)
    for it in range(iters):
        for p, a, b, d_, w in zip(plans, A, B, D, W):
            call("cfd_rbgs3d_pass_f32", ptr(a), ptr(b), ptr(d_), p.nz_total, ny, nx, p.z_update_begin,
                 p.z_update_end, int(p.z_lo == 0), int(p.z_hi == nz), p.z_lo - p.ghost, dx, dy, dz,
                 float(dt), tol, it, ptr(w), s)
        for p, b in zip(plans, B):
            for first, count, peer, recv in p.exchanges():
                B[peer][recv:recv + count].copy_(b[first:first + count])
        # global max of iteration `it` (float32 maxc array at byte 16)
        mx = [w[16:].view(torch.float32)[it:it + 1] for w in W]
        g = torch.stack(mx).max(dim=0).values
        for m in mx:
            m.copy_(g)
        A, B = B, A
    n = []
    for p, a, b, w, dn in zip(plans, A, B, W, done):
        # A holds iteration `iters`; the buffer of iteration k alternates, so
        # finish against the START buffer (B after an odd count of swaps)
        start, other = (a, b) if iters % 2 == 0 else (b, a)
        call("cfd_rbgs_finish", ptr(w), ptr(start), ptr(other), start.numel(), ptr(dn), s)
        n.append(int(host(dn)[0]))
        A[plans.index(p)] = start
    assert n == [n_ref] * R
    if tol > 0:
        assert 1 < n_ref < iters
    got = np.concatenate([host(a)[p.owned()] for p, a in zip(plans, A)])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("ghost,steps", [(1, 0), (2, 0), (2, 2), (4, 4), (3, 0)])
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("tol", [0.0, 2e-5])
def test_slab_rbgs_rccl_single_rank(overlap, ghost, steps, tol):
    """cfd_slab_rbgs3d_f32 with a one-rank communicator equals the oracle
    (one or two iterations per fused pass, early stop included)."""
    call("cfd_set_jacobi3d_blocking", steps, 0, 0)
    nz, ny, nx, iters = 30, 26, 40, 300 if tol > 0 else 9
    rng = np.random.default_rng(11)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2), iters=iters, tol=tol)
    comm = S.RcclComm(0, 1)
    try:
        plan = S.SlabPlan(nz, 1, 0, ghost=ghost)
        sg = S.SlabRBGS3D(plan, ny, nx, 0.05, 0.05, 0.05, np.float32(1e-2), comm)
        sg.div.copy_(dev(plan.scatter(div)))
        sg.solve(iters, tolerance=tol, overlap=overlap)
        assert int(host(sg.iters_done)[0]) == n_ref
        assert np.array_equal(host(sg.owned()), ref)
    finally:
        comm.close()


@pytest.mark.parametrize("gs", [False, True])
def test_slab_rccl_self_peered_rehearsal(gs):
    """The per-rank rehearsal mode (scripts/slab_rehearsal.py --rccl-self): a
    one-rank RCCL comm named as both neighbours runs a middle rank's pass
    sequence -- boundary planes, RCCL send/recv to self on the reserved-CU
    exchange stream beside the interior (the CU partition), the GS max
    allreduce.  Its result is not a solve, but the overlapped (partitioned)
    schedule must equal the serial one bit for bit, and repeat exactly."""
    nzl, ny, nx, iters = 24, 34, 64, 10
    G = 2 if gs else 3
    rng = np.random.default_rng(5)
    div = dev(rng.standard_normal((nzl + 2 * G, ny, nx)).astype(np.float32) * np.float32(1e-3))
    comm = S.RcclComm(0, 1)
    cs = torch.cuda.Stream(priority=-1)
    ws = torch.zeros(int(lib().cfd_rbgs_workspace_bytes(iters)), dtype=torch.uint8, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    outs = []
    try:
        for overlap in (0, 1, 1):
            phi, tmp = torch.zeros_like(div), torch.zeros_like(div)
            if gs:
                call("cfd_slab_rbgs3d_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), None, nzl, G, ny, nx,
                     0, 0, G, nzl + G, 100, 0.05, 0.05, 0.05, 1e-2, iters, 1e-30, ptr(ws), ptr(done),
                     overlap, stream_handle(), cs.cuda_stream)
            else:
                rhs = torch.empty_like(div)
                call("cfd_slab_jacobi3d_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), ptr(rhs), None, nzl,
                     G, ny, nx, 0, 0, G, nzl + G, 0.05, 1e-3, iters, overlap, stream_handle(),
                     cs.cuda_stream)
            outs.append(host(phi))
    finally:
        comm.close()
    assert np.isfinite(outs[0]).all() and np.abs(outs[0]).max() > 0
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])


@pytest.mark.parametrize("gs", [False, True])
def test_slab_copy_engine_self_peered_rehearsal(gs):
    """The copy-engine transport's rehearsal mode (scripts/slab_rehearsal.py
    --self): a one-rank comm named as both neighbours -- SDMA copies of the
    boundary planes into its own ghost planes, the sequence words, the sync
    kernel's waits (and for the GS, its one-rank max gather).  Not a solve, but
    overlapped must equal serial bit for bit, repeat exactly, and no wait may
    time out."""
    nzl, ny, nx, iters = 24, 34, 64, 10
    G = 4 if gs else 3
    rng = np.random.default_rng(5)
    div = dev(rng.standard_normal((nzl + 2 * G, ny, nx)).astype(np.float32) * np.float32(1e-3))
    comm = S.CopyEngineComm(0, 1)
    phi, tmp = torch.zeros_like(div), torch.zeros_like(div)
    comm.attach(phi, tmp)
    ws = torch.zeros(int(lib().cfd_rbgs_workspace_bytes(iters)), dtype=torch.uint8, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    rhs = torch.empty_like(div)
    outs = []
    try:
        for overlap in (0, 1, 1):
            phi.zero_()
            tmp.zero_()
            if gs:
                call("cfd_slab_rbgs3d_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), None, nzl, G, ny, nx,
                     0, 0, G, nzl + G, 100, 0.05, 0.05, 0.05, 1e-2, iters, 1e-30, ptr(ws), ptr(done),
                     overlap, stream_handle(), None)
            else:
                call("cfd_slab_jacobi3d_zero_f32", comm.handle, ptr(div), ptr(phi), ptr(tmp), ptr(rhs), nzl, G,
                     ny, nx, 0, 0, G, nzl + G, 0.05, 1e-3, iters, overlap, stream_handle(), None)
            outs.append(host(phi))
        assert comm.status() == 0
    finally:
        comm.close()
    assert np.isfinite(outs[0]).all() and np.abs(outs[0]).max() > 0
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])


@pytest.mark.parametrize("ghost", [1, 2, 3, 4])
@pytest.mark.parametrize("overlap", [False, True])
def test_slab_copy_engine_single_rank(overlap, ghost):
    """cfd_slab_jacobi3d_f32 / cfd_slab_rbgs3d_f32 on a one-rank copy-engine
    comm (no neighbours: the drivers' pass sequence with nothing to send)."""
    n, iters = 40, 7
    rng = np.random.default_rng(10)
    div = rng.standard_normal((n, n, n + 8)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(1e-3), iters=iters)
    comm = S.CopyEngineComm(0, 1)
    try:
        plan = S.SlabPlan(n, 1, 0, ghost=ghost)
        sj = S.SlabJacobi3D(plan, n, n + 8, 0.05, np.float32(1e-3), comm)
        sj.div.copy_(dev(plan.scatter(div)))
        sj.solve(iters, overlap=overlap)
        assert np.array_equal(host(sj.owned()), ref)
    finally:
        comm.close()


@pytest.mark.parametrize("landing", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_slab_copy_engine_multiprocess(world, landing):
    """The copy-engine transport between real processes: `world` ranks, each
    its own process on this GPU (torch.distributed.run, gloo for the IPC
    handle blobs), mapping each other's buffers and flag blocks.  Jacobi
    (ghost 1 and 3, zero and nonzero start, overlap on / off) and red-black GS
    (one and two iterations per pass, fixed count and early stop through the
    gathered global maxima): the gathered owned planes equal the single-domain
    oracle bit for bit (scripts/multirank_check.py).  landing: every rank takes
    its ghosts through its landing buffer (CFD_CE_LANDING=1, the path of pairs
    of 2 GiB or more, which IPC cannot map: the 1024^3 grid at two ranks)."""
    import os
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + world + 10 * landing),
           str(ROOT / "scripts" / "multirank_check.py"), "--share-gpu", "--transport", "ce", "--quick", "--size", "48"]
    env = dict(os.environ)
    if landing:
        env["CFD_CE_LANDING"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(ROOT), env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "MULTIRANK OK" in out, out[-4000:]


# ------------------------------------------------- multi-rank, one GPU (threads)
def _run_local_group(R, make, run, tuning=None):
    """R ranks of an in-process slab group (cfd_comm_init_local), one host
    thread and one stream per rank, running the real slab drivers.  The
    tuning knobs are per host thread: ``tuning`` (the blocking arguments)
    is applied inside every rank's thread."""
    import threading
    comms = S.LocalComm.group(R)
    solvers = [make(r, comms[r]) for r in range(R)]
    streams = [torch.cuda.Stream() for _ in range(R)]
    torch.cuda.synchronize()
    errs = [None] * R

    def work(r):
        try:
            if tuning is not None:
                call("cfd_set_jacobi3d_blocking", *tuning)
            with torch.cuda.stream(streams[r]):
                run(solvers[r])
            streams[r].synchronize()
        except Exception as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    threads = [threading.Thread(target=work, args=(r,)) for r in range(R)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=600)
    torch.cuda.synchronize()
    for c in comms:
        c.close()
    assert not any(t.is_alive() for t in threads), "a rank hung"
    assert errs == [None] * R, errs
    return solvers


@pytest.mark.parametrize("R", [2, 3, 4])
@pytest.mark.parametrize("ghost", [1, 2, 3, 4])
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("iters", [7, 12])
def test_slab_jacobi_local_group_multirank(R, ghost, overlap, iters):
    """cfd_slab_jacobi3d_f32 with R real ranks (threads on one GPU, device
    copies for the send/recv pairs): the owned planes, gathered, equal the
    single-domain oracle bit for bit -- K-level passes, boundary-first overlap,
    remainders."""
    nz, ny, nx = 41, 30, 72
    rng = np.random.default_rng(40 + R)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    ref = oracle.jacobi3d(div, h=0.05, dt=np.float32(1e-3), iters=iters)

    def make(r, comm):
        plan = S.SlabPlan(nz, R, r, ghost=ghost)
        sj = S.SlabJacobi3D(plan, ny, nx, 0.05, np.float32(1e-3), comm)
        sj.div.copy_(dev(plan.scatter(div)))
        return sj

    sols = _run_local_group(R, make, lambda sj: sj.solve(iters, overlap=overlap))
    got = np.concatenate([host(sj.owned()) for sj in sols])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("R", [2, 3])
@pytest.mark.parametrize("ghost,steps", [(1, 0), (2, 0), (2, 2), (4, 4)])
@pytest.mark.parametrize("overlap", [False, True])
@pytest.mark.parametrize("tol,iters", [(0.0, 9), (2e-5, 300), (1.5e-5, 300)])
def test_slab_rbgs_local_group_multirank(R, ghost, steps, overlap, tol, iters):
    """cfd_slab_rbgs3d_f32 with R real ranks on one GPU: global colours, the
    global stop rule through the max-allreduce, the rollback of a stop inside
    a pair pass -- bit-identical to the oracle, same count on every rank."""
    blocking = (steps, 0, 0)
    call("cfd_set_jacobi3d_blocking", *blocking)
    nz, ny, nx = 30, 26, 40
    rng = np.random.default_rng(11)
    div = rng.standard_normal((nz, ny, nx)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2), iters=iters, tol=tol)

    def make(r, comm):
        plan = S.SlabPlan(nz, R, r, ghost=ghost)
        sg = S.SlabRBGS3D(plan, ny, nx, 0.05, 0.05, 0.05, np.float32(1e-2), comm)
        sg.div.copy_(dev(plan.scatter(div)))
        return sg

    sols = _run_local_group(R, make, lambda sg: sg.solve(iters, tolerance=tol, overlap=overlap), tuning=blocking)
    assert [int(host(sg.iters_done)[0]) for sg in sols] == [n_ref] * R
    got = np.concatenate([host(sg.owned()) for sg in sols])
    assert np.array_equal(got, ref)
