"""GPU parity at the bench geometries, and the corner cases the round-1 review
found unpinned.  All bit-exact against the oracle (BIT-EXACT bar: the Jacobi and
red-black GS paths reassociate nothing).

* The headline kernel: 1024^3 Jacobi with 4, 5 and 6 sweeps on the default
  blocking (4 sweeps per pass, the tall-tile jacobi3d_tbr<4, 11 row waves x 2
  rows> the bench runs) and 3, 4, 5 on the 3-sweep one (tbr<3, 10 x 2>), with
  and without the RHS workspace; the test asserts that these shapes ran.
* Config 5's kernel: 1024^3 red-black GS, 2 and 3 iterations on the default
  16-row tile (4 levels, 11 x 2) and on the 3-level one (10 x 2), and every
  explicit GS tile (2, 3, 4 levels) on a ragged grid, with an early stop.
* Config 4's grid: 1024 x 1024 x 512 through SlabJacobi3D with a one-rank RCCL
  communicator (3-deep ghosts, overlap on).
* The device powf behind the SUPG tau vs libm.
* 2-D RB-GS on the small-grid kernel with an odd iteration count whose stop
  falls on the first iteration of the last pair (the single-iteration tail
  launch must skip), for every small-kernel shape.

The full-size references come from the oracle's OpenMP forms (bit-identical
to the serial ones, tests/test_oracle_golden.py).
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from cfd_simulations_amd import kernels as K
from cfd_simulations_amd import slab as S
from cfd_simulations_amd._lib import call, lib, ptr, stream_handle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def last_shape():
    v = [ctypes.c_int() for _ in range(4)]
    call("cfd_get_last_tbr_shape", *[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)


@pytest.fixture(autouse=True)
def _reset_tuning():
    call("cfd_reset_tuning")
    yield
    call("cfd_reset_tuning")


@pytest.fixture(scope="module")
def div1024():
    n = 1024
    rng = np.random.default_rng(1234)
    return rng.standard_normal((n, n, n), dtype=np.float32)


# ------------------------------------------------------------- north star
def test_jacobi3d_1024_headline_kernel_bitexact(div1024):
    """1024^3, h = 1/1023, dt = 5e-5 (the bench's grid and constants), with and
    without the RHS workspace (the bench uses it).  Default blocking (4 sweeps
    per pass, tbr<4, 11 row waves x 2 rows>): 4, 5 and 6 sweeps -- one pass;
    a 3-sweep first pass and a 2-sweep remainder; a 2-sweep first pass and a
    tbr<4> pass.  Three sweeps per pass (tbr<3, 10 x 2>): 3, 4 and 5."""
    n = 1024
    h, dt = 1.0 / (n - 1), np.float32(5e-5)
    assert int(lib().cfd_get_jacobi3d_levels()) == 4
    ref = {3: oracle.jacobi3d(div1024, h=h, dt=dt, iters=3, mt=True)}
    for it in (4, 5, 6):
        ref[it] = oracle.jacobi3d(div1024, ref[it - 1], h=h, dt=dt, iters=1, mt=True)
    d = dev(div1024)
    phi = torch.zeros_like(d)
    tmp = torch.empty_like(d)
    for levels, shape in ((0, (4, 11, 2, n - 2)), (3, (3, 10, 2, n - 2))):
        call("cfd_set_jacobi3d_blocking", levels, 0, 0)
        k = levels or 4
        for rhs in (torch.empty_like(d), None):
            for iters in (k, k + 1, k + 2):
                phi.zero_()
                K.solve_pressure_jacobi3d(phi, d, h, dt, None, iters, phi_tmp=tmp, rhs_ws=rhs)
                if iters == k:  # the bench's kernel for this depth, one z-chunk
                    assert last_shape() == shape, last_shape()
                assert np.array_equal(host(phi), ref[iters]), (levels, iters, rhs is None)


def test_rbgs3d_1024_default_tile_bitexact(div1024):
    """Config 5's kernel at full size: 2 and 3 red-black iterations (tolerance
    1e-8, no stop) on the default tile -- four half-sweeps per pass on the
    16-row 4-level tile (11 row waves x 2 rows; 3 iterations = a 4-level pass
    and a 2-level one) -- and on the 3-level tile (passes of colours 0,1,0
    then 1(,0,1)), phi_tmp ping-pong with the result copied back on the
    device."""
    n = 1024
    h, dt = 1.0 / (n - 1), np.float32(5e-5)
    ref2, n2 = oracle.rbgs3d(div1024, dx=h, dy=h, dz=h, dt=dt, iters=2, tol=1e-8, mt=True)
    ref3, n3 = oracle.rbgs3d(div1024, ref2, dx=h, dy=h, dz=h, dt=dt, iters=1, tol=1e-8, mt=True)
    assert n2 == 2 and n3 == 1
    d = dev(div1024)
    phi = torch.zeros_like(d)
    tmp = torch.empty_like(d)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    assert int(lib().cfd_get_rbgs3d_levels()) == 4
    for levels in (0, 3):
        call("cfd_set_jacobi3d_blocking", levels, 0, 0)
        for iters, ref in ((2, ref2), (3, ref3)):
            for tol in (1e-8, 0.0):  # tol 0: no stop possible, no rollback launch after the passes
                phi.zero_()
                K.solve_pressure_gauss_seidel3d(phi, d, h, h, h, dt, None, iters, tol, iters_done=done,
                                                phi_tmp=tmp)
                if tol == 0.0 and iters == (2 if levels == 0 else 3):
                    assert last_shape()[:3] == ((4, 11, 2) if levels == 0 else (3, 10, 2)), last_shape()
                assert int(host(done)[0]) == iters
                assert np.array_equal(host(phi), ref), (levels, iters)


@pytest.mark.parametrize("levels,rows,shape", [(2, 16, (2, 9, 2)), (2, 18, (2, 10, 2)), (2, 20, (2, 11, 2)),
                                               (2, 28, (2, 10, 3)), (3, 16, (3, 10, 2)), (3, 18, (3, 11, 2)),
                                               (4, 15, (4, 7, 3)), (4, 16, (4, 11, 2))])
@pytest.mark.parametrize("tol,iters", [(0.0, 6), (1.5e-5, 300)])
def test_rbgs3d_explicit_gs_tiles_ragged(levels, rows, shape, tol, iters):
    """Every GS tile shape (half-sweeps per pass 2, 3, 4) on a ragged grid (y
    and z not multiples of the tile, two x-segments), fixed count and early
    stop."""
    call("cfd_set_jacobi3d_blocking", levels, rows, 0)
    rng = np.random.default_rng(rows)
    div = rng.standard_normal((29, 53, 264)).astype(np.float32) * np.float32(1e-3)
    ref, n_ref = oracle.rbgs3d(div, dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2), iters=iters, tol=tol)
    if tol > 0:
        assert 1 < n_ref < iters
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel3d(phi, dev(div), 0.05, 0.05, 0.05, np.float32(1e-2), None, iters, tol,
                                    iters_done=done, phi_tmp=torch.empty_like(phi))
    if tol == 0.0:  # 12 half-sweeps: whole passes of 2, 3 and 4, no rollback launch
        assert last_shape()[:3] == shape, last_shape()
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("iters", [4, 9, 10])
def test_channel_1024x1024x512_slab_rccl_bitexact(iters):
    """Config 4's grid (nz = 512, ny = nx = 1024) through the RCCL slab driver
    with a one-rank communicator: 3-deep ghosts, blocked passes (9 sweeps =
    three full tall-tile passes; 10 = three and a remainder), overlap on."""
    nz, ny, nx = 512, 1024, 1024
    h, dt = 1.0 / (nx - 1), np.float32(5e-5)
    rng = np.random.default_rng(77)
    div = rng.standard_normal((nz, ny, nx), dtype=np.float32)
    ref = oracle.jacobi3d(div, h=h, dt=dt, iters=iters, mt=True)
    comm = S.RcclComm(0, 1)
    try:
        plan = S.SlabPlan(nz, 1, 0, ghost=3)
        sj = S.SlabJacobi3D(plan, ny, nx, h, dt, comm)
        sj.div[plan.owned()].copy_(dev(div))
        del div
        sj.solve(iters, overlap=True)
        assert np.array_equal(host(sj.owned()), ref)
    finally:
        comm.close()


def test_jacobi3d_512_bench_step_200_sweeps_bitexact():
    """Config 3's whole bench step at full size: phi = 0 and 200 sweeps
    (cfd_jacobi3d_zero_f32: the fused first pass of 4 sweeps, then 49 passes
    of jacobi3d_tbr<4> on the cost model's 512^3 shape -- 16-row tiles, four
    z-chunks of 128 planes, 256 workgroups) against the oracle's 200 sweeps
    (OpenMP form, bit-identical to the serial one)."""
    n, iters = 512, 200
    h, dt = 1.0 / (n - 1), np.float32(5e-5)
    rng = np.random.default_rng(512)
    div = rng.standard_normal((n, n, n), dtype=np.float32)
    ref = oracle.jacobi3d(div, h=h, dt=dt, iters=iters, mt=True)
    d = dev(div)
    del div
    phi = torch.empty_like(d)
    tmp, rhs = torch.empty_like(d), torch.empty_like(d)
    K.solve_pressure_jacobi3d_zero(phi, d, h, dt, iters, phi_tmp=tmp, rhs_ws=rhs)
    assert last_shape() == (4, 11, 2, 128), last_shape()
    assert np.array_equal(host(phi), ref)


# ------------------------------------------------------------- device powf
@pytest.mark.parametrize("y", [2.0, 0.5])
def test_device_powf_is_libm(y):
    """cfd_numpy_powf_f32 (the device glibc powf of the SUPG tau) equals libm
    powf -- NumPy's float32 scalar `**` -- on random bit patterns, the values
    where powf(x, 2) is not x*x, subnormals, zeros, infinities and NaN."""
    rng = np.random.default_rng(int(y * 10))
    bits = rng.integers(0, 2 ** 32, 1 << 22, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    extra = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, 1e-38, 3.4e38, 5.0, 0.1],
                     np.float32)
    vel = rng.uniform(-5, 5, 1 << 20).astype(np.float32)
    # values whose exact square / root lies near a float rounding midpoint:
    # the exact-path forms (powf_sq / powf_sqrt) hand these to the full powf
    cand = rng.uniform(0.01, 8.0, 1 << 22).astype(np.float32)
    d = cand.astype(np.float64) ** 2 if y == 2.0 else np.sqrt(cand.astype(np.float64))
    lo = (d.view(np.uint64) & np.uint64((1 << 29) - 1)).astype(np.int64) - (1 << 28)
    near = cand[np.abs(lo) < 2_000_000]
    assert near.size > 1000
    x = np.concatenate([x, extra, vel, vel * vel, near])
    if y == 0.5:
        x = np.abs(x)
    ref = oracle.numpy_powf(x, y)
    out = torch.empty(x.size, dtype=torch.float32, device=DEV)
    xd = dev(x)
    call("cfd_numpy_powf_f32", ptr(xd), float(y), ptr(out), x.size, stream_handle())
    got = host(out)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), x[~same][:8]
    if y == 2.0:
        sq = ref[-2 * vel.size - near.size:-vel.size - near.size]
        assert (sq != vel * vel).any()  # the case a plain u*u misses


@pytest.mark.parametrize("y", [2.0, 0.5])
def test_device_pow_f64_is_libm(y):
    """cfd_numpy_pow_f64 (the device glibc pow of the float64 SUPG tau)
    equals libm pow -- NumPy's float64 scalar `**` -- on random bit patterns,
    velocity-like values and their squares (where pow(x, 2) != x*x and
    pow(x, 0.5) != sqrt(x) now and then), subnormals, zeros, infinities, NaN."""
    rng = np.random.default_rng(int(y * 10) + 7)
    x = rng.integers(0, 2 ** 63, 1 << 21, dtype=np.uint64).view(np.float64)
    extra = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 5e-324, 1e-310, 2.2e-308, 1.7e308, 5.0, 0.1])
    vel = rng.uniform(-5, 5, 1 << 20)
    x = np.concatenate([x, -x[: x.size // 2], extra, vel, vel * vel])
    if y == 0.5:
        x = np.abs(x)
    ref = oracle.numpy_pow(x, y)
    out = torch.empty(x.size, dtype=torch.float64, device=DEV)
    xd = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    call("cfd_numpy_pow_f64", ptr(xd), float(y), ptr(out), x.size, stream_handle())
    got = host(out)
    same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), x[~same][:8]
    naive = vel * vel if y == 2.0 else np.sqrt(np.abs(vel))
    tail = ref[-2 * vel.size:-vel.size] if y == 2.0 else ref[-2 * vel.size:-vel.size]
    assert (tail != naive).any()  # the cases a correctly rounded form misses


# ------------------------------------------------- 2-D RB-GS, odd tail + stop
def _stop_at_first_of_last_pair():
    """A small grid and tolerance whose oracle stop falls on iteration s (0-based,
    s even, so with N = s + 3 odd it is the first iteration of the last pair
    before the single tail launch) while iteration s + 1's max|change| stays
    at or above the tolerance: max|change| is not monotone once float32 GS
    reaches rounding noise."""
    for seed in range(40):
        rng = np.random.default_rng(seed)
        div = rng.standard_normal((20, 36)).astype(np.float32) * np.float32(1e-2)
        _, _, mc = oracle.rbgs2d_maxc(div, dx=0.1, dy=0.1, dt=np.float32(1.0), iters=3000, tol=0.0)
        run_min = np.minimum.accumulate(mc)
        for s in range(2, len(mc) - 1, 2):
            lo, hi = mc[s], min(run_min[s - 1], mc[s + 1])
            if lo < hi:
                tol = float(np.float32((np.float64(lo) + np.float64(hi)) / 2))
                if lo < np.float32(tol) <= hi:
                    return div, tol, s
    pytest.skip("no non-monotone max|change| found")


@pytest.mark.parametrize("shape", [(0, 0, 0), (1, 1, 4), (1, 2, 16), (4, 1, 4), (4, 2, 4)])
def test_rbgs2d_small_odd_tail_stop_in_last_pair(shape):
    """N odd, stop at iteration N - 3 (the first of the last pair), iteration
    N - 2 above the tolerance: the single-iteration tail launch must skip, or it
    overwrites the pair's input that the rollback re-reads.  Every
    small-kernel shape: (cells per lane, rows per wave, waves per workgroup)."""
    vec, rw, wpb = shape
    call("cfd_set_small2d_shape", 0, 0, 0, rw, vec, wpb)
    call("cfd_set_small2d_gs_iters", 2, 1)  # the per-wave kernel, iteration pairs
    div, tol, s = _stop_at_first_of_last_pair()
    N = s + 3
    ref, n_ref = oracle.rbgs2d(div, dx=0.1, dy=0.1, dt=np.float32(1.0), iters=N, tol=tol)
    assert n_ref == s + 1 and N % 2 == 1
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.1, 0.1, np.float32(1.0), None, N, tol, iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("shape", [(1, 1, 4), (1, 2, 16), (4, 1, 4), (4, 2, 4), (4, 2, 16)])
@pytest.mark.parametrize("iters,tol", [(25, 1e-8), (400, 3e-5), (401, 1.5e-5)])
def test_rbgs2d_small_shapes_bitexact(shape, iters, tol):
    """The non-default small-grid GS instantiations (set per thread through
    cfd_set_small2d_shape) stay bit-exact: masks, early stops of both
    parities, odd counts."""
    vec, rw, wpb = shape
    call("cfd_set_small2d_shape", 0, 0, 0, rw, vec, wpb)
    call("cfd_set_small2d_gs_iters", 2, 1)  # the per-wave kernel (the default shares rows)
    rng = np.random.default_rng(12)
    div = rng.standard_normal((66, 132)).astype(np.float32) * np.float32(1e-3)
    mask = rng.random(div.shape) < 0.05
    ref, n_ref = oracle.rbgs2d(div, dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=iters, tol=tol, mask=mask)
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), dev(mask), iters, tol,
                                       iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("persistent", [1, 2, 3])
@pytest.mark.parametrize("ni", [2, 3, 4, 5])
@pytest.mark.parametrize("iters,tol", [(37, 0.0), (400, 3e-5), (401, 1.5e-5)])
def test_rbgs2d_shared_rows_cylinder_grid(ni, iters, tol, persistent):
    """The shared-row small-grid GS with 2..5 iterations per block on the v5
    cylinder's grid shape, one launch per block (rbgs2d_wg, persistent = 1,
    at most 4 per launch) or the whole solve as one persistent launch
    (rbgs2d_persist, 2, the default; 5 per block, 210 tiles, is its default
    here): several tiles in x and y, solid cells, counts not a multiple of
    the block depth, early stops of both parities."""
    call("cfd_set_small2d_gs_iters", ni, 2)
    call("cfd_set_small2d_gs_persistent", persistent)
    rng = np.random.default_rng(31 + ni)
    div = rng.standard_normal((180, 600)).astype(np.float32) * np.float32(1e-3)
    mask = rng.random(div.shape) < 0.03
    ref, n_ref = oracle.rbgs2d(div, dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=iters, tol=tol, mask=mask)
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), dev(mask), iters, tol,
                                       iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("k,rw,vec", [(1, 1, 1), (3, 2, 1), (5, 1, 4), (8, 2, 4), (4, 2, 1)])
def test_jacobi2d_small_shapes_bitexact(k, rw, vec):
    """The small-grid Jacobi kernel's non-default shapes (sweeps per launch
    1..8, rows per wave, cells per lane) on the cylinder case's kind of grid
    (the launch-per-pass path: the persistent solve off)."""
    call("cfd_set_small2d_shape", k, rw, vec, 0, 0, 0)
    call("cfd_set_small2d_jacobi_persistent", 1, 0)
    rng = np.random.default_rng(k)
    div = rng.standard_normal((180, 600)).astype(np.float32)
    mask = rng.random(div.shape) < 0.03
    ref = oracle.jacobi2d(div, dx=20 / 599, dt=np.float32(5e-5), iters=37, mask=mask)
    phi = torch.zeros_like(dev(div))
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), 37)
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("ni", [4, 6, 8, 10])
@pytest.mark.parametrize("shape,iters,pre", [((180, 600), 1500, True), ((180, 600), 37, False),
                                             ((36, 120), 9, True), ((53, 131), 17, False), ((3, 70), 12, True),
                                             ((97, 64), 25, False), ((53, 131), 23, True),
                                             ((180, 1200), 47, True)])
def test_jacobi2d_persistent_bitexact(ni, shape, iters, pre, mode):
    """The small-grid Jacobi as one persistent launch (jacobi2d_persist): the
    cylinder's grid at the reference's 1500 sweeps, ragged grids (tiles cut
    by the edges, one tile row, a one-row interior), sweep counts that are no
    multiple of the block (odd remainders: a last single sweep after the
    pairs), with and without the RHS workspace; the mask covers interior and
    edge cells (edge ones become 0 too, also where the edge row is a tile's
    last row), phi starts non-zero; 180 x 1200: 10 or 8 sweeps per block
    would not fit on the chip, so the solve takes 6.  mode 2: two sweeps per
    LDS exchange (the default), 3: one."""
    call("cfd_set_small2d_jacobi_persistent", mode, ni)
    rng = np.random.default_rng(ni * 1000 + iters)
    div = rng.standard_normal(shape).astype(np.float32)
    phi0 = rng.standard_normal(shape).astype(np.float32)
    mask = rng.random(shape) < 0.03
    mask[0, 5] = mask[-1, 7] = mask[shape[0] // 2, 0] = True
    ref = oracle.jacobi2d(div, phi0, dx=20 / 599, dt=np.float32(5e-5), iters=iters, mask=mask)
    phi = dev(phi0)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), iters,
                            rhs_ws=torch.empty_like(phi) if pre else None)
    assert np.array_equal(host(phi), ref)
    # and again on the same ring (a stale granule must not pass for a new one)
    phi = dev(phi0)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), iters)
    assert np.array_equal(host(phi), ref)


def test_jacobi2d_persistent_streams_and_threads():
    """The persistent Jacobi's library-owned ring: solves queued on two streams
    of one thread (the second waits for the first), and two host threads with
    a ring each, all equal to the oracle."""
    import threading
    shape, iters = (180, 600), 300
    rng = np.random.default_rng(7)
    cases = []
    for _ in range(4):
        div = rng.standard_normal(shape).astype(np.float32)
        mask = rng.random(shape) < 0.03
        cases.append((div, mask, oracle.jacobi2d(div, dx=20 / 599, dt=np.float32(5e-5), iters=iters, mask=mask)))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = []
    for i, (div, mask, _) in enumerate(cases):
        with torch.cuda.stream(streams[i % 2]):
            phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
            K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), iters)
            out.append(phi)
    torch.cuda.synchronize()
    for phi, (_, _, ref) in zip(out, cases):
        assert np.array_equal(host(phi), ref)

    res = [None] * len(cases)

    def work(i):
        div, mask, _ = cases[i]
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
            K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), iters)
            s.synchronize()
            res[i] = phi.cpu().numpy()
        call("cfd_release_thread_resources")  # this thread's ring, freed after its solve

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for r, (_, _, ref) in zip(res, cases):
        assert r is not None and np.array_equal(r, ref)


@pytest.mark.parametrize("shape,masked,dtype", [((180, 600), False, np.float32), ((180, 600), True, np.float32),
                                                ((37, 70), True, np.float32), ((180, 600), False, np.float64),
                                                ((1030, 70), False, np.float32)])
def test_jacobi2d_zero_start_matches_fill_then_solve(shape, masked, dtype):
    """cfd_jacobi2d_zero_* (phi = zeros inside the solve, v5.py:337): phi
    starts as garbage -- NaN inside, 7.0 on the boundary ring -- and ends
    equal to the oracle's zero-start solve, boundary ring included, on the
    persistent small-grid path (cylinder grid, with and without a mask) and
    on the fill-then-sweeps paths (f64; a grid past the persistent tiles)."""
    rng = np.random.default_rng(shape[0] + shape[1] + int(masked))
    div = rng.standard_normal(shape).astype(dtype)
    mask = rng.random(shape) < 0.03 if masked else None
    dx, dt, it = 20 / (shape[1] - 1), np.float32(5e-5), 40
    phi = torch.full(shape, float("nan"), dtype=torch.from_numpy(div).dtype, device=DEV)
    phi[0, :] = phi[-1, :] = phi[:, 0] = phi[:, -1] = 7.0
    K.solve_pressure_jacobi(phi, dev(div), dx, dt, None if mask is None else dev(mask), it, zero_start=True)
    ref = oracle.jacobi2d(div, dx=dx, dt=dt, iters=it, mask=mask)
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("cooperative", [1, 0])
def test_persistent_cooperative_and_plain_launch_bitexact(cooperative):
    """Both persistent small-grid solves, launched plainly (the default since
    r05) and cooperatively, on the cylinder grid: bit-exact, and no failure
    counted."""
    call("cfd_set_persistent_launch", cooperative, 0)
    shape = (180, 600)
    rng = np.random.default_rng(21 + cooperative)
    div = rng.standard_normal(shape).astype(np.float32)
    mask = rng.random(shape) < 0.03
    ref = oracle.jacobi2d(div, dx=20 / 599, dt=np.float32(5e-5), iters=300, mask=mask)
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), dev(mask), 300)
    assert np.array_equal(host(phi), ref)
    gdiv = div * np.float32(1e-3)
    gref, n_ref = oracle.rbgs2d(gdiv, dx=20 / 599, dy=4 / 179, dt=np.float32(5e-5), mask=mask, iters=200, tol=1e-8)
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(int(lib().cfd_rbgs2d_workspace_bytes(shape[0], shape[1], 200)), dtype=torch.uint8, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(gdiv), 20 / 599, 4 / 179, np.float32(5e-5), dev(mask), 200, 1e-8,
                                       workspace=ws, iters_done=done, phi_tmp=torch.zeros_like(phi))
    assert np.array_equal(host(phi), gref) and int(host(done)[0]) == n_ref
    assert K.persistent_failures() == 0


def test_last_jacobi2d_path_reports_the_persistent_solve():
    """cfd_get_last_jacobi2d_path (the bench's per-launch roofline): the small
    grid's solve is one persistent launch of all its sweeps, a forced
    launch-per-pass solve reports its depth."""
    import ctypes
    shape = (128, 128)
    div = dev(np.random.default_rng(5).standard_normal(shape).astype(np.float32))
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    spl = ctypes.c_int(0)
    K.solve_pressure_jacobi(phi, div, 1 / 127, np.float32(1e-3), None, 500)
    assert lib().cfd_get_last_jacobi2d_path(ctypes.byref(spl)) == 1 and spl.value == 500
    call("cfd_set_small2d_jacobi_persistent", 1, 0)
    try:
        K.solve_pressure_jacobi(phi, div, 1 / 127, np.float32(1e-3), None, 500)
        assert lib().cfd_get_last_jacobi2d_path(ctypes.byref(spl)) == 0 and 1 <= spl.value <= 8
    finally:
        call("cfd_set_small2d_jacobi_persistent", 0, 0)


def test_clean_divergence_multi_cu_expiry_fails_loudly():
    """clean_divergence past one band of row blocks runs one block per
    workgroup (k_lex_gs_skew_mc), each waiting for the block above's progress
    word; the wait is bounded like the persistent solves'.  With a 1-tick
    bound every wait expires at once: no hang, and the failures are counted
    (cfd_persistent_status).  With the default bound the result is the
    oracle's again and nothing is counted."""
    assert K.persistent_failures() == 0
    ny, nx = 1030, 70  # 16 row blocks: past one band of 4
    rng = np.random.default_rng(77)
    u0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    v0 = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    dx, dy = 20.0 / (nx - 1), 6.0 / (ny - 1)
    call("cfd_set_persistent_launch", 0, 1)
    u, v = dev(u0), dev(v0)
    K.clean_divergence_fast(u, v, dx, dy, iterations=2)
    assert K.persistent_failures() >= 1
    call("cfd_set_persistent_launch", 0, 0)
    u, v = dev(u0), dev(v0)
    K.clean_divergence_fast(u, v, dx, dy, iterations=2)
    cu, cv = oracle.clean_divergence2d(u0, v0, dx=dx, dy=dy, iterations=2)
    assert np.array_equal(host(u), cu) and np.array_equal(host(v), cv)
    assert K.persistent_failures() == 0


def test_persistent_forced_expiry_fails_loudly():
    """A neighbour wait that expires (forced by a 1-tick poll bound) must not
    pass silently: the persistent Jacobi leaves phi all NaN, the persistent
    GS phi all NaN and iters_done = -1, each counts a failure that
    cfd_persistent_status returns, and the solver's health check
    (monitor_simulation_health, v5.py:599-613) reports the step as failed.
    The next solve with the default bound is correct again."""
    from cfd_simulations_amd.solver import OptimizedTurbulentConfig, OptimizedTurbulentSolver, \
        monitor_simulation_health
    assert K.persistent_failures() == 0
    shape = (180, 600)
    rng = np.random.default_rng(5)
    div = rng.standard_normal(shape).astype(np.float32)
    call("cfd_set_persistent_launch", 1, 1)
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), None, 300)
    assert np.isnan(host(phi)).all()
    assert K.persistent_failures() == 1
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    ws = torch.empty(int(lib().cfd_rbgs2d_workspace_bytes(shape[0], shape[1], 100)), dtype=torch.uint8, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 20 / 599, 4 / 179, np.float32(5e-5), None, 100, 1e-8,
                                       workspace=ws, iters_done=done, phi_tmp=torch.zeros_like(phi))
    assert int(host(done)[0]) == -1 and np.isnan(host(phi)).all()
    assert K.persistent_failures() == 1
    for fast in (False, True):
        solver = OptimizedTurbulentSolver(OptimizedTurbulentConfig(use_fast_pressure=fast, pressure_iterations=64))
        solver.time_step()
        assert monitor_simulation_health(solver, 1) is False
    call("cfd_set_persistent_launch", 1, 0)
    phi = torch.zeros(shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), None, 300)
    assert np.array_equal(host(phi), oracle.jacobi2d(div, dx=20 / 599, dt=np.float32(5e-5), iters=300))
    assert K.persistent_failures() == 0


def test_jacobi2d_persistent_status_after_a_larger_grid():
    """The persistent Jacobi's status words (poll expired, workgroups done)
    must not move with the grid: a larger grid's solve, then a smaller one's
    on the same library-owned ring with a forced expiry, must still report
    it (phi all NaN, one failure), and a normal solve after it is exact."""
    rng = np.random.default_rng(12)
    big = rng.standard_normal((180, 1200)).astype(np.float32)
    div = rng.standard_normal((180, 600)).astype(np.float32)
    phi = torch.zeros(big.shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(big), 20 / 599, np.float32(5e-5), None, 300)
    assert np.array_equal(host(phi), oracle.jacobi2d(big, dx=20 / 599, dt=np.float32(5e-5), iters=300))
    assert K.persistent_failures() == 0
    call("cfd_set_persistent_launch", 0, 1)
    phi = torch.zeros(div.shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), None, 300)
    assert np.isnan(host(phi)).all()
    assert K.persistent_failures() == 1
    call("cfd_set_persistent_launch", 0, 0)
    phi = torch.zeros(div.shape, dtype=torch.float32, device=DEV)
    K.solve_pressure_jacobi(phi, dev(div), 20 / 599, np.float32(5e-5), None, 300)
    assert np.array_equal(host(phi), oracle.jacobi2d(div, dx=20 / 599, dt=np.float32(5e-5), iters=300))
    assert K.persistent_failures() == 0


def test_health_check_is_per_stream():
    """Two solvers on two streams (v5.py:599-613's health check per solver):
    a neighbour-wait expiry forced in solver A's step (1-tick poll bound, on
    stream A) is counted in stream A's failure word only.  Stream B's status
    reads 0 and leaves A's count alone; A's then reads 1 and A's
    monitor_simulation_health fails.  Reading B's status is an async copy on
    B plus a wait for B: work queued on stream A is still running after it."""
    from cfd_simulations_amd.solver import OptimizedTurbulentConfig, OptimizedTurbulentSolver, \
        monitor_simulation_health
    torch.cuda.synchronize()
    assert K.persistent_failures() == 0
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    cfg = OptimizedTurbulentConfig(use_fast_pressure=False, pressure_iterations=64)
    with torch.cuda.stream(sa):
        a = OptimizedTurbulentSolver(cfg)
    with torch.cuda.stream(sb):
        b = OptimizedTurbulentSolver(cfg)
    torch.cuda.synchronize()
    call("cfd_set_persistent_launch", 1, 1)
    try:
        with torch.cuda.stream(sa):
            a.time_step()
    finally:
        call("cfd_set_persistent_launch", 1, 0)
    with torch.cuda.stream(sb):
        b.time_step()
    sa.synchronize()
    assert K.persistent_failures(sb) == 0
    assert K.persistent_failures(sa) == 1
    assert K.persistent_failures(sa) == 0  # read and cleared
    assert torch.isfinite(b.u).all() and torch.isfinite(b.phi).all()
    # the failed step's phi is NaN: A's own health check fails on it
    with torch.cuda.stream(sa):
        assert monitor_simulation_health(a, 1) is False
    # no device-wide synchronisation: stream A stays busy while B's status is read
    with torch.cuda.stream(sa):
        torch.cuda._sleep(400_000_000)
    assert K.persistent_failures(sb) == 0
    assert not sa.query(), "reading stream B's status waited for stream A"
    sa.synchronize()
    call("cfd_set_persistent_launch", 0, 0)


# ------------------------------------------- zero-start solve, fused first pass
def test_jacobi3d_1024_zero_start_bitexact(div1024):
    """cfd_jacobi3d_zero_f32 at the bench geometry: phi = zeros then 2..9 and
    200 sweeps (the bench's step at the default 4 sweeps per pass: a fused
    4-sweep first pass that starts from the zeros and forms the RHS
    workspace, then 49 passes of 4; 7 and 9 sweeps open with a 3-sweep first
    pass, 9 ends with a 2-sweep remainder).  phi and the workspace start as
    NaN garbage: the first pass must read neither."""
    n = 1024
    h, dt = 1.0 / (n - 1), np.float32(5e-5)
    refs = {}
    ref = np.zeros_like(div1024)
    for it in range(1, 10):
        ref = oracle.jacobi3d(div1024, ref, h=h, dt=dt, iters=1, mt=True)
        refs[it] = ref
    d = dev(div1024)
    phi = torch.empty_like(d)
    tmp = torch.empty_like(d)
    rhs = torch.empty_like(d)
    for iters in (2, 3, 4, 5, 6, 7, 8, 9):
        phi.fill_(float("nan"))
        tmp.fill_(float("nan"))
        rhs.fill_(float("nan"))
        K.solve_pressure_jacobi3d_zero(phi, d, h, dt, iters, phi_tmp=tmp, rhs_ws=rhs)
        assert np.array_equal(host(phi), refs[iters]), iters
    del refs, ref
    # the bench step itself: 200 sweeps, vs the general path (pinned above) on the same inputs
    phi.fill_(float("nan"))
    K.solve_pressure_jacobi3d_zero(phi, d, h, dt, 200, phi_tmp=tmp, rhs_ws=rhs)
    want = torch.zeros_like(d)
    K.solve_pressure_jacobi3d(want, d, h, dt, None, 200, phi_tmp=tmp, rhs_ws=None)
    torch.cuda.synchronize()
    assert torch.equal(phi, want)


@pytest.mark.parametrize("levels", [0, 2, 4])
@pytest.mark.parametrize("shape", [(17, 19, 260), (6, 40, 8), (3, 3, 4), (40, 5, 516)])
def test_jacobi3d_zero_start_ragged_bitexact(levels, shape):
    """Zero-start solves on ragged grids (two x-segments, y and z not tile
    multiples, minimal 3-plane grids), every sweep count 1..10 (first passes
    of 2 and 3, remainders of 1 and 2, both result parities), blocking depth
    auto / 2 / 4, with and without the RHS workspace."""
    call("cfd_set_jacobi3d_blocking", levels, 0, 0)
    rng = np.random.default_rng(sum(shape))
    div = rng.standard_normal(shape).astype(np.float32)
    d = dev(div)
    ref = np.zeros_like(div)
    for iters in range(1, 11):
        ref = oracle.jacobi3d(div, ref, h=0.03, dt=np.float32(1e-3), iters=1)
        for rhs in (torch.full_like(d, float("nan")), None):
            phi = torch.full_like(d, float("nan"))
            tmp = torch.full_like(d, float("nan"))
            K.solve_pressure_jacobi3d_zero(phi, d, 0.03, np.float32(1e-3), iters, phi_tmp=tmp, rhs_ws=rhs)
            assert np.array_equal(host(phi), ref), (iters, rhs is None)


def test_jacobi3d_first_pass_general_start_bitexact():
    """The general solve with a workspace now forms it in its first pass (no
    RHS prologue) from a non-zero initial guess: still the oracle's bits."""
    rng = np.random.default_rng(5)
    div = rng.standard_normal((21, 35, 264)).astype(np.float32)
    phi0 = rng.standard_normal(div.shape).astype(np.float32)
    for iters in (2, 3, 5, 7):
        ref = oracle.jacobi3d(div, phi0, h=0.05, dt=np.float32(2e-3), iters=iters)
        phi = dev(phi0)
        rhs = torch.full_like(phi, float("nan"))
        K.solve_pressure_jacobi3d(phi, dev(div), 0.05, np.float32(2e-3), None, iters, rhs_ws=rhs)
        assert np.array_equal(host(phi), ref), iters


# ------------------------------------------ GS passes of 1..4 half-sweeps
def _rbgs3d_maxc(div, n, **kw):
    """The oracle's per-iteration max|change|: each cell is updated once per
    iteration, so it is max|phi_(i+1) - phi_i| in float32 (the kernel's
    fabsf(new - old))."""
    phi = np.zeros_like(div)
    out = []
    for _ in range(n):
        nxt, _ = oracle.rbgs3d(div, phi, iters=1, tol=0.0, **kw)
        out.append(float(np.abs(nxt - phi).max()))
        phi = nxt
    return np.array(out, np.float32)


@pytest.mark.parametrize("levels", [0, 2, 3, 4])
def test_rbgs3d_stop_at_every_iteration(levels):
    """A stop at every iteration 1..N of solves of N = 13 and 14 iterations,
    for passes of 2, 3 (auto) and 4 half-sweeps: with 3 per pass an iteration
    can end in the middle of a pass, which the rollback launches (1 or 2
    half-sweeps) undo; the count, the buffer the result lands in and every
    value must be the oracle's."""
    call("cfd_set_jacobi3d_blocking", levels, 0, 0)
    rng = np.random.default_rng(40 + levels)
    div = rng.standard_normal((19, 27, 132)).astype(np.float32) * np.float32(1e-3)
    kw = dict(dx=0.05, dy=0.05, dz=0.05, dt=np.float32(1e-2))
    mc = _rbgs3d_maxc(div, 14, **kw)
    d = dev(div)
    tmp = torch.empty_like(d)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    seen = set()
    for c in range(1, 15):
        lo = mc[c - 1]
        hi = mc[:c - 1].min() if c > 1 else np.float32(np.inf)
        if not lo < hi:
            continue
        tol = float(lo) * 1.0000005 if not np.isfinite(hi) else float((np.float64(lo) + np.float64(hi)) / 2)
        if not (lo < np.float32(tol) <= hi):
            continue
        for N in (13, 14):
            ref, n_ref = oracle.rbgs3d(div, iters=N, tol=tol, **kw)
            phi = torch.zeros_like(d)
            K.solve_pressure_gauss_seidel3d(phi, d, *(0.05,) * 3, kw["dt"], None, N, tol, iters_done=done,
                                            phi_tmp=tmp)
            assert int(host(done)[0]) == n_ref, (c, N, n_ref)
            assert np.array_equal(host(phi), ref), (c, N)
            seen.add(n_ref)
    assert len(seen) >= 10, seen


@pytest.mark.parametrize("persistent", [1, 2])
@pytest.mark.parametrize("iters,tol", [(37, 0.0), (400, 3e-5), (0, 0.0)])
def test_rbgs2d_zero_start_bitexact(iters, tol, persistent):
    """cfd_rbgs2d_zero_f32_ws (solve_pressure_fast's np.zeros + GS,
    v5.py:337-342) on the cylinder's grid shape: phi holds garbage (NaN rows
    included) before the call and must end as the oracle's solve from zeros,
    edge rows zero too; the persistent solve (2) reads nothing of phi, the
    launch-per-block path (1) zero-fills it first."""
    call("cfd_set_small2d_gs_persistent", persistent)
    rng = np.random.default_rng(44)
    div = rng.standard_normal((180, 600)).astype(np.float32) * np.float32(1e-3)
    mask = rng.random(div.shape) < 0.03
    ref, n_ref = oracle.rbgs2d(div, dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=iters, tol=tol, mask=mask)
    junk = rng.standard_normal(div.shape).astype(np.float32)
    junk[0, :] = np.nan
    junk[-1, 3] = np.inf
    phi = dev(junk)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), dev(mask), iters, tol,
                                       iters_done=done, zero_start=True)
    if iters:
        assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("iters,tol", [(23, 0.0), (300, 2e-5)])
def test_rbgs2d_persistent_fewer_iterations_per_block_when_tiles_do_not_fit(iters, tol):
    """180 x 1000: 5 iterations per block would need 23 x 15 = 345 tiles, more
    than the chip holds at once; the persistent solve takes the most that fit
    (4: 21 x 12 = 252 tiles) instead of the launch-per-block path."""
    call("cfd_set_small2d_gs_iters", 5, 2)
    call("cfd_set_small2d_gs_persistent", 2)
    rng = np.random.default_rng(91)
    div = rng.standard_normal((180, 1000)).astype(np.float32) * np.float32(1e-3)
    mask = rng.random(div.shape) < 0.03
    ref, n_ref = oracle.rbgs2d(div, dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=iters, tol=tol, mask=mask)
    phi = torch.zeros_like(dev(div))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), dev(mask), iters, tol,
                                       iters_done=done)
    assert int(host(done)[0]) == n_ref
    assert np.array_equal(host(phi), ref)


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("ni", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("masked", [True, False])
def test_rbgs2d_persistent_stop_at_every_iteration(ni, masked, mode):
    """The persistent small-grid GS (one launch, tiles handing their edge
    cells to each other): a stop at every iteration 1..N of solves of N = 22
    and 23 iterations on a grid of 3 x 4 .. 5 x 7 tiles.  A stop is seen two
    blocks late (or after the loop, for the last two blocks) and the block it
    fell in is re-run from its input granules; the count and every value must
    be the oracle's.  Then the same solve with tol = 0 and a stop-free tol."""
    call("cfd_set_small2d_gs_iters", ni, 2)
    call("cfd_set_small2d_gs_persistent", mode)
    rng = np.random.default_rng(70 + ni)
    div = rng.standard_normal((75, 170)).astype(np.float32) * np.float32(1e-2)
    mask = (rng.random(div.shape) < 0.05) if masked else None
    kw = dict(dx=0.1, dy=0.1, dt=np.float32(1.0), mask=mask)
    _, _, mc = oracle.rbgs2d_maxc(div, iters=23, tol=0.0, **kw)
    d = dev(div)
    m = None if mask is None else dev(mask)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    seen = set()
    for c in range(1, 24):
        lo = mc[c - 1]
        hi = mc[:c - 1].min() if c > 1 else np.float32(np.inf)
        if not lo < hi:
            continue
        tol = float(lo) * 1.0000005 if not np.isfinite(hi) else float((np.float64(lo) + np.float64(hi)) / 2)
        if not (lo < np.float32(tol) <= hi):
            continue
        for N in (22, 23):
            ref, n_ref = oracle.rbgs2d(div, iters=N, tol=tol, **kw)
            phi = torch.zeros_like(d)
            K.solve_pressure_gauss_seidel_fast(phi, d, 0.1, 0.1, np.float32(1.0), m, N, tol, iters_done=done)
            assert int(host(done)[0]) == n_ref, (c, N)
            assert np.array_equal(host(phi), ref), (c, N)
            seen.add(n_ref)
    assert len(seen) >= 8, seen
    for tol in (0.0, 1e-30):
        for N in (1, 2, 5, 23):
            ref, n_ref = oracle.rbgs2d(div, iters=N, tol=tol, **kw)
            phi = torch.zeros_like(d)
            K.solve_pressure_gauss_seidel_fast(phi, d, 0.1, 0.1, np.float32(1.0), m, N, tol, iters_done=done)
            assert int(host(done)[0]) == n_ref == N, (tol, N)
            assert np.array_equal(host(phi), ref), (tol, N)


def test_rbgs2d_persistent_repeated_solves_reuse_workspace():
    """Back-to-back persistent solves on one workspace (the time-step loop's
    pattern): a stale granule of the previous solve must never be taken for
    this one's (the rings are reset per solve); then the C entry without
    the workspace size (cfd_rbgs2d_f32) on the same workspace, which takes
    the launch-per-block path: same bits."""
    rng = np.random.default_rng(99)
    shape = (180, 600)
    ws = torch.empty(int(lib().cfd_rbgs2d_workspace_bytes(*shape, 50)), dtype=torch.uint8, device=DEV)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    for rep in range(3):
        div = rng.standard_normal(shape).astype(np.float32) * np.float32(1e-3)
        phi0 = rng.standard_normal(shape).astype(np.float32) * np.float32(1e-4)
        ref, n_ref = oracle.rbgs2d(div, phi0, dx=0.05, dy=0.05, dt=np.float32(1e-2), iters=50, tol=1e-8)
        phi = dev(phi0)
        K.solve_pressure_gauss_seidel_fast(phi, dev(div), 0.05, 0.05, np.float32(1e-2), None, 50, 1e-8,
                                           workspace=ws, iters_done=done)
        assert int(host(done)[0]) == n_ref, rep
        assert np.array_equal(host(phi), ref), rep
        phi = dev(phi0)
        tmp = torch.empty_like(phi)
        dv = dev(div)
        call("cfd_rbgs2d_f32", ptr(phi), ptr(dv), None, shape[0], shape[1], 0.05, 0.05, float(np.float32(1e-2)),
             50, 1e-8, ptr(tmp), ptr(ws), ptr(done), stream_handle())
        assert int(host(done)[0]) == n_ref, rep
        assert np.array_equal(host(phi), ref), rep


@pytest.mark.parametrize("ni", [1, 2, 3, 4])
@pytest.mark.parametrize("shape,masked,shared", [((1, 2, 4), True, 1), ((4, 2, 4), False, 1), ((1, 1, 16), True, 1),
                                                 ((1, 2, 4), True, 2), ((1, 2, 4), False, 2)])
def test_rbgs2d_small_stop_at_every_iteration(ni, shape, masked, shared):
    """Small-grid red-black GS with 1..4 iterations per launch: a stop at
    every iteration of solves of N = 16 and 17 iterations (a stop inside a
    launch is re-run from the launch's input by the rollback launch of the
    remainder), for the kernel's shapes, with and without solid cells; the
    count, the buffer the result lands in and every value are the oracle's."""
    vec, rw, wpb = shape
    call("cfd_set_small2d_shape", 0, 0, 0, rw, vec, wpb)
    call("cfd_set_small2d_gs_iters", ni, shared)
    rng = np.random.default_rng(7 + ni)
    div = rng.standard_normal((22, 40)).astype(np.float32) * np.float32(1e-2)
    mask = (rng.random(div.shape) < 0.06) if masked else None
    kw = dict(dx=0.1, dy=0.1, dt=np.float32(1.0), mask=mask)
    _, _, mc = oracle.rbgs2d_maxc(div, iters=17, tol=0.0, **kw)
    d = dev(div)
    m = None if mask is None else dev(mask)
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    seen = set()
    for c in range(1, 18):
        lo = mc[c - 1]
        hi = mc[:c - 1].min() if c > 1 else np.float32(np.inf)
        if not lo < hi:
            continue
        tol = float(lo) * 1.0000005 if not np.isfinite(hi) else float((np.float64(lo) + np.float64(hi)) / 2)
        if not (lo < np.float32(tol) <= hi):
            continue
        for N in (16, 17):
            ref, n_ref = oracle.rbgs2d(div, iters=N, tol=tol, **kw)
            phi = torch.zeros_like(d)
            K.solve_pressure_gauss_seidel_fast(phi, d, 0.1, 0.1, np.float32(1.0), m, N, tol, iters_done=done)
            assert int(host(done)[0]) == n_ref, (c, N)
            assert np.array_equal(host(phi), ref), (c, N)
            seen.add(n_ref)
    assert len(seen) >= 8, seen
