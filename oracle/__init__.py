"""CPU oracle for the pressure-Poisson / predictor hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this package, and only as the
checker (or the timed CPU baseline), never as the thing measured or shipped.
The product path (``cfd-simulations_amd``) never imports it and fails loudly
when its HIP library is missing.

Contents
--------
* ``liboracle.so`` (built from ``stencil_oracle.c`` by ``oracle/Makefile``):
  C restatements of the reference kernels, each citing the v5.py line range it
  follows.  Pinned bit-for-bit against ``tests/golden/*.npz``.  The reference
  generated those fixtures (``tests/golden/make_golden.py``).
* ``jacobi2d_numpy``: NumPy restatement of the reference's Jacobi branch
  (v5.py:336-346) in the reference's own array-expression form.  This is the
  ``cpu_baseline`` ("port") that bench.py times.
* ``OracleSolver``: ``time_step()`` (v5.py:375-441) composed from the C
  kernels and NumPy.  It is the end-to-end checker for the GPU solver.

All paths below are relative to the reference's
``python/flow_over_cylinder (Fischer)/v5.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_u8p = ctypes.c_void_p
_i, _d, _f = ctypes.c_int, ctypes.c_double, ctypes.c_float


def build() -> Path:
    """Compile liboracle.so with the committed Makefile (gcc, no fast-math)."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _HERE / "liboracle.so"


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        so = _HERE / "liboracle.so"
        if not so.exists() or so.stat().st_mtime < (_HERE / "stencil_oracle.c").stat().st_mtime:
            build()
        L = ctypes.CDLL(str(so))
        L.oracle_jacobi2d_f32.argtypes = [_f32p, _u8p, _f32p, _i, _i, _d, _f, _i]
        L.oracle_jacobi2d_f64.argtypes = [_f64p, _u8p, _f64p, _i, _i, _d, _f, _i]
        L.oracle_jacobi3d_f32.argtypes = [_f32p, _u8p, _f32p, _i, _i, _i, _d, _f, _i]
        L.oracle_rbgs2d_f32.argtypes = [_f32p, _f32p, _u8p, _i, _i, _d, _d, _f, _i, _d]
        L.oracle_rbgs2d_f32.restype = _i
        L.oracle_rbgs3d_f32.argtypes = [_f32p, _f32p, _u8p, _i, _i, _i, _d, _d, _d, _f, _i, _d]
        L.oracle_rbgs3d_f32.restype = _i
        L.oracle_rbgs2d_f32_maxc.argtypes = [_f32p, _f32p, _u8p, _i, _i, _d, _d, _f, _i, _d, _f32p]
        L.oracle_rbgs2d_f32_maxc.restype = _i
        L.oracle_jacobi3d_f32_mt.argtypes = [_f32p, _u8p, _f32p, _i, _i, _i, _d, _f, _i]
        L.oracle_rbgs3d_f32_mt.argtypes = [_f32p, _f32p, _u8p, _i, _i, _i, _d, _d, _d, _f, _i, _d]
        L.oracle_rbgs3d_f32_mt.restype = _i
        L.oracle_rbgs2d_f32_mt.argtypes = [_f32p, _f32p, _u8p, _i, _i, _d, _d, _f, _i, _d]
        L.oracle_rbgs2d_f32_mt.restype = _i
        L.oracle_threads.restype = _i
        L.oracle_predictor2d_f32.argtypes = [_f32p, _f32p, _f32p, _i, _i, _d, _d, _f, _i] + [_f32p] * 7
        L.oracle_predictor2d_f32_mode.argtypes = [_f32p, _f32p, _f32p, _i, _i, _d, _d, _f, _i, _i] + [_f32p] * 7
        L.oracle_predictor2d_f64.argtypes = [_f64p, _f64p, _f64p, _i, _i, _d, _d, _d, _i, _i] + [_f64p] * 7
        L.oracle_divergence2d_f32.argtypes = [_f32p, _f32p, _f32p, _i, _i, _d, _d]
        L.oracle_gradient2d_f32.argtypes = [_f32p, _f32p, _f32p, _i, _i, _d, _d]
        L.oracle_powf_f32.argtypes = [_f32p, _f, _f32p, ctypes.c_size_t]
        L.oracle_pow_f64.argtypes = [_f64p, _d, _f64p, ctypes.c_size_t]
        L.oracle_clean_divergence2d_f32.argtypes = [_f32p, _f32p, _i, _i, _d, _d, _i]
        _LIB = L
    return _LIB


def _mask_ptr(mask, shape):
    if mask is None:
        return None, None
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    assert m.shape == tuple(shape)
    return m, m.ctypes.data


# ---------------------------------------------------------------- Poisson
def jacobi2d(div, phi0=None, *, dx, dt, iters, mask=None):
    """a2 (v5.py:336-346).  float32 or float64 by ``div.dtype``."""
    div = np.ascontiguousarray(div)
    phi = np.zeros_like(div) if phi0 is None else np.array(phi0, dtype=div.dtype, copy=True)
    keep, mp = _mask_ptr(mask, div.shape)
    fn = lib().oracle_jacobi2d_f32 if div.dtype == np.float32 else lib().oracle_jacobi2d_f64
    fn(div, mp, phi, div.shape[0], div.shape[1], float(dx), np.float32(dt), int(iters))
    return phi


def threads() -> int:
    """Host threads the multi-threaded (``mt=True``) restatements use (OpenMP)."""
    return int(lib().oracle_threads())


def jacobi3d(div, phi0=None, *, h, dt, iters, mask=None, mt=False):
    """7-point generalisation of a2 (the build's own template).  ``mt``: the
    OpenMP form (planes split over host threads; bit-identical)."""
    div = np.ascontiguousarray(div, dtype=np.float32)
    phi = np.zeros_like(div) if phi0 is None else np.array(phi0, dtype=np.float32, copy=True)
    keep, mp = _mask_ptr(mask, div.shape)
    nz, ny, nx = div.shape
    fn = lib().oracle_jacobi3d_f32_mt if mt else lib().oracle_jacobi3d_f32
    fn(div, mp, phi, nz, ny, nx, float(h), np.float32(dt), int(iters))
    return phi


def rbgs2d(div, phi0=None, *, dx, dy, dt, iters, tol, mask=None, mt=False):
    """a3 (v5.py:202-226), serial semantics.  Returns (phi, iterations_done).
    ``mt``: the OpenMP form (rows of a colour over host threads, as the
    reference's prange; bit-identical)."""
    div = np.ascontiguousarray(div, dtype=np.float32)
    phi = np.zeros_like(div) if phi0 is None else np.array(phi0, dtype=np.float32, copy=True)
    keep, mp = _mask_ptr(mask, div.shape)
    fn = lib().oracle_rbgs2d_f32_mt if mt else lib().oracle_rbgs2d_f32
    done = fn(phi, div, mp, div.shape[0], div.shape[1], float(dx), float(dy), np.float32(dt), int(iters),
              float(tol))
    return phi, done


def rbgs2d_maxc(div, phi0=None, *, dx, dy, dt, iters, tol, mask=None):
    """rbgs2d plus the per-iteration max|change| history: (phi, done, maxc[done])."""
    div = np.ascontiguousarray(div, dtype=np.float32)
    phi = np.zeros_like(div) if phi0 is None else np.array(phi0, dtype=np.float32, copy=True)
    keep, mp = _mask_ptr(mask, div.shape)
    maxc = np.zeros(max(int(iters), 1), np.float32)
    done = lib().oracle_rbgs2d_f32_maxc(phi, div, mp, div.shape[0], div.shape[1], float(dx), float(dy),
                                        np.float32(dt), int(iters), float(tol), maxc)
    return phi, done, maxc[:done]


def rbgs3d(div, phi0=None, *, dx, dy, dz, dt, iters, tol, mask=None, mt=False):
    """3-D red-black generalisation of a3.  ``mt``: the OpenMP form."""
    div = np.ascontiguousarray(div, dtype=np.float32)
    phi = np.zeros_like(div) if phi0 is None else np.array(phi0, dtype=np.float32, copy=True)
    keep, mp = _mask_ptr(mask, div.shape)
    nz, ny, nx = div.shape
    fn = lib().oracle_rbgs3d_f32_mt if mt else lib().oracle_rbgs3d_f32
    done = fn(phi, div, mp, nz, ny, nx, float(dx), float(dy), float(dz), np.float32(dt), int(iters), float(tol))
    return phi, done


def jacobi2d_numpy(div, *, dx, dt, iters, mask=None):
    """NumPy restatement of v5.py:336-346 in the reference's own array form
    (~10 full-array passes per iteration).  The CPU baseline bench.py times."""
    phi = np.zeros_like(div)
    for _ in range(iters):
        phi_new = phi.copy()
        phi_new[1:-1, 1:-1] = 0.25 * (
            phi[1:-1, 2:] + phi[1:-1, :-2] + phi[2:, 1:-1] + phi[:-2, 1:-1]
            - dx ** 2 * div[1:-1, 1:-1] / dt)
        if mask is not None:
            phi_new[mask] = 0
        phi = phi_new
    return phi


def jacobi3d_numpy(div, *, h, dt, iters):
    """NumPy form of the 7-point template (same op order as oracle_jacobi3d_f32):
    the CPU baseline for the 3-D workloads."""
    sixth = np.float32(1.0) / np.float32(6.0)
    rhs = (np.float32(h * h) * div) / np.float32(dt)
    phi = np.zeros_like(div)
    c = (slice(1, -1),) * 3
    for _ in range(iters):
        phi_new = phi.copy()
        s = phi[1:-1, 1:-1, 2:] + phi[1:-1, 1:-1, :-2]
        s += phi[1:-1, 2:, 1:-1]
        s += phi[1:-1, :-2, 1:-1]
        s += phi[2:, 1:-1, 1:-1]
        s += phi[:-2, 1:-1, 1:-1]
        s -= rhs[c]
        s *= sixth
        phi_new[c] = s
        phi = phi_new
    return phi


# ---------------------------------------------------------------- predictor
def predictor2d(u, v, nu_eff, *, dx, dy, dt, use_supg=True, fastmath=False, dtype=np.float32):
    """a6-a10 (v5.py:112-176, :388-403).  Returns a dict of every array.

    dtype float32 (memory_efficient=True) or float64 (False, v5.py:287-296:
    float64 scalars, libm pow, Python constants unrounded).  fastmath: |V| as
    the compiled reference computes it (@njit(fastmath=True), v5.py:149:
    x**2 -> x*x, **0.5 -> a correctly rounded sqrt) instead of NumPy's scalar
    `**` (libm powf / pow) -- the checker of the build's tau mode 1."""
    dtype = np.dtype(dtype)
    u = np.ascontiguousarray(u, dtype)
    v = np.ascontiguousarray(v, dtype)
    nu = np.ascontiguousarray(np.broadcast_to(np.asarray(nu_eff, dtype), u.shape))
    out = {k: np.empty_like(u) for k in ("tau", "conv_u", "conv_v", "lap_u", "lap_v", "u_star", "v_star")}
    if dtype == np.float64:
        lib().oracle_predictor2d_f64(u, v, nu, u.shape[0], u.shape[1], float(dx), float(dy), float(dt),
                                     int(bool(use_supg)), int(bool(fastmath)), out["tau"], out["conv_u"],
                                     out["conv_v"], out["lap_u"], out["lap_v"], out["u_star"], out["v_star"])
    else:
        lib().oracle_predictor2d_f32_mode(u, v, nu, u.shape[0], u.shape[1], float(dx), float(dy), np.float32(dt),
                                          int(bool(use_supg)), int(bool(fastmath)), out["tau"], out["conv_u"],
                                          out["conv_v"], out["lap_u"], out["lap_v"], out["u_star"], out["v_star"])
    return out


def numpy_pow(x, y):
    """libm pow elementwise: NumPy's float64 scalar ``x ** y``."""
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    lib().oracle_pow_f64(x, float(y), out, x.size)
    return out


def numpy_powf(x, y):
    """libm powf elementwise: NumPy's float32 scalar ``x ** y``."""
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().oracle_powf_f32(x, np.float32(y), out, x.size)
    return out


def divergence2d(u, v, *, dx, dy):
    """a4 (v5.py:178-187)."""
    u = np.ascontiguousarray(u, np.float32)
    v = np.ascontiguousarray(v, np.float32)
    d = np.empty_like(u)
    lib().oracle_divergence2d_f32(u, v, d, u.shape[0], u.shape[1], float(dx), float(dy))
    return d


def gradient2d(phi, *, dx, dy):
    """a5 (v5.py:189-200)."""
    phi = np.ascontiguousarray(phi, np.float32)
    gx, gy = np.empty_like(phi), np.empty_like(phi)
    lib().oracle_gradient2d_f32(phi, gx, gy, phi.shape[0], phi.shape[1], float(dx), float(dy))
    return gx, gy


def clean_divergence2d(u, v, *, dx, dy, iterations=2):
    """clean_divergence_fast (v5.py:239-257), serial lexicographic semantics."""
    u = np.array(u, np.float32, copy=True)
    v = np.array(v, np.float32, copy=True)
    lib().oracle_clean_divergence2d_f32(u, v, u.shape[0], u.shape[1], float(dx), float(dy), int(iterations))
    return u, v


# ---------------------------------------------------------------- full step
class OracleSolver:
    """CPU restatement of OptimizedTurbulentSolver.time_step (v5.py:375-441)
    built from the C kernels above plus NumPy for the array glue.  Takes an
    already-initialised state (fields, masks) so it checks the GPU solver on
    identical inputs.  Returns dt like the reference."""

    numpy_jacobi = False  # True: the Jacobi branch in the reference's NumPy form (jacobi2d_numpy)
    mt = False            # True: the GS solve on all host threads (oracle_rbgs2d_f32_mt)

    def __init__(self, cfg, u, v, cylinder_mask, ibm_mask, y):
        self.cfg = cfg
        self.u = np.array(u, np.float32, copy=True)
        self.v = np.array(v, np.float32, copy=True)
        self.cylinder_mask = np.asarray(cylinder_mask, bool)
        self.ibm_mask = np.asarray(ibm_mask, np.float64)
        self.y = np.asarray(y, np.float64)
        self.phi = np.zeros_like(self.u)
        self.step = 0
        self.energy_history = []
        self.diagnostics = {}  # the last step's log values (v5.py:410, 415, 422, 428)

    def adaptive_time_step(self):  # v5.py:316-326
        c = self.cfg
        if not c.adaptive_dt:
            return c.dt_base
        if self.step < 1000:
            return np.float32(0.00002)
        vel_max = max(np.max(np.abs(self.u)), np.max(np.abs(self.v)), 1e-10)
        dt_cfl = c.cfl_target * min(c.dx, c.dy) / vel_max
        nu_total = c.nu + 0.0 + c.artificial_viscosity
        dt_visc = 0.4 * min(c.dx, c.dy) ** 2 / nu_total
        return np.float32(np.clip(min(dt_cfl, dt_visc), c.dt_min, c.dt_max))

    def compute_vorticity(self):  # v5.py:365-373
        c = self.cfg
        w = np.zeros_like(self.u)
        w[1:-1, 1:-1] = ((self.v[1:-1, 2:] - self.v[1:-1, :-2]) / (2 * c.dx)
                         - (self.u[2:, 1:-1] - self.u[:-2, 1:-1]) / (2 * c.dy))
        w[self.cylinder_mask] = np.nan
        return w

    def apply_boundary_conditions(self, u, v):  # v5.py:349-360
        c = self.cfg
        pert_scale = min(1.0, self.step / 1000.0) * 0.01
        pert = pert_scale * np.sin(2 * np.pi * self.y / c.y_max + 0.02 * self.step)
        u[:, 0] = c.V_inf * (1 + pert)
        v[:, 0] = 0
        u[:, -1] = u[:, -2]
        v[:, -1] = v[:, -2]
        u[0, :] = 0
        u[-1, :] = 0
        v[0, :] = 0
        v[-1, :] = 0

    def apply_ibm(self, u, v, fs):  # apply_ibm_fast v5.py:228-237, serial
        m = self.ibm_mask
        sel = m > 0
        fac = 1.0 - m[sel] * fs
        u[sel] = (u[sel].astype(np.float64) * fac).astype(np.float32)
        v[sel] = (v[sel].astype(np.float64) * fac).astype(np.float32)

    def time_step(self):
        c = self.cfg
        dt = self.adaptive_time_step()
        u_old, v_old = self.u.copy(), self.v.copy()
        nu_eff = c.nu + np.zeros_like(self.u) + c.artificial_viscosity
        pr = predictor2d(u_old, v_old, nu_eff, dx=c.dx, dy=c.dy, dt=dt, use_supg=c.use_supg)
        self.tau_supg = pr["tau"]
        u_star, v_star = pr["u_star"], pr["v_star"]
        self.apply_boundary_conditions(u_star, v_star)
        fs = min(1.0, self.step / c.initial_steps)
        self.apply_ibm(u_star, v_star, fs)
        self.u_star, self.v_star = u_star, v_star
        self.div_u_star = divergence2d(u_star, v_star, dx=c.dx, dy=c.dy)
        diag = {"pre_div_max": np.max(np.abs(self.div_u_star))}
        if c.use_fast_pressure:
            self.phi, _ = rbgs2d(self.div_u_star, dx=c.dx, dy=c.dy, dt=c.dt, iters=c.pressure_iterations,
                                 tol=c.pressure_tolerance, mask=self.cylinder_mask, mt=self.mt)
        elif self.numpy_jacobi:
            self.phi = jacobi2d_numpy(self.div_u_star, dx=c.dx, dt=c.dt, iters=c.pressure_iterations,
                                      mask=self.cylinder_mask if self.cylinder_mask.any() else None)
        else:
            self.phi = jacobi2d(self.div_u_star, dx=c.dx, dt=c.dt, iters=c.pressure_iterations,
                                mask=self.cylinder_mask)
        gx, gy = gradient2d(self.phi, dx=c.dx, dy=c.dy)
        diag["grad_max"] = np.max(np.abs(np.sqrt(gx ** 2 + gy ** 2)))
        self.u = u_star - dt * gx
        self.v = v_star - dt * gy
        self.u, self.v = clean_divergence2d(self.u, self.v, dx=c.dx, dy=c.dy, iterations=2)
        diag["post_div_max"] = np.max(np.abs(divergence2d(self.u, self.v, dx=c.dx, dy=c.dy)))
        self.apply_boundary_conditions(self.u, self.v)
        self.apply_ibm(self.u, self.v, fs)
        diag["vorticity_max"] = np.nanmax(np.abs(self.compute_vorticity()))
        self.diagnostics = diag
        energy = 0.5 * (self.u ** 2 + self.v ** 2)
        self.energy_history.append((self.step, np.nanmean(energy)))
        np.clip(self.u, -c.max_velocity, c.max_velocity, out=self.u)
        np.clip(self.v, -c.max_velocity, c.max_velocity, out=self.v)
        self.step += 1
        return dt


class OracleCavitySolver(OracleSolver):
    """The same step on the lid-driven cavity (BASELINE config 1; the build's
    own case, see cfd_simulations_amd.solver.LidDrivenCavityConfig): cavity
    walls, no solid cells, zero initial velocity.  With ``numpy_jacobi`` its
    pressure solve is the reference's NumPy Jacobi form: the CPU path of
    config 1 that bench.py times."""

    def __init__(self, cfg, numpy_jacobi=False):
        z = np.zeros((cfg.ny, cfg.nx), np.float32)
        super().__init__(cfg, z, z, np.zeros(z.shape, bool), np.zeros(z.shape), np.linspace(cfg.y_min, cfg.y_max,
                                                                                          cfg.ny))
        self.numpy_jacobi = numpy_jacobi

    def apply_boundary_conditions(self, u, v):
        u[:, 0] = 0
        v[:, 0] = 0
        u[:, -1] = 0
        v[:, -1] = 0
        u[0, :] = 0
        v[0, :] = 0
        u[-1, :] = np.float32(self.cfg.lid_velocity)
        v[-1, :] = 0

    def apply_ibm(self, u, v, fs):  # no immersed boundary in the cavity
        pass


def monitor_simulation_health(u, v, cfg, step) -> bool:
    """v5.py:599-613 on host arrays: non-finite values, |V| > max_velocity,
    max|div| above 20 (step <= 1000) or 2 (after)."""
    if np.any(~np.isfinite(u)) or np.any(~np.isfinite(v)):
        return False
    if max(np.max(np.abs(u)), np.max(np.abs(v))) > cfg.max_velocity:
        return False
    div_max = np.max(np.abs(divergence2d(u, v, dx=cfg.dx, dy=cfg.dy)))
    return not (div_max > (20.0 if step <= 1000 else 2.0))


def cpu_count() -> int:
    return os.cpu_count() or 1
