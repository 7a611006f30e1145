"""Reference-named device kernels: drop-ins for the @njit functions of v5.py.

Each function keeps the name, argument order and meaning, and the ownership
rules of its reference counterpart in
``python/flow_over_cylinder (Fischer)/v5.py``.  Allocating kernels return fresh
arrays with a zero boundary ring (``np.zeros_like``).  GS, IBM and
divergence cleaning mutate their inputs in place and return them.  The arrays
are torch tensors on the HIP device.  The work runs in the hand-written gfx950
kernels of libcfdsim.so, on the current torch stream.  Nothing here falls back
to the CPU: CPU tensors raise ``TypeError``.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import call, ptr, stream_handle, lib

__all__ = [
    "compute_convection_fast", "compute_convection_supg_fast", "compute_supg_stabilization_fast",
    "compute_laplacian_fast", "compute_divergence_fast", "compute_gradient_fast",
    "solve_pressure_gauss_seidel_fast", "solve_pressure_jacobi", "apply_ibm_fast",
    "clean_divergence_fast", "predictor_fused", "project_velocity", "solve_pressure_jacobi3d",
    "solve_pressure_jacobi3d_zero",
    "solve_pressure_gauss_seidel3d", "persistent_failures",
]


def _f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (memory_efficient fields), got {t.dtype}")
    return t


_SFX = {torch.float32: "_f32", torch.float64: "_f64"}


def _fields(name, *ts):
    """Entry point `name` + _f32 / _f64 for the fields' dtype: float32
    (memory_efficient=True, v5.py:287) or float64 (False); every field of one
    call must share it."""
    dt = ts[0].dtype
    if dt not in _SFX:
        raise TypeError(f"{name}: fields must be float32 or float64, got {dt}")
    for t in ts[1:]:
        if t is not None and t.dtype != dt:
            raise TypeError(f"{name}: mixed field dtypes {dt} and {t.dtype}")
    return name + _SFX[dt]


def _dt_arg(dt, field_dtype):
    """The step's dt as it meets the fields (NEP 50): float32 fields round it
    to float32 (np.float32 or a Python float dt_base alike); float64 fields
    take it exactly (the f64 entry points take a double)."""
    return float(np.float32(dt)) if field_dtype == torch.float32 else float(dt)


def _like(phi: torch.Tensor, t, name: str):
    """A companion array of phi (div, scratch, workspace): same shape, dtype,
    device, C-contiguous -- the kernels index it with phi's strides, so a
    mismatch would read or write out of bounds.  None passes through."""
    if t is None:
        return None
    if tuple(t.shape) != tuple(phi.shape) or t.dtype != phi.dtype or t.device != phi.device:
        raise ValueError(f"{name} must match phi: got {tuple(t.shape)} {t.dtype} on {t.device}, "
                         f"phi is {tuple(phi.shape)} {phi.dtype} on {phi.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be C-contiguous")
    return t


def _shape2d(t: torch.Tensor):
    if t.dim() != 2:
        raise ValueError(f"expected a 2-D (ny, nx) array, got shape {tuple(t.shape)}")
    return int(t.shape[0]), int(t.shape[1])


def _mask_u8(mask, shape):
    if mask is None:
        return None
    if tuple(mask.shape) != tuple(shape):
        raise ValueError(f"mask shape {tuple(mask.shape)} != field shape {tuple(shape)}")
    m = mask if mask.dtype == torch.uint8 else mask.to(torch.uint8)
    return m.contiguous()


def _nu(nu_eff, dtype=torch.float32):
    """nu_eff as (array_or_None, scalar): an array is passed through, a scalar
    (LES off: nu + 0 + art_visc, v5.py:388) is broadcast by the kernel, in the
    fields' precision."""
    if isinstance(nu_eff, torch.Tensor) and nu_eff.dim() > 0:
        if nu_eff.dtype != dtype:
            raise TypeError(f"nu_eff must be {dtype}, got {nu_eff.dtype}")
        return nu_eff.contiguous(), 0.0
    return None, float(np.float32(nu_eff)) if dtype == torch.float32 else float(nu_eff)


def compute_supg_stabilization_fast(u, v, dx, dy, dt, nu_eff):
    """v5.py:149-162."""
    ny, nx = _shape2d(u)
    tau = torch.empty_like(u)
    nu_a, nu_s = _nu(nu_eff, u.dtype)
    call(_fields("cfd_supg_tau2d", u, v), ptr(u), ptr(v), ptr(nu_a), nu_s, ptr(tau), ny, nx, float(dx), float(dy),
         _dt_arg(dt, u.dtype), stream_handle())
    return tau


def compute_convection_supg_fast(u, v, phi, dx, dy, tau_supg):
    """v5.py:127-147 (derivative factors 1/(4dx), 1/(4dx^2): the reference's quirk)."""
    ny, nx = _shape2d(phi)
    conv = torch.empty_like(phi)
    call(_fields("cfd_convection_supg2d", phi, u, v, tau_supg), ptr(u), ptr(v), ptr(phi), ptr(tau_supg), ptr(conv),
         ny, nx, float(dx), float(dy), stream_handle())
    return conv


def compute_convection_fast(u, v, phi, dx, dy):
    """First-order upwind convection, v5.py:112-125."""
    ny, nx = _shape2d(phi)
    conv = torch.empty_like(phi)
    call(_fields("cfd_convection_upwind2d", phi, u, v), ptr(u), ptr(v), ptr(phi), ptr(conv), ny, nx, float(dx),
         float(dy), stream_handle())
    return conv


def compute_laplacian_fast(phi, dx, dy, nu_eff):
    """v5.py:164-176."""
    ny, nx = _shape2d(phi)
    lap = torch.empty_like(phi)
    nu_a, nu_s = _nu(nu_eff, phi.dtype)
    call(_fields("cfd_laplacian2d", phi), ptr(phi), ptr(nu_a), nu_s, ptr(lap), ny, nx, float(dx), float(dy),
         stream_handle())
    return lap


def compute_divergence_fast(u, v, dx, dy, absmax=None):
    """v5.py:178-187.  ``absmax``: optional zeroed device scalar of the
    fields' dtype that receives max|div| (the v5.py:410 diagnostic) without a
    host sync."""
    ny, nx = _shape2d(u)
    div = torch.empty_like(u)
    call(_fields("cfd_divergence2d", u, v, absmax), ptr(u), ptr(v), ptr(div), ny, nx, float(dx), float(dy),
         ptr(absmax), stream_handle())
    return div


def compute_gradient_fast(phi, dx, dy):
    """v5.py:189-200."""
    ny, nx = _shape2d(phi)
    gx, gy = torch.empty_like(phi), torch.empty_like(phi)
    call(_fields("cfd_gradient2d", phi), ptr(phi), ptr(gx), ptr(gy), ny, nx, float(dx), float(dy), stream_handle())
    return gx, gy


def solve_pressure_gauss_seidel_fast(phi, div_u_star, dx, dy, dt, mask, iterations, tolerance,
                                     workspace=None, iters_done=None, phi_tmp=None, zero_start=False):
    """v5.py:202-226: red-black GS, in place on ``phi``; returns ``phi``.
    ``zero_start``: phi = zeros first (v5.py:337) inside the solve
    (cfd_rbgs2d_zero_f32_ws: the persistent small-grid solve reads nothing of
    phi; other paths zero-fill it first).
    ``iters_done`` (optional int32 device scalar) receives the iteration count.
    float32: ``phi_tmp`` (same-size scratch field, allocated if omitted) lets
    every iteration run as one fused out-of-place pass; the result still lands
    in ``phi``, bit-identical to the in-place colour passes.  float64
    (memory_efficient=False): in-place colour passes (phi_tmp unused)."""
    ny, nx = _shape2d(phi)
    m = _mask_u8(mask, phi.shape)
    ws = workspace
    # the grid-sized workspace (small grids: the persistent solve's exchange
    # rings, cfd_rbgs2d_workspace_bytes) when float32, the base one otherwise
    need = int(lib().cfd_rbgs2d_workspace_bytes(ny, nx, int(iterations)) if phi.dtype == torch.float32
               else lib().cfd_rbgs_workspace_bytes(int(iterations)))
    if ws is None or ws.numel() * ws.element_size() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=phi.device)
    _like(phi, div_u_star, "div_u_star")
    if phi.dtype == torch.float64:
        if zero_start:
            phi.zero_()
        call("cfd_rbgs2d_f64", ptr(phi), ptr(div_u_star), ptr(m), ny, nx, float(dx), float(dy),
             float(np.float32(dt)), int(iterations), float(tolerance), ptr(ws), ptr(iters_done), stream_handle())
        return phi
    tmp = torch.empty_like(phi) if phi_tmp is None else _like(phi, phi_tmp, "phi_tmp")
    call("cfd_rbgs2d_zero_f32_ws" if zero_start else "cfd_rbgs2d_f32_ws", ptr(_f32(phi, "phi")), ptr(_f32(div_u_star, "div_u_star")), ptr(m), ny, nx,
         float(dx), float(dy), float(np.float32(dt)), int(iterations), float(tolerance), ptr(_f32(tmp, "phi_tmp")),
         ptr(ws), ws.numel() * ws.element_size(), ptr(iters_done), stream_handle())
    return phi


def solve_pressure_jacobi(phi, div_u_star, dx, dt, mask, iterations, phi_tmp=None,
                          resid_every=0, resid_out=None, rhs_ws=None, zero_start=False):
    """Jacobi branch of solve_pressure_fast, v5.py:336-346, bit-exact; in place
    on ``phi`` (float32 or float64 fields); returns ``phi``.  ``rhs_ws``: an
    optional same-size workspace that lets the sweeps skip the division.
    ``zero_start``: phi = zeros first (v5.py:337) inside the solve
    (cfd_jacobi2d_zero_*: the persistent small-grid solve reads nothing of
    phi, no fill launch)."""
    ny, nx = _shape2d(phi)
    if div_u_star.dtype != phi.dtype:
        raise TypeError("phi and div_u_star must share a dtype")
    _like(phi, div_u_star, "div_u_star")
    _like(phi, rhs_ws, "rhs_ws")
    tmp = torch.empty_like(phi) if phi_tmp is None else _like(phi, phi_tmp, "phi_tmp")
    m = _mask_u8(mask, phi.shape)
    z = "_zero" if zero_start else ""
    fn = {torch.float32: f"cfd_jacobi2d{z}_f32", torch.float64: f"cfd_jacobi2d{z}_f64"}.get(phi.dtype)
    if fn is None:
        raise TypeError(f"unsupported dtype {phi.dtype}")
    call(fn, ptr(div_u_star), ptr(phi), ptr(tmp), ptr(rhs_ws), ptr(m), ny, nx, float(dx),
         float(np.float32(dt)), int(iterations), int(resid_every), ptr(resid_out), stream_handle())
    return phi


def solve_pressure_jacobi3d(phi, div, h, dt, mask, iterations, phi_tmp=None, resid_every=0,
                            resid_out=None, rhs_ws=None):
    """7-point generalisation of the Jacobi branch on an (nz, ny, nx) float32 grid."""
    if phi.dim() != 3:
        raise ValueError("expected (nz, ny, nx)")
    nz, ny, nx = (int(s) for s in phi.shape)
    _like(phi, _f32(div, "div"), "div")
    _like(phi, rhs_ws, "rhs_ws")
    tmp = torch.empty_like(phi) if phi_tmp is None else _like(phi, phi_tmp, "phi_tmp")
    m = _mask_u8(mask, phi.shape)
    call("cfd_jacobi3d_f32", ptr(_f32(div, "div")), ptr(_f32(phi, "phi")), ptr(tmp), ptr(rhs_ws), ptr(m),
         nz, ny, nx, float(h), float(np.float32(dt)), int(iterations), int(resid_every), ptr(resid_out),
         stream_handle())
    return phi


def solve_pressure_jacobi3d_zero(phi, div, h, dt, iterations, phi_tmp=None, rhs_ws=None):
    """The Jacobi branch of solve_pressure_fast in 3-D, zero fill included
    (v5.py:337-346): phi = zeros, then `iterations` sweeps.  With ``rhs_ws``
    the first pass starts from the zeros itself (no fill, no RHS prologue, no
    final copy; cfd_jacobi3d_zero_f32).  Returns phi."""
    if phi.dim() != 3:
        raise ValueError("expected (nz, ny, nx)")
    nz, ny, nx = (int(s) for s in phi.shape)
    tmp = torch.empty_like(phi) if phi_tmp is None else phi_tmp
    _f32(phi, "phi")
    for t, name in ((tmp, "phi_tmp"), (rhs_ws, "rhs_ws"), (div, "div")):
        _like(phi, t, name)
    call("cfd_jacobi3d_zero_f32", ptr(_f32(div, "div")), ptr(_f32(phi, "phi")), ptr(tmp), ptr(rhs_ws),
         nz, ny, nx, float(h), float(np.float32(dt)), int(iterations), stream_handle())
    return phi


def solve_pressure_gauss_seidel3d(phi, div, dx, dy, dz, dt, mask, iterations, tolerance,
                                  workspace=None, iters_done=None, phi_tmp=None):
    """3-D red-black generalisation of v5.py:202-226, in place on ``phi``
    (``phi_tmp``: as in solve_pressure_gauss_seidel_fast)."""
    nz, ny, nx = (int(s) for s in phi.shape)
    m = _mask_u8(mask, phi.shape)
    need = int(lib().cfd_rbgs_workspace_bytes(int(iterations)))
    ws = workspace
    if ws is None or ws.numel() * ws.element_size() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=phi.device)
    tmp = torch.empty_like(phi) if phi_tmp is None else _like(phi, phi_tmp, "phi_tmp")
    _like(phi, div, "div")
    call("cfd_rbgs3d_f32", ptr(_f32(phi, "phi")), ptr(_f32(div, "div")), ptr(m), nz, ny, nx, float(dx),
         float(dy), float(dz), float(np.float32(dt)), int(iterations), float(tolerance), ptr(_f32(tmp, "phi_tmp")),
         ptr(ws), ptr(iters_done), stream_handle())
    return phi


def apply_ibm_fast(u, v, ibm_mask, force_strength):
    """v5.py:228-237, in place; ``ibm_mask`` is the float64 mask. Returns (u, v)."""
    if ibm_mask.dtype != torch.float64:
        raise TypeError("ibm_mask is float64 in the reference (v5.py:281-283)")
    call(_fields("cfd_apply_ibm2d", u, v), ptr(u), ptr(v), ptr(ibm_mask), int(u.numel()), float(force_strength),
         stream_handle())
    return u, v


def clean_divergence_fast(u, v, dx, dy, iterations=2, workspace=None):
    """v5.py:239-257, in place; serial (lexicographic) order of the phi sweep."""
    ny, nx = _shape2d(u)
    need = int(lib().cfd_clean_divergence_workspace_bytes(ny, nx))
    ws = workspace
    if ws is None or ws.numel() * ws.element_size() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=u.device)
    call(_fields("cfd_clean_divergence2d", u, v), ptr(u), ptr(v), ny, nx, float(dx), float(dy), int(iterations),
         ptr(ws), stream_handle())
    return u, v


TAU_MODES = {"exact": 0, "fast": 1}


def predictor_fused(u, v, dx, dy, dt, nu_eff, use_supg=True, u_star=None, v_star=None, tau=None, tau_mode=None):
    """v5.py:388-403 in one pass: returns (u_star, v_star, tau).

    tau_mode: "exact" (the reference's NumPy scalar `**`: glibc powf / pow,
    bit-exact), "fast" (the compiled reference's fastmath x*x / sqrt, within
    1e-6 relative L-inf), or None (the calling thread's current setting,
    cfd_set_predictor2d_tau_mode; "exact" unless changed).  A given mode
    applies to this call only: the thread's setting is restored after it.
    Without SUPG a given tau is filled with zeros (the reference's
    never-assigned np.zeros, v5.py:292)."""
    ny, nx = _shape2d(u)
    if tau_mode is not None and tau_mode not in TAU_MODES:
        raise ValueError(f"tau_mode must be one of {sorted(TAU_MODES)}, not {tau_mode!r}")
    us = torch.empty_like(u) if u_star is None else u_star
    vs = torch.empty_like(v) if v_star is None else v_star
    if tau is None and use_supg:
        tau = torch.empty_like(u)
    nu_a, nu_s = _nu(nu_eff, u.dtype)
    prev = None
    if tau_mode is not None:
        prev = int(lib().cfd_get_predictor2d_tau_mode())
        if prev != TAU_MODES[tau_mode]:
            call("cfd_set_predictor2d_tau_mode", TAU_MODES[tau_mode])
        else:
            prev = None
    try:
        call(_fields("cfd_predictor2d", u, v, us, vs, tau), ptr(u), ptr(v), ptr(nu_a), nu_s, ptr(us), ptr(vs),
             ptr(tau), ny, nx, float(dx), float(dy), _dt_arg(dt, u.dtype), int(bool(use_supg)),
             stream_handle())
    finally:
        if prev is not None:
            call("cfd_set_predictor2d_tau_mode", prev)
    return us, vs, tau


def project_velocity(phi, u_star, v_star, dx, dy, dt, u=None, v=None, gradmax=None):
    """v5.py:413-417: u = u* - dt*dphi/dx, v = v* - dt*dphi/dy.  Returns (u, v)."""
    ny, nx = _shape2d(phi)
    u = torch.empty_like(u_star) if u is None else u
    v = torch.empty_like(v_star) if v is None else v
    call(_fields("cfd_project2d", phi, u_star, v_star, u, v, gradmax), ptr(phi), ptr(u_star), ptr(v_star), ptr(u),
         ptr(v), ny, nx, float(dx), float(dy), _dt_arg(dt, phi.dtype), ptr(gradmax), stream_handle())
    return u, v


def persistent_failures(stream=None) -> int:
    """How many persistent small-grid solves (the one-launch 2-D Jacobi /
    red-black GS) run on ``stream`` (default: the current stream) had a tile
    wait expire since the last call; their phi is all NaN.  Reads and clears
    that stream's failure word with an async copy and synchronises that
    stream only (cfd_persistent_status_stream): solvers on other streams keep
    running and keep their own counts."""
    import ctypes
    n = ctypes.c_int(0)
    call("cfd_persistent_status_stream", stream_handle(stream), ctypes.byref(n))
    return int(n.value)
