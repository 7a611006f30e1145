"""Generate the golden parity fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container, where the read-only reference checkout lives at
/root/reference.  It imports the reference's canonical solver module
``python/flow_over_cylinder (Fischer)/v5.py`` with two absent third-party
modules stubbed:

* ``numba`` -> ``njit`` is an identity decorator and ``prange`` is ``range``
  (so every ``@njit`` kernel runs as serial, interpreted NumPy-scalar code;
  see SURVEY.md section 8c for what that means for fidelity), and
* ``h5py`` -> an empty module (only used for snapshots, never called here).

Nothing from the reference is copied: this script only CALLS the reference's
functions and methods on seeded synthetic inputs and stores the inputs and the
outputs as ``.npz`` data.  The fixtures travel to the GPU box; this script and
the reference do not need to.

Usage:  python tests/golden/make_golden.py            (regenerates every fixture)
"""
from __future__ import annotations

import contextlib
import importlib.util
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

REF_FILE = Path("/root/reference/python/flow_over_cylinder (Fischer)/v5.py")
OUT = Path(__file__).resolve().parent


def _install_stubs() -> None:
    numba = types.ModuleType("numba")

    def njit(*args, **kwargs):
        if len(args) == 1 and callable(args[0]) and not kwargs:
            return args[0]
        return lambda f: f

    numba.njit = njit
    numba.prange = range
    sys.modules["numba"] = numba
    sys.modules["h5py"] = types.ModuleType("h5py")


def load_reference():
    """Import v5.py (module name ``ref_v5``) from a scratch cwd: its import
    creates ``logs/`` in the working directory (v5.py:27-34)."""
    _install_stubs()
    scratch = tempfile.mkdtemp(prefix="ref_v5_")
    cwd = os.getcwd()
    os.chdir(scratch)
    try:
        spec = importlib.util.spec_from_file_location("ref_v5", REF_FILE)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    # keep the reference's logger quiet and away from the repo
    import logging
    mod.logger.handlers.clear()
    mod.logger.addHandler(logging.NullHandler())
    mod.logger.propagate = False
    return mod


def disk_mask(ny: int, nx: int, cy: float, cx: float, r: float) -> np.ndarray:
    yy, xx = np.mgrid[0:ny, 0:nx]
    return (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r


@contextlib.contextmanager
def _quiet_cwd():
    scratch = tempfile.mkdtemp(prefix="ref_v5_run_")
    cwd = os.getcwd()
    os.chdir(scratch)
    try:
        yield
    finally:
        os.chdir(cwd)


def make_cfg(ref, **kw):
    with _quiet_cwd():
        return ref.OptimizedTurbulentConfig(**kw)


def gen_jacobi(ref) -> None:
    """Reference Jacobi branch, OptimizedTurbulentSolver.solve_pressure_fast
    with use_fast_pressure=False (v5.py:336-346), 128x128, 500 iterations."""
    n, iters = 128, 500
    for dtype, mem_eff in ((np.float32, True), (np.float64, False)):
        for masked in (False, True):
            cfg = make_cfg(ref, nx=n, ny=n, x_min=0.0, x_max=1.0, y_min=0.0, y_max=1.0,
                           dt_base=5e-5, use_fast_pressure=False, pressure_iterations=iters,
                           memory_efficient=mem_eff, cylinder_center=(0.3, 0.55), R_cylinder=0.12)
            with _quiet_cwd():
                solver = ref.OptimizedTurbulentSolver(cfg)
            rng = np.random.default_rng(1234)
            div = rng.standard_normal((n, n)).astype(dtype)
            mask = solver.cylinder_mask.copy() if masked else np.zeros((n, n), dtype=bool)
            solver.cylinder_mask = mask
            phi = solver.solve_pressure_fast(div).copy()
            tag = "f32" if dtype is np.float32 else "f64"
            name = f"jacobi2d_{tag}_{n}x{n}_it{iters}_seed1234{'_mask' if masked else ''}.npz"
            np.savez_compressed(OUT / name, div=div, mask=mask, phi=phi,
                                dx=np.float64(cfg.dx), dt=np.float32(cfg.dt), iters=np.int64(iters))
            print("wrote", name, phi.dtype, float(np.abs(phi).max()))


def gen_jacobi_rect(ref) -> None:
    """Non-square, dx != dy Jacobi case (the branch uses dx only, v5.py:343)."""
    ny, nx, iters = 40, 72, 60
    cfg = make_cfg(ref, nx=nx, ny=ny, dt_base=5e-5, use_fast_pressure=False,
                   pressure_iterations=iters, memory_efficient=True,
                   cylinder_center=(4.0, 2.0), R_cylinder=0.5)
    with _quiet_cwd():
        solver = ref.OptimizedTurbulentSolver(cfg)
    rng = np.random.default_rng(99)
    div = (rng.standard_normal((ny, nx)) * 3).astype(np.float32)
    phi = solver.solve_pressure_fast(div).copy()
    np.savez_compressed(OUT / "jacobi2d_f32_40x72_it60_cyl.npz", div=div, mask=solver.cylinder_mask,
                        phi=phi, dx=np.float64(cfg.dx), dt=np.float32(cfg.dt), iters=np.int64(iters))
    print("wrote jacobi2d_f32_40x72_it60_cyl.npz")


def gen_rbgs(ref) -> None:
    """Module-level solve_pressure_gauss_seidel_fast (v5.py:202-226), serial."""
    ny, nx = 64, 64
    dx, dy = 1.0 / 63.0, 1.0 / 63.0
    dt = np.float32(5e-5)
    rng = np.random.default_rng(7)
    div = rng.standard_normal((ny, nx)).astype(np.float32)
    cases = [("rbgs2d_f32_64x64_it20_seed7.npz", 20, 1e-8, np.zeros((ny, nx), bool), dx, dy)]
    mask = disk_mask(ny, nx, 30.0, 22.0, 9.0)
    cases.append(("rbgs2d_f32_64x64_it20_seed7_mask.npz", 20, 1e-8, mask, dx, dy))
    # anisotropic spacing, 48x80
    cases.append(("rbgs2d_f32_48x80_it15_aniso.npz", 15, 1e-8, np.zeros((48, 80), bool), 20 / 79, 4 / 47))
    for name, iters, tol, m, ddx, ddy in cases:
        d = div if m.shape == div.shape else rng.standard_normal(m.shape).astype(np.float32)
        phi = np.zeros(m.shape, np.float32)
        out = ref.solve_pressure_gauss_seidel_fast(phi, d, ddx, ddy, dt, m, iters, tol)
        assert out is phi  # in place, same object (v5.py:223,226)
        np.savez_compressed(OUT / name, div=d, mask=m, phi=phi, dx=np.float64(ddx), dy=np.float64(ddy),
                            dt=dt, iters=np.int64(iters), tol=np.float64(tol))
        print("wrote", name)
    # early-exit case: tolerance reached after a few iterations on a small RHS
    ny2, nx2 = 24, 24
    d2 = rng.standard_normal((ny2, nx2)).astype(np.float32)
    hist = [np.zeros((ny2, nx2), np.float32)]
    for k in range(1, 41):
        p = np.zeros((ny2, nx2), np.float32)
        ref.solve_pressure_gauss_seidel_fast(p, d2, 1.0, 1.0, np.float32(1.0), np.zeros((ny2, nx2), bool), k, 0.0)
        hist.append(p)
    # per-iteration max |change| (each cell is written once per iteration)
    mc = [float(np.abs(hist[k] - hist[k - 1]).max()) for k in range(1, 41)]
    tol = float(np.sqrt(mc[11] * mc[12]))  # break lands mid-way through the run
    hist = hist[1:]
    p = np.zeros((ny2, nx2), np.float32)
    ref.solve_pressure_gauss_seidel_fast(p, d2, 1.0, 1.0, np.float32(1.0), np.zeros((ny2, nx2), bool), 400, tol)
    done = next(k + 1 for k in range(40) if np.array_equal(hist[k], p))
    np.savez_compressed(OUT / "rbgs2d_f32_24x24_earlyexit.npz", div=d2, mask=np.zeros((ny2, nx2), bool), phi=p,
                        dx=np.float64(1.0), dy=np.float64(1.0), dt=np.float32(1.0), iters=np.int64(400),
                        tol=np.float64(tol), iters_done=np.int64(done))
    print("wrote rbgs2d_f32_24x24_earlyexit.npz iters_done", done)


def gen_predictor(ref) -> None:
    """Predictor a6-a10: time_step lines v5.py:380-403 driven through the
    reference's own kernel functions, SUPG and upwind variants."""
    ny, nx = 40, 56
    cfg = make_cfg(ref, nx=nx, ny=ny)
    rng = np.random.default_rng(3)
    u = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    v = rng.uniform(-1, 1, (ny, nx)).astype(np.float32)
    u[5, 7] = 0.0
    v[5, 7] = 0.0  # exercises the |V| <= 1e-10 branch of tau (v5.py:160-161)
    dt = np.float32(0.00002)
    nu_t = np.zeros((ny, nx), np.float32)
    nu_eff = cfg.nu + nu_t + cfg.artificial_viscosity
    tau = ref.compute_supg_stabilization_fast(u, v, cfg.dx, cfg.dy, dt, nu_eff)
    cu = ref.compute_convection_supg_fast(u, v, u, cfg.dx, cfg.dy, tau)
    cv = ref.compute_convection_supg_fast(u, v, v, cfg.dx, cfg.dy, tau)
    lu = ref.compute_laplacian_fast(u, cfg.dx, cfg.dy, nu_eff)
    lv = ref.compute_laplacian_fast(v, cfg.dx, cfg.dy, nu_eff)
    us = u + dt * (-cu + lu)
    vs = v + dt * (-cv + lv)
    uc = ref.compute_convection_fast(u, v, u, cfg.dx, cfg.dy)
    vc = ref.compute_convection_fast(u, v, v, cfg.dx, cfg.dy)
    us_up = u + dt * (-uc + lu)
    vs_up = v + dt * (-vc + lv)
    div = ref.compute_divergence_fast(us, vs, cfg.dx, cfg.dy)
    gx, gy = ref.compute_gradient_fast(us, cfg.dx, cfg.dy)
    np.savez_compressed(OUT / "predictor2d_f32_40x56_seed3.npz", u=u, v=v, dt=dt, dx=np.float64(cfg.dx),
                        dy=np.float64(cfg.dy), nu_eff=nu_eff, tau=tau, conv_u=cu, conv_v=cv, lap_u=lu,
                        lap_v=lv, u_star=us, v_star=vs, conv_u_upwind=uc, conv_v_upwind=vc,
                        u_star_upwind=us_up, v_star_upwind=vs_up, div=div, grad_x=gx, grad_y=gy)
    print("wrote predictor2d_f32_40x56_seed3.npz")


def gen_steps(ref) -> None:
    """Three full OptimizedTurbulentSolver.time_step() calls (v5.py:375-441)
    from the potential-flow initial condition, for both pressure branches."""
    for fast in (True, False):
        cfg = make_cfg(ref, nx=120, ny=36, pressure_iterations=200, use_fast_pressure=fast)
        with _quiet_cwd():
            solver = ref.OptimizedTurbulentSolver(cfg)
        rec = {"u0": solver.u.copy(), "v0": solver.v.copy(), "cylinder_mask": solver.cylinder_mask,
               "ibm_mask": solver.ibm_mask}
        for s in range(3):
            dt = solver.time_step()
            rec[f"dt{s}"] = np.float32(dt)
            rec[f"u{s + 1}"] = solver.u.copy()
            rec[f"v{s + 1}"] = solver.v.copy()
            rec[f"phi{s + 1}"] = solver.phi.copy()
            rec[f"u_star{s + 1}"] = solver.u_star.copy()
            rec[f"v_star{s + 1}"] = solver.v_star.copy()
            rec[f"div{s + 1}"] = solver.div_u_star.copy()
            rec[f"tau{s + 1}"] = solver.tau_supg.copy()
        rec["energy"] = np.array([e for _, e in solver.energy_history], np.float64)
        name = f"step_v5_120x36_n3_{'gs' if fast else 'jacobi'}.npz"
        np.savez_compressed(OUT / name, **rec)
        print("wrote", name)


def _recorders(ref, solver):
    """Wrap the reference's module-level kernels and compute_vorticity so one
    time_step() call exposes the values its log lines print (v5.py:410, 415,
    422, 428-432) at full precision: max|div_u_star|, max|grad phi|, max|post
    div| and nanmax|vorticity|.  The wrappers only record what the reference
    returns; time_step() itself runs unchanged."""
    rec = {"div": [], "grad": [], "vort": []}
    div0, grad0 = ref.compute_divergence_fast, ref.compute_gradient_fast
    vort0 = solver.compute_vorticity

    def div_w(u, v, dx, dy):
        out = div0(u, v, dx, dy)
        rec["div"].append(np.max(np.abs(out)))
        return out

    def grad_w(phi, dx, dy):
        gx, gy = grad0(phi, dx, dy)
        rec["grad"].append(np.max(np.abs(np.sqrt(gx ** 2 + gy ** 2))))
        return gx, gy

    def vort_w():
        w = vort0()
        rec["vort"].append(np.nanmax(np.abs(w)))
        return w

    ref.compute_divergence_fast, ref.compute_gradient_fast = div_w, grad_w
    solver.compute_vorticity = vort_w

    def restore():
        ref.compute_divergence_fast, ref.compute_gradient_fast = div0, grad0
        del solver.compute_vorticity
    return rec, restore


def gen_diagnostics(ref) -> None:
    """The per-step log values of the two 3-step runs of gen_steps, recorded
    at full precision from the reference's own calls (see _recorders), plus
    the log lines themselves (3 decimals, as the reference prints them)."""
    import logging
    for fast in (True, False):
        cfg = make_cfg(ref, nx=120, ny=36, pressure_iterations=200, use_fast_pressure=fast)
        with _quiet_cwd():
            solver = ref.OptimizedTurbulentSolver(cfg)
        lines = []

        class Grab(logging.Handler):
            def emit(self, record):
                lines.append(record.getMessage())
        h = Grab()
        ref.logger.addHandler(h)
        ref.logger.setLevel(logging.INFO)
        rec, restore = _recorders(ref, solver)
        try:
            for _ in range(3):
                solver.time_step()
        finally:
            restore()
            ref.logger.removeHandler(h)
        # per step, compute_divergence_fast runs 4 times (pre-pressure, twice
        # inside clean_divergence_fast, post) and compute_gradient_fast 3 times
        # (the projection, then twice inside clean_divergence_fast)
        assert len(rec["div"]) == 12 and len(rec["grad"]) == 9 and len(rec["vort"]) == 3
        out = {"pre_div_max": np.array(rec["div"][0::4], np.float32),
               "post_div_max": np.array(rec["div"][3::4], np.float32),
               "grad_max": np.array(rec["grad"][0::3], np.float32),
               "vorticity_max": np.array(rec["vort"], np.float32),
               "energy": np.array([e for _, e in solver.energy_history], np.float32),
               "log_lines": np.array(lines)}
        name = f"diag_v5_120x36_n3_{'gs' if fast else 'jacobi'}.npz"
        np.savez_compressed(OUT / name, **out)
        print("wrote", name, len(lines), "log lines")


def gen_steps_late(ref) -> None:
    """Two time_step() calls from the potential-flow state with the step
    counter set to 1000 and to 1500: the CFL / viscous dt branch
    (v5.py:322-326), the saturated IBM force (v5.py:406) and the full inlet
    perturbation ramp (v5.py:351-352), for both pressure branches."""
    for fast in (True, False):
        rec = {}
        for start in (1000, 1500):
            cfg = make_cfg(ref, nx=120, ny=36, pressure_iterations=200, use_fast_pressure=fast)
            with _quiet_cwd():
                solver = ref.OptimizedTurbulentSolver(cfg)
            solver.step = start
            for s in range(2):
                dt = solver.time_step()
                k = f"s{start}_{s + 1}"
                rec[f"dt_{k}"] = np.float32(dt)
                rec[f"u_{k}"] = solver.u.copy()
                rec[f"v_{k}"] = solver.v.copy()
                rec[f"phi_{k}"] = solver.phi.copy()
                rec[f"u_star_{k}"] = solver.u_star.copy()
                rec[f"div_{k}"] = solver.div_u_star.copy()
            rec[f"energy_s{start}"] = np.array([e for _, e in solver.energy_history], np.float64)
        name = f"step_v5_120x36_late_{'gs' if fast else 'jacobi'}.npz"
        np.savez_compressed(OUT / name, **rec)
        print("wrote", name)


def gen_steps_f64(ref) -> None:
    """Three time_step() calls with memory_efficient=False (v5.py:287-296:
    every field float64, the dtype-generic kernels then run in float64), for
    both pressure branches, from the potential-flow initial condition."""
    for fast in (True, False):
        cfg = make_cfg(ref, nx=120, ny=36, pressure_iterations=200, use_fast_pressure=fast,
                       memory_efficient=False)
        with _quiet_cwd():
            solver = ref.OptimizedTurbulentSolver(cfg)
        assert solver.u.dtype == np.float64
        rec = {"u0": solver.u.copy(), "v0": solver.v.copy(), "cylinder_mask": solver.cylinder_mask,
               "ibm_mask": solver.ibm_mask}
        for s in range(3):
            dt = solver.time_step()
            rec[f"dt{s}"] = np.float64(dt)
            for f, a in (("u", solver.u), ("v", solver.v), ("phi", solver.phi), ("u_star", solver.u_star),
                         ("v_star", solver.v_star), ("div", solver.div_u_star), ("tau", solver.tau_supg)):
                rec[f"{f}{s + 1}"] = a.copy()
        rec["energy"] = np.array([e for _, e in solver.energy_history], np.float64)
        name = f"step_v5_120x36_n3_f64_{'gs' if fast else 'jacobi'}.npz"
        np.savez_compressed(OUT / name, **rec)
        print("wrote", name, rec["u3"].dtype)


def gen_steps_fixed_dt(ref) -> None:
    """adaptive_dt=False (v5.py:317-318): adaptive_time_step returns the
    Python float dt_base, which meets the float32 fields under NEP 50 (rounded
    to float32 per operation); two GS-branch steps, and two from step 1500
    (where the adaptive branch would otherwise take the CFL dt)."""
    rec = {}
    for start in (0, 1500):
        cfg = make_cfg(ref, nx=120, ny=36, pressure_iterations=200, adaptive_dt=False, dt_base=7e-5)
        with _quiet_cwd():
            solver = ref.OptimizedTurbulentSolver(cfg)
        solver.step = start
        for s in range(2):
            dt = solver.time_step()
            assert type(dt) is float
            k = f"s{start}_{s + 1}"
            rec[f"dt_{k}"] = np.float64(dt)
            for f, a in (("u", solver.u), ("v", solver.v), ("phi", solver.phi), ("u_star", solver.u_star),
                         ("div", solver.div_u_star), ("tau", solver.tau_supg)):
                rec[f"{f}_{k}"] = a.copy()
        rec[f"energy_s{start}"] = np.array([e for _, e in solver.energy_history], np.float64)
    np.savez_compressed(OUT / "step_v5_120x36_fixed_dt.npz", **rec)
    print("wrote step_v5_120x36_fixed_dt.npz")


def gen_health(ref) -> None:
    """monitor_simulation_health (v5.py:599-613) on crafted states: healthy,
    non-finite u / v, over-speed, and a divergence between the two
    thresholds (20 up to step 1000, 2 after), each at steps 500 and 1500."""
    cfg = make_cfg(ref, nx=120, ny=36)
    with _quiet_cwd():
        solver = ref.OptimizedTurbulentSolver(cfg)
    rng = np.random.default_rng(5)
    u0, v0 = solver.u.copy(), solver.v.copy()
    noisy_u = (u0 + rng.uniform(-0.3, 0.3, u0.shape)).astype(np.float32)
    cases = {"healthy": (u0, v0), "nan_u": (u0.copy(), v0), "inf_v": (u0, v0.copy()),
             "fast_u": (u0.copy(), v0), "at_limit": (u0.copy(), v0), "divergent": (noisy_u, v0)}
    cases["nan_u"][0][7, 9] = np.nan
    cases["inf_v"][1][3, 50] = -np.inf
    cases["fast_u"][0][10, 20] = np.float32(5.25)
    cases["at_limit"][0][10, 20] = np.float32(5.0)
    out = {}
    for name, (u, v) in cases.items():
        solver.u, solver.v = u, v
        div_max = np.max(np.abs(ref.compute_divergence_fast(u, v, cfg.dx, cfg.dy)))
        out[f"{name}_u"], out[f"{name}_v"] = u, v
        out[f"{name}_div_max"] = np.float32(div_max)
        for step in (500, 1500):
            out[f"{name}_ok_{step}"] = np.bool_(ref.monitor_simulation_health(solver, step))
    np.savez_compressed(OUT / "health_v5_120x36.npz", **out)
    print("wrote health_v5_120x36.npz", {k: bool(v) for k, v in out.items() if "_ok_" in k})


GENERATORS = {"jacobi": gen_jacobi, "jacobi_rect": gen_jacobi_rect, "rbgs": gen_rbgs,
              "predictor": gen_predictor, "steps": gen_steps, "diagnostics": gen_diagnostics,
              "steps_late": gen_steps_late, "health": gen_health, "steps_f64": gen_steps_f64,
              "steps_fixed_dt": gen_steps_fixed_dt}


def main() -> None:
    """python tests/golden/make_golden.py [generator ...]  (default: all)"""
    if not REF_FILE.exists():
        raise SystemExit(f"reference not found at {REF_FILE}; fixtures are generated in the build container only")
    names = sys.argv[1:] or list(GENERATORS)
    unknown = [n for n in names if n not in GENERATORS]
    if unknown:
        raise SystemExit(f"unknown generators {unknown}; choose from {list(GENERATORS)}")
    ref = load_reference()
    for n in names:
        GENERATORS[n](ref)


if __name__ == "__main__":
    main()
