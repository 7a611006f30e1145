"""GPU drop-in for the reference cylinder solver's time-stepping path.

``OptimizedTurbulentConfig`` and ``OptimizedTurbulentSolver`` keep the field
names, method names and return values of
``python/flow_over_cylinder (Fischer)/v5.py:41-441``.  The fields (``u``, ``v``,
``phi``, ``u_star``, ...) are torch tensors on the HIP device, float32
(``memory_efficient=True``, the reference default) or float64 (False,
v5.py:287).  Every
per-step array pass runs in libcfdsim's gfx950 kernels, and the step needs no
host synchronisation (except adaptive dt after step 1000, which, like the
reference, reads max|V|).

Out of scope: LES (``use_les=True`` raises,
v5.py:60,381-384), plotting and video (OptimizedVisualizer), and HDF5 output
(h5py is absent; ``save_snapshot`` writes the same layout to ``.npz``).
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import kernels as K
from ._lib import call, ptr, stream_handle, lib


@dataclass
class OptimizedTurbulentConfig:
    """v5.py:41-94; same fields, defaults and derived values (dx, dy, and the
    float32 casts of nu, dt and artificial_viscosity, v5.py:78-83)."""
    L: float = 1.0
    R_cylinder: float = 0.5
    V_inf: float = 1.0
    cylinder_center: tuple = (4.0, 2.0)
    x_min: float = 0.0
    x_max: float = 20.0
    y_min: float = 0.0
    y_max: float = 4.0
    nx: int = 600
    ny: int = 180
    T_total: float = 30.0
    dt_base: float = 0.00005
    cfl_target: float = 0.1
    adaptive_dt: bool = True
    dt_min: float = 1e-6
    dt_max: float = 0.0001
    Re: float = 600.0
    use_les: bool = False
    smagorinsky_constant: float = 0.0
    use_supg: bool = True
    artificial_viscosity: float = 0.001
    pressure_iterations: int = 1500
    pressure_tolerance: float = 1e-8
    max_velocity: float = 5.0
    initial_steps: int = 1000
    parallel_threads: int = 4
    use_fast_pressure: bool = True
    memory_efficient: bool = True
    vectorized_ops: bool = True
    save_interval: int = 200
    output_dir: str = "v5_re_600"
    hdf5_file: str = "v5_re_600.h5"
    dpi: int = 200
    # build-only knobs (not in the reference)
    log_diagnostics: bool = False   # compute the v5.py:410-435 log values on device
    # SUPG tau arithmetic: "exact" = the reference's NumPy scalar `**` (glibc
    # powf / pow; bit-exact time_step), "fast" = the compiled reference's
    # fastmath form (x*x, correctly rounded sqrt; within 1e-6 relative L-inf)
    supg_tau: str = "exact"
    device: str = "cuda"

    def __post_init__(self):
        self.dx = (self.x_max - self.x_min) / (self.nx - 1)
        self.dy = (self.y_max - self.y_min) / (self.ny - 1)
        self.nu = np.float32(1.0 / self.Re)
        self.dt = np.float32(self.dt_base)
        self.artificial_viscosity = np.float32(self.artificial_viscosity)
        self.parallel_threads = min(self.parallel_threads, os.cpu_count() or 1)
        if self.supg_tau not in ("exact", "fast"):
            raise ValueError(f"supg_tau must be 'exact' or 'fast', not {self.supg_tau!r}")


# ------------------------------------------------------------ host setup
# One-time host-side setup, kept as pure NumPy functions so the CPU tests can
# check them against the reference-generated fixtures without a GPU.
def host_grid(cfg):
    """setup_grid, v5.py:269-273."""
    x = np.linspace(cfg.x_min, cfg.x_max, cfg.nx)
    y = np.linspace(cfg.y_min, cfg.y_max, cfg.ny)
    X, Y = np.meshgrid(x, y, indexing="xy")
    return x, y, X, Y


def host_masks(cfg, X, Y):
    """setup_boundary_masks, v5.py:275-283: (dist, cylinder_mask, ibm_mask)."""
    x_c, y_c = cfg.cylinder_center
    dist = np.sqrt((X - x_c) ** 2 + (Y - y_c) ** 2)
    cyl = dist <= cfg.R_cylinder
    sigma = 2 * cfg.dx
    ibm = np.exp(-((dist - cfg.R_cylinder) / sigma) ** 2)
    ibm = np.where(dist < cfg.R_cylinder, 1.0,
                   np.where(dist < cfg.R_cylinder + 5 * cfg.dx, ibm, 0.0))
    return dist, cyl, ibm


def host_potential_flow(cfg, X, Y, dist, ibm_mask, dtype=np.float32):
    """initialize_potential_flow, v5.py:299-314, vectorised (same formulas,
    float64 then cast to the fields' dtype on assignment: float32, or float64
    when memory_efficient=False)."""
    x_c, y_c = cfg.cylinder_center
    r, m = dist, ibm_mask
    u = np.zeros((cfg.ny, cfg.nx), dtype)
    v = np.zeros((cfg.ny, cfg.nx), dtype)
    if dtype == np.float64:
        # float64 keeps every bit of the per-cell scalar arithmetic: NumPy
        # float64 scalar `**` is libm pow and scalar sin / cos take the scalar
        # loops, which the vectorised array forms below do not reproduce to
        # the last bit (float32 rounding hides that), so restate the loop
        for i in range(cfg.ny):
            for j in range(cfg.nx):
                rij, mv = r[i, j], m[i, j]
                if rij > cfg.R_cylinder + 4 * cfg.dx:
                    theta = np.arctan2(Y[i, j] - y_c, X[i, j] - x_c)
                    factor = (cfg.R_cylinder / rij) ** 2
                    u[i, j] = cfg.V_inf * (1 - factor * np.cos(2 * theta)) * (1 - mv)
                    v[i, j] = -cfg.V_inf * factor * np.sin(2 * theta) * (1 - mv)
                else:
                    blend = min(1.0, ((rij - cfg.R_cylinder) / (4 * cfg.dx)) ** 2)
                    u[i, j] = cfg.V_inf * blend * (1 - mv)
        return u, v
    far = r > cfg.R_cylinder + 4 * cfg.dx
    with np.errstate(divide="ignore", invalid="ignore"):
        theta = np.arctan2(Y - y_c, X - x_c)
        factor = (cfg.R_cylinder / r) ** 2
        u_far = cfg.V_inf * (1 - factor * np.cos(2 * theta)) * (1 - m)
        v_far = -cfg.V_inf * factor * np.sin(2 * theta) * (1 - m)
    blend = np.minimum(1.0, ((r - cfg.R_cylinder) / (4 * cfg.dx)) ** 2)
    u_near = cfg.V_inf * blend * (1 - m)
    u[far] = u_far[far]
    v[far] = v_far[far]
    u[~far] = u_near[~far]
    return u, v


class OptimizedTurbulentSolver:
    """v5.py:259-441 on the GPU.  Array attributes are device tensors."""

    def __init__(self, config: OptimizedTurbulentConfig):
        if config.use_les:
            raise NotImplementedError("use_les=True is out of scope (LES is off in v3-v5, v5.py:60)")
        self.config = config
        # v5.py:287: float32 fields when memory_efficient, else float64
        self.dtype = torch.float32 if config.memory_efficient else torch.float64
        self._sfx = "_f32" if config.memory_efficient else "_f64"
        self._np = np.float32 if config.memory_efficient else np.float64
        self.device = torch.device(config.device)
        if self.device.type != "cuda":
            raise TypeError("OptimizedTurbulentSolver runs on the HIP device only")
        self._has_ibm = True  # immersed-boundary forcing (the cylinder); the cavity has none
        self.setup_grid()
        self.setup_boundary_masks()
        self.initialize_fields()
        self.step = 0
        self._energy = torch.zeros(1024, dtype=torch.float64, device=self.device)
        self._energy_steps = []
        self.times = []

    # ------------------------------------------------------------- setup
    def setup_grid(self):  # v5.py:269-273 (host, one-time)
        self.x, self.y, self.X, self.Y = host_grid(self.config)
        self._y_dev = torch.from_numpy(self.y).to(self.device)

    def setup_boundary_masks(self):  # v5.py:275-283 (host, one-time)
        self.dist, cyl, ibm = host_masks(self.config, self.X, self.Y)
        self.cylinder_mask_host = cyl
        self.ibm_mask_host = ibm
        self.cylinder_mask = torch.from_numpy(cyl).to(self.device)
        self._mask_u8 = self.cylinder_mask.to(torch.uint8)
        self.ibm_mask = torch.from_numpy(ibm).to(self.device)

    def initialize_fields(self):  # v5.py:285-297
        cfg = self.config
        shape = (cfg.ny, cfg.nx)
        z = lambda: torch.zeros(shape, dtype=self.dtype, device=self.device)  # noqa: E731
        self.u, self.v, self.p, self.nu_t, self.tau_supg = z(), z(), z(), z(), z()
        self.u_star, self.v_star, self.div_u_star, self.phi = z(), z(), z(), z()
        self._phi_tmp = z()
        self._rhs_ws = z()
        # the GS workspace (small float32 grids: with the persistent solve's rings)
        self._gs_ws = torch.empty(int(lib().cfd_rbgs2d_workspace_bytes(cfg.ny, cfg.nx, cfg.pressure_iterations)),
                                  dtype=torch.uint8, device=self.device)
        self._gs_done = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._clean_ws = torch.empty(int(lib().cfd_clean_divergence_workspace_bytes(cfg.ny, cfg.nx)),
                                     dtype=torch.uint8, device=self.device)
        self._scal = torch.zeros(8, dtype=self.dtype, device=self.device)  # diagnostics
        self.initialize_potential_flow()

    def initialize_potential_flow(self):  # v5.py:299-314 (host, one-time)
        u, v = host_potential_flow(self.config, self.X, self.Y, self.dist, self.ibm_mask_host, self._np)
        self.u.copy_(torch.from_numpy(u))
        self.v.copy_(torch.from_numpy(v))

    # --------------------------------------------------------- step parts
    def adaptive_time_step(self):  # v5.py:316-326
        cfg = self.config
        if not cfg.adaptive_dt:
            return cfg.dt_base
        if self.step < 1000:
            return np.float32(0.00002)
        out = self._scal[0:1]
        out.zero_()
        call("cfd_absmax2" + self._sfx, ptr(self.u), ptr(self.v), self.u.numel(), ptr(out), stream_handle())
        vmax = self._np(out.item())  # the one host read of the step (as in the reference)
        vel_max = max(vmax, 1e-10)
        dt_cfl = cfg.cfl_target * min(cfg.dx, cfg.dy) / vel_max
        nu_total = cfg.nu + self._np(0.0) + cfg.artificial_viscosity  # np.mean(nu_t) == 0 in the fields' dtype
        dt_visc = 0.4 * min(cfg.dx, cfg.dy) ** 2 / nu_total
        return np.float32(np.clip(min(dt_cfl, dt_visc), cfg.dt_min, cfg.dt_max))

    def solve_pressure_fast(self, div_u_star):  # v5.py:328-347
        cfg = self.config
        if cfg.use_fast_pressure:  # phi = zeros (v5.py:337) inside the solve
            K.solve_pressure_gauss_seidel_fast(self.phi, div_u_star, cfg.dx, cfg.dy, cfg.dt,
                                               self._mask_u8, cfg.pressure_iterations,
                                               cfg.pressure_tolerance, workspace=self._gs_ws,
                                               iters_done=self._gs_done, phi_tmp=self._phi_tmp,
                                               zero_start=True)
        else:  # phi = zeros (v5.py:337) inside the solve
            K.solve_pressure_jacobi(self.phi, div_u_star, cfg.dx, cfg.dt, self._mask_u8,
                                    cfg.pressure_iterations, phi_tmp=self._phi_tmp, rhs_ws=self._rhs_ws,
                                    zero_start=True)
        return self.phi

    def apply_boundary_conditions(self, u, v):  # v5.py:349-360
        cfg = self.config
        call("cfd_apply_bc2d" + self._sfx, ptr(u), ptr(v), ptr(self._y_dev), cfg.ny, cfg.nx, float(cfg.y_max),
             float(cfg.V_inf), int(self.step), stream_handle())

    def _bc_ibm(self, u, v, force_strength):
        """apply_boundary_conditions followed by apply_ibm_fast (when the
        cylinder mask exists) as one kernel, bit-identical to the two calls.
        A subclass with its own boundary conditions (the lid-driven cavity)
        gets its method, then the IBM call."""
        cfg = self.config
        if type(self).apply_boundary_conditions is not OptimizedTurbulentSolver.apply_boundary_conditions:
            self.apply_boundary_conditions(u, v)
            if self._has_ibm:
                K.apply_ibm_fast(u, v, self.ibm_mask, force_strength)
            return
        call("cfd_apply_bc_ibm2d" + self._sfx, ptr(u), ptr(v), ptr(self._y_dev), cfg.ny, cfg.nx, float(cfg.y_max),
             float(cfg.V_inf), int(self.step), ptr(self.ibm_mask) if self._has_ibm else None, float(force_strength),
             stream_handle())

    def compute_energy(self):  # v5.py:362-363
        return 0.5 * (self.u ** 2 + self.v ** 2)

    def compute_vorticity(self):  # v5.py:365-373
        cfg = self.config
        w = torch.empty_like(self.u)
        if self.dtype == torch.float64:
            call("cfd_vorticity2d_f64", ptr(self.u), ptr(self.v), ptr(self._mask_u8), ptr(w), None, cfg.ny,
                 cfg.nx, float(cfg.dx), float(cfg.dy), stream_handle())
        else:
            call("cfd_vorticity2d_f32", ptr(self.u), ptr(self.v), ptr(self._mask_u8), ptr(w), cfg.ny, cfg.nx,
                 float(cfg.dx), float(cfg.dy), stream_handle())
        return w

    @property
    def energy_history(self):
        """[(step, mean kinetic energy)] like v5.py:433; read lazily from the
        device so time_step() never synchronises for it."""
        n = len(self._energy_steps)
        vals = self._energy[:n].cpu().numpy() if n else np.zeros(0)
        return [(s, float(e)) for s, e in zip(self._energy_steps, vals)]

    @property
    def diagnostics(self):
        """The last step's log values (v5.py:410, 415, 422, 428-432), the same
        numbers the reference prints: max|div u*| before the pressure solve,
        max|grad phi|, max|div u| after the cleaning, nanmax|vorticity| (the
        first four need log_diagnostics=True) and the mean kinetic energy."""
        d = self._scal[1:5].cpu().numpy()
        n = len(self._energy_steps)
        e = float(self._energy[n - 1].item()) if n else float("nan")
        return {"pre_div_max": float(d[0]), "grad_max": float(d[1]), "post_div_max": float(d[2]),
                "vorticity_max": float(d[3]), "energy_mean": e}

    def log_lines(self):
        """The reference's five per-step INFO lines (v5.py:410-435) for the
        last step, formatted as it formats them (log_diagnostics=True)."""
        d, k = self.diagnostics, self.step - 1
        return [f"Step {k}: Pre-pressure divergence = {d['pre_div_max']:.3f}",
                f"Step {k}: Max pressure gradient = {d['grad_max']:.3f}",
                f"Step {k}: Post-pressure divergence = {d['post_div_max']:.3f}",
                f"Step {k}: Max vorticity = {d['vorticity_max']:.3f}",
                f"Step {k}: Mean kinetic energy = {d['energy_mean']:.3f}"]

    def _energy_slot(self):
        k = len(self._energy_steps)
        if k >= self._energy.numel():
            grown = torch.zeros(2 * self._energy.numel(), dtype=torch.float64, device=self.device)
            grown[:k] = self._energy[:k]
            self._energy = grown
        return self._energy[k:k + 1]

    def time_step(self):  # v5.py:375-441
        cfg = self.config
        s = stream_handle()
        diag = cfg.log_diagnostics
        dt = self.adaptive_time_step()
        if diag:
            self._scal[1:5].zero_()
        # predictor (v5.py:378-403): u_old/v_old are read-only here, so u/v are used directly;
        # nu_eff = nu + nu_t + art_visc with nu_t == 0 in the fields' dtype (v5.py:388)
        nu_eff = self._np(self._np(cfg.nu) + self._np(0.0)) + self._np(cfg.artificial_viscosity)
        K.predictor_fused(self.u, self.v, cfg.dx, cfg.dy, dt, nu_eff, cfg.use_supg,
                          u_star=self.u_star, v_star=self.v_star, tau=self.tau_supg, tau_mode=cfg.supg_tau)
        # (without SUPG the predictor writes tau_supg's zeros itself)
        force_strength = min(1.0, self.step / cfg.initial_steps)
        # apply_boundary_conditions then apply_ibm_fast (v5.py:405-407), one launch
        self._bc_ibm(self.u_star, self.v_star, force_strength)
        call("cfd_divergence2d" + self._sfx, ptr(self.u_star), ptr(self.v_star), ptr(self.div_u_star), cfg.ny,
             cfg.nx, float(cfg.dx), float(cfg.dy), ptr(self._scal[1:2]) if diag else None, s)
        self.solve_pressure_fast(self.div_u_star)
        K.project_velocity(self.phi, self.u_star, self.v_star, cfg.dx, cfg.dy, dt, u=self.u, v=self.v,
                           gradmax=self._scal[2:3] if diag else None)
        K.clean_divergence_fast(self.u, self.v, cfg.dx, cfg.dy, iterations=2, workspace=self._clean_ws)
        if diag:
            call("cfd_divergence2d" + self._sfx, ptr(self.u), ptr(self.v), ptr(self.div_u_star), cfg.ny, cfg.nx,
                 float(cfg.dx), float(cfg.dy), ptr(self._scal[3:4]), s)
            # the reference recomputes div for logging only; keep div_u_star as the pre-pressure one
            call("cfd_divergence2d" + self._sfx, ptr(self.u_star), ptr(self.v_star), ptr(self.div_u_star),
                 cfg.ny, cfg.nx, float(cfg.dx), float(cfg.dy), None, s)
        self._bc_ibm(self.u, self.v, force_strength)  # v5.py:424-425
        if diag and self.dtype == torch.float64:
            call("cfd_vorticity2d_f64", ptr(self.u), ptr(self.v), ptr(self._mask_u8), None, ptr(self._scal[4:5]),
                 cfg.ny, cfg.nx, float(cfg.dx), float(cfg.dy), s)
        elif diag:
            call("cfd_vorticity_absmax2d_f32", ptr(self.u), ptr(self.v), ptr(self._mask_u8), cfg.ny,
                 cfg.nx, float(cfg.dx), float(cfg.dy), ptr(self._scal[4:5]), s)
        # the energy of the unclipped fields (v5.py:431-435), then both clips (v5.py:437-438)
        call("cfd_energy_mean_clip2d" + self._sfx, ptr(self.u), ptr(self.v), self.u.numel(),
             ptr(self._energy_slot()), -float(cfg.max_velocity), float(cfg.max_velocity), s)
        self._energy_steps.append(self.step)
        self.times.append(self.step * dt)
        self.step += 1
        return dt

    # ------------------------------------------------------------ output
    def save_snapshot(self, path, step: int, current_time: float):
        """save_data_to_hdf5 layout (v5.py:454-470) as .npz (h5py is absent):
        group step_%06d with u, v, vorticity, X, Y and the time attribute.
        Like the reference's file (opened in append mode, a group written
        once, v5.py:457-458), an existing snapshot file keeps its groups and
        gains this one: the new group's arrays are appended as members of the
        .npz zip archive, so a save costs O(one group) however many the file
        holds, and a group already present is left alone without reading the
        device.  phi and the step counter are added (the reference stores
        neither) so that load_snapshot restarts the run exactly."""
        import zipfile
        g = f"step_{step:06d}"
        exists = os.path.exists(path)
        if exists:
            with zipfile.ZipFile(path, "r") as z:
                if f"{g}/u.npy" in z.namelist():  # `if group_name not in f` (v5.py:458)
                    return
        groups = {f"{g}/u": self.u.cpu().numpy(), f"{g}/v": self.v.cpu().numpy(),
                  f"{g}/vorticity": self.compute_vorticity().cpu().numpy(),
                  f"{g}/X": self.X, f"{g}/Y": self.Y, f"{g}/phi": self.phi.cpu().numpy(),
                  f"{g}/time": np.float64(current_time), f"{g}/solver_step": np.int64(self.step)}
        with zipfile.ZipFile(path, "a" if exists else "w", compression=zipfile.ZIP_DEFLATED) as z:
            for k, arr in groups.items():
                with z.open(f"{k}.npy", "w", force_zip64=True) as f:
                    np.lib.format.write_array(f, np.asanyarray(arr), allow_pickle=False)

    def load_snapshot(self, path, step=None):
        """Restart from a save_snapshot file: group step_%06d (the latest
        when ``step`` is None) gives u, v, phi and the step counter; returns
        the stored time.  The next time_step() then equals the uninterrupted
        run's bit for bit: a step reads only u, v and the counter (phi is
        zero-filled before each solve, v5.py:331/337)."""
        with np.load(path, allow_pickle=False) as f:
            steps = sorted({int(k.split("/")[0][5:]) for k in f.files if k.startswith("step_")})
            if not steps:
                raise ValueError(f"{path}: no step_%06d groups")
            g = f"step_{(steps[-1] if step is None else int(step)):06d}"
            if f"{g}/u" not in f.files:
                raise KeyError(f"{path}: no group {g} (have {steps})")
            shape = (self.config.ny, self.config.nx)
            if f[f"{g}/u"].shape != shape:
                raise ValueError(f"{path}: {g} holds a {f[f'{g}/u'].shape} grid, the solver {shape}")
            self.u.copy_(torch.from_numpy(f[f"{g}/u"]))
            self.v.copy_(torch.from_numpy(f[f"{g}/v"]))
            self.phi.copy_(torch.from_numpy(f[f"{g}/phi"]))
            self.step = int(f[f"{g}/solver_step"]) if f"{g}/solver_step" in f.files else int(g[5:])
            return float(f[f"{g}/time"])


# ------------------------------------------------------ lid-driven cavity
@dataclass
class LidDrivenCavityConfig(OptimizedTurbulentConfig):
    """BASELINE.json config 1: the 2-D lid-driven cavity, 128 x 128, Re = 100,
    500 Jacobi iterations per pressure solve.  The reference has no
    incompressible cavity (its SWA cavity is compressible Euler,
    SWA/cavity_flow_v1.py:39-69), so this is the v5 projection step
    (v5.py:375-441, every kernel and quirk unchanged) on the unit square with
    cavity walls instead of the cylinder channel's inlet / outlet / IBM:
    nu = 1/Re = 0.01, artificial viscosity 1e-3, the
    NumPy Jacobi branch (use_fast_pressure=False), fluid at rest initially."""
    x_max: float = 1.0
    y_max: float = 1.0
    nx: int = 128
    ny: int = 128
    Re: float = 100.0
    artificial_viscosity: float = 0.001
    pressure_iterations: int = 500
    use_fast_pressure: bool = False
    lid_velocity: float = 1.0
    output_dir: str = "cavity_re_100"
    hdf5_file: str = "cavity_re_100.h5"


def host_lid_bc(u, v, u_lid):
    """The cavity walls on host arrays (what cfd_apply_lid_bc2d_f32 does):
    no-slip left / right / bottom, the lid u = u_lid on the top row, written
    last so it owns the top corners (the assignment pattern of v5.py:349-360)."""
    u[:, 0] = 0
    v[:, 0] = 0
    u[:, -1] = 0
    v[:, -1] = 0
    u[0, :] = 0
    v[0, :] = 0
    u[-1, :] = np.float32(u_lid)
    v[-1, :] = 0


class LidDrivenCavitySolver(OptimizedTurbulentSolver):
    """The v5 time step (OptimizedTurbulentSolver.time_step) on the lid-driven
    cavity: no solid cells (no mask, no IBM forcing), cavity walls as the
    boundary conditions, zero initial velocity."""

    def __init__(self, config: LidDrivenCavityConfig):
        super().__init__(config)
        self._has_ibm = False

    def setup_boundary_masks(self):
        cfg = self.config
        self.dist = None
        self.cylinder_mask_host = np.zeros((cfg.ny, cfg.nx), bool)
        self.ibm_mask_host = np.zeros((cfg.ny, cfg.nx), np.float64)
        self.cylinder_mask = torch.from_numpy(self.cylinder_mask_host).to(self.device)
        self._mask_u8 = None  # no solid cells: the sweeps skip the mask read
        self.ibm_mask = torch.from_numpy(self.ibm_mask_host).to(self.device)

    def initialize_potential_flow(self):
        self.u.zero_()
        self.v.zero_()

    def apply_boundary_conditions(self, u, v):
        call("cfd_apply_lid_bc2d" + self._sfx, ptr(u), ptr(v), self.config.ny, self.config.nx,
             float(self._np(self.config.lid_velocity)), stream_handle())


def monitor_simulation_health(solver: OptimizedTurbulentSolver, step: int) -> bool:
    """v5.py:599-613 as device reductions with one host read."""
    cfg = solver.config
    s = stream_handle()
    sfx = "_f32" if solver.u.dtype == torch.float32 else "_f64"
    cnt = torch.zeros(1, dtype=torch.int32, device=solver.device)
    red = torch.zeros(2, dtype=solver.u.dtype, device=solver.device)
    call("cfd_nonfinite_count" + sfx, ptr(solver.u), ptr(solver.v), solver.u.numel(), ptr(cnt), s)
    call("cfd_absmax2" + sfx, ptr(solver.u), ptr(solver.v), solver.u.numel(), ptr(red[0:1]), s)
    div = torch.empty_like(solver.u)
    call("cfd_divergence2d" + sfx, ptr(solver.u), ptr(solver.v), ptr(div), cfg.ny, cfg.nx, float(cfg.dx),
         float(cfg.dy), ptr(red[1:2]), s)
    n_bad = int(cnt.item())
    vel_max, div_max = (float(x) for x in red.cpu().numpy())
    # a persistent pressure solve whose tiles could not all run (a wait for a
    # neighbour tile expired) left phi all NaN: a failed step, reported here
    if K.persistent_failures():
        logging.getLogger(__name__).error("Step %d: a persistent pressure solve failed (a tile wait expired)",
                                          step)
        return False
    if n_bad:
        return False
    if vel_max > cfg.max_velocity:
        return False
    div_threshold = 20.0 if step <= 1000 else 2.0
    return not (div_max > div_threshold)
