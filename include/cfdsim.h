/*
 * cfdsim.h -- C ABI of the MI355X-native pressure-Poisson / predictor hot path.
 *
 * This is the drop-in boundary for the numba-compiled kernels and the two solver
 * methods of the reference cylinder solver
 *   python/flow_over_cylinder (Fischer)/v5.py            (cited as "v5.py:<line>")
 * The reference has no FFI of its own: its boundary is numba's @njit dispatcher
 * (module-level functions, v5.py:96-257) and OptimizedTurbulentSolver's
 * solve_pressure_fast / time_step (v5.py:328, :375).  Each entry point below
 * states the reference symbol it replaces.  INTEGRATION.md shows the ctypes
 * binding a maintainer adds on the reference side.
 *
 * Conventions (all entry points):
 *  - Arrays are caller-owned DEVICE pointers (hipMalloc'd or from any allocator
 *    on the current HIP device), C order, x fastest: 2-D (ny, nx), 3-D
 *    (nz, ny, nx).  Sizes are plain ints.  Nothing is allocated on the hot path.
 *    Workspaces are passed in by the caller, sized by the *_workspace_* helpers.
 *  - `stream` is a hipStream_t passed as void* (NULL = the default stream).
 *    Every call is asynchronous on that stream, with no host synchronisation,
 *    so it can be captured into a hipGraph.
 *  - Return 0 on success, or a negative CFD_E_* code; cfd_last_error() then
 *    gives a thread-local message.  NaN/Inf propagate like the reference
 *    (no numerical error codes, v5.py:599-613 detects them at the driver).
 *  - mask: optional uint8 (ny,nx)/(nz,ny,nx), nonzero = solid cell
 *    (cylinder_mask, v5.py:279); NULL = no solid cells.
 *  - Scalars keep the reference's meaning and type: dx/dy are Python floats
 *    (double here), dt is np.float32 (float here).  The library rounds derived
 *    constants exactly as NumPy's NEP-50 promotion does in the reference.
 */
#ifndef CFDSIM_H
#define CFDSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFD_ABI_VERSION 1

#define CFD_OK 0
#define CFD_E_INVALID (-1)   /* bad argument (shape, pointer, alignment) */
#define CFD_E_HIP (-2)       /* a HIP runtime call failed */
#define CFD_E_COMM (-3)      /* an RCCL call failed */
#define CFD_E_UNSUPPORTED (-4)

int cfd_abi_version(void);
const char *cfd_last_error(void);
/* Name of the gfx target the library's device code was built for ("gfx950"). */
const char *cfd_device_arch(void);

/* ------------------------------------------------------------------ Poisson */

/* Replaces the Jacobi branch of OptimizedTurbulentSolver.solve_pressure_fast,
 * v5.py:336-346 (use_fast_pressure=False):
 *   repeat iters: phi_new = phi; phi_new[1:-1,1:-1] =
 *       0.25*(E + W + N + S - f32(dx**2)*div/dt);  phi_new[mask] = 0
 * Bit-exact with the reference (same op order, no FMA contraction).
 * phi (in/out) holds the initial guess; the reference zero-fills it first
 * (v5.py:337); the caller does that.  phi_tmp is a same-size scratch array.
 * rhs_ws (optional, same size): when given, the RHS f32(dx**2)*div/dt is
 * formed once per solve (the same bits) and the sweeps skip the division.
 * Edges keep their values (Dirichlet), except masked edge cells -> 0.
 * resid_every > 0: after every resid_every-th iteration k, max|phi_new - phi|
 * over updated cells is written to resid_out[k/resid_every - 1] (device array
 * of floor(iters/resid_every) elements; an extension, the reference has none). */
int cfd_jacobi2d_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                     const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                     int resid_every, float *resid_out, void *stream);
/* fp64 fields (memory_efficient=False, v5.py:287); dt promotes exactly. */
/* Both 2-D solves fuse `steps` sweeps per HBM pass (temporal blocking, same
 * bits; a remainder iters % steps runs as a shorter pass): 0 auto (8 on grids
 * that fill the chip with long row chunks, e.g. 8192^2; 2 on small ones such as
 * the 600 x 180 cylinder, where a pass is latency-bound), 1 off,
 * 2..6, 8, 10, 12.  Residual requests and unaligned / nx % (16/sizeof(T)) != 0 arrays
 * always run single sweeps.  (The 2-D red-black GS fuses its two colours per
 * pass unless steps == 1.) */
int cfd_set_jacobi2d_blocking(int steps);
/* 2-D Jacobi sweeps per blocked pass: the set depth, or the large-grid auto
 * depth (8). */
int cfd_get_jacobi2d_levels(void);
/* Blocked 2-D passes at 4, 6 or 8 sweeps without a mask may stage their rows
 * through a per-wave LDS ring filled by LDS-DMA this many rows ahead (4 or 6);
 * 0 = the register march that prefetches one row ahead (the default: it is
 * the faster of the two on MI355X).  Same bits either way (a tuning knob, per
 * host thread like the others). */
int cfd_set_jacobi2d_staging(int rows_ahead);
/* The calling thread's last 2-D Jacobi solve: returns 1 if it ran as one
 * persistent launch (small grids), else 0; *sweeps_per_launch (may be NULL)
 * = the sweeps one launch fused (the iterations, for the persistent solve). */
int cfd_get_last_jacobi2d_path(int *sweeps_per_launch);
int cfd_jacobi2d_f64(const double *div, double *phi, double *phi_tmp, double *rhs_ws,
                     const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                     int resid_every, double *resid_out, void *stream);
/* The reference's whole Jacobi solve, zero fill included (v5.py:337-346):
 * phi = zeros (boundary ring included), then iters sweeps as cfd_jacobi2d_*.
 * The persistent small-grid solve starts from the zeros itself (it reads
 * nothing of phi, and writes every cell); other paths zero-fill phi first. */
int cfd_jacobi2d_zero_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                          const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                          int resid_every, float *resid_out, void *stream);
int cfd_jacobi2d_zero_f64(const double *div, double *phi, double *phi_tmp, double *rhs_ws,
                          const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                          int resid_every, double *resid_out, void *stream);

/* 3-D 7-point generalisation of the same Jacobi template (the reference is
 * 2-D only): phi_new = f32(1/6) * (((((E+W)+N)+S)+U)+D - f32(h*h)*div/dt),
 * six Dirichlet faces held, mask -> 0.  Layout (nz, ny, nx). */
int cfd_jacobi3d_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                     const uint8_t *mask, int nz, int ny, int nx, double h, float dt, int iters,
                     int resid_every, float *resid_out, void *stream);

/* The whole Jacobi branch of solve_pressure_fast in 3-D, v5.py:337-346:
 * phi = zeros (v5.py:337), then iters sweeps of cfd_jacobi3d_f32 -- the same
 * bits as a zero fill followed by cfd_jacobi3d_f32.  With rhs_ws (and nx % 4
 * == 0, 16-byte aligned arrays, blocking on) the first pass starts from the
 * zeros without reading phi, forms rhs_ws itself, and writes the array that
 * makes the last pass land in phi: no fill, no RHS prologue, no final copy.
 * phi's prior contents are ignored; phi_tmp is scratch. */
int cfd_jacobi3d_zero_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws, int nz,
                          int ny, int nx, double h, float dt, int iters, void *stream);

/* Replaces solve_pressure_gauss_seidel_fast, v5.py:202-226 (the
 * use_fast_pressure=True branch, v5.py:330-335): red-black Gauss-Seidel in
 * place on phi; colour 0 = cells with (i+j) odd first; masked cells skipped;
 * stop after the first iteration whose max|change| < tolerance.
 * phi_tmp: same-size scratch (optional).  When given (and nx % 4 == 0, 16-byte
 * aligned arrays, blocking not switched off), each iteration runs as ONE fused
 * out-of-place pass over both colours (ping-pong phi/phi_tmp; the result
 * still ends in phi, bit-identical); NULL = in-place colour passes.  3-D:
 * fused only without a mask.  cfd_set_jacobi2d_blocking(1) /
 * cfd_set_jacobi3d_blocking(1, ...) switch the fused path off.
 * ws: cfd_rbgs_workspace_bytes(iterations) bytes.
 * iters_done (device int*, optional) receives the iteration count executed. */
size_t cfd_rbgs_workspace_bytes(int iterations);
int cfd_rbgs2d_f32(float *phi, const float *div, const uint8_t *mask, int ny, int nx,
                   double dx, double dy, float dt, int iterations, double tolerance,
                   float *phi_tmp, void *ws, int *iters_done, void *stream);
/* The same solve with the workspace's size given.  On small grids (the v5
 * cylinder's 600 x 180) a workspace of cfd_rbgs2d_workspace_bytes(ny, nx,
 * iterations) bytes (with phi_tmp given) lets the whole solve run as ONE
 * persistent launch whose tiles hand their edge cells to each other through
 * the workspace instead of ending a launch every 4 iterations (same bits);
 * a smaller one (>= cfd_rbgs_workspace_bytes(iterations)) takes the
 * launch-per-block path, as cfd_rbgs2d_f32 does.  *iters_done is -1 if a
 * persistent solve's tiles could not all run at once (another kernel held the
 * CUs for 20 s); phi is then garbage. */
size_t cfd_rbgs2d_workspace_bytes(int ny, int nx, int iterations);
int cfd_rbgs2d_f32_ws(float *phi, const float *div, const uint8_t *mask, int ny, int nx,
                      double dx, double dy, float dt, int iterations, double tolerance,
                      float *phi_tmp, void *ws, size_t ws_bytes, int *iters_done, void *stream);
/* The reference's GS solve with its zero fill (v5.py:337: phi = zeros, then
 * the iterations of cfd_rbgs2d_f32_ws; the same bits).  The persistent
 * small-grid solve starts from the zeros itself (it reads nothing of phi and
 * writes every cell); other paths zero-fill phi first.  Replaces
 * solve_pressure_fast's np.zeros + solve_pressure_gauss_seidel_fast
 * (v5.py:337-342). */
int cfd_rbgs2d_zero_f32_ws(float *phi, const float *div, const uint8_t *mask, int ny, int nx,
                           double dx, double dy, float dt, int iterations, double tolerance,
                           float *phi_tmp, void *ws, size_t ws_bytes, int *iters_done, void *stream);
/* 3-D red-black generalisation: colour c updates (z+i+j) parity == (1+c)%2.
 * The fused 3-D path runs cfd_get_rbgs3d_levels() half-sweeps per HBM pass
 * (default 4: two iterations; cfd_set_jacobi3d_blocking(2..4, ...) sets it),
 * a stop inside a pass rolled back on the device. */
int cfd_rbgs3d_f32(float *phi, const float *div, const uint8_t *mask, int nz, int ny, int nx,
                   double dx, double dy, double dz, float dt, int iterations, double tolerance,
                   float *phi_tmp, void *ws, int *iters_done, void *stream);

/* ---------------------------------------------------------------- predictor */

/* compute_supg_stabilization_fast, v5.py:149-162.  nu_eff: (ny,nx) array or
 * NULL to use nu_eff_scalar everywhere (LES off: nu_t == 0, v5.py:386-388). */
int cfd_supg_tau2d_f32(const float *u, const float *v, const float *nu_eff, float nu_eff_scalar,
                       float *tau, int ny, int nx, double dx, double dy, float dt, void *stream);
/* compute_convection_supg_fast, v5.py:127-147 (phi is u or v). */
int cfd_convection_supg2d_f32(const float *u, const float *v, const float *phi, const float *tau,
                              float *conv, int ny, int nx, double dx, double dy, void *stream);
/* compute_convection_fast (first-order upwind), v5.py:112-125. */
int cfd_convection_upwind2d_f32(const float *u, const float *v, const float *phi, float *conv,
                                int ny, int nx, double dx, double dy, void *stream);
/* compute_laplacian_fast, v5.py:164-176. */
int cfd_laplacian2d_f32(const float *phi, const float *nu_eff, float nu_eff_scalar, float *lap,
                        int ny, int nx, double dx, double dy, void *stream);
/* Fused predictor, v5.py:388-403: tau (SUPG), conv_u/v, lap_u/v and
 *   u_star = u + dt*(-conv_u + lap_u),  v_star = v + dt*(-conv_v + lap_v)
 * in one pass over u, v.  tau may be NULL (not stored); with use_supg = 0
 * it is filled with zeros (the reference never assigns its np.zeros tau
 * without SUPG, v5.py:292). */
int cfd_predictor2d_f32(const float *u, const float *v, const float *nu_eff, float nu_eff_scalar,
                        float *u_star, float *v_star, float *tau, int ny, int nx,
                        double dx, double dy, float dt, int use_supg, void *stream);
/* Kernel of cfd_predictor2d_f32 / _f64 (tuning, per host thread; same bits
 * either way): variant 0 = auto (the row-march tile kernel when the arrays are
 * below 2^31 bytes; else one thread per cell), 1 = one thread per cell, 2 =
 * row march where it applies; rows = rows per row-march chunk (0 = auto: every
 * workgroup resident in one round, 2..16 rows); cells_per_lane = adjacent
 * cells per lane of the row march (0 = auto: 2; f32 1, 2, 4; f64 1, 2),
 * halved until nx % it == 0 and every array is aligned to it elements. */
int cfd_set_predictor2d_config(int variant, int rows, int cells_per_lane);
/* SUPG tau arithmetic of cfd_predictor2d_f32 / _f64 (per host thread):
 * 0 = exact (default): |V| = (u**2 + v**2)**0.5 through device copies of
 *     glibc's powf / pow, as the reference's NumPy scalar `**` runs it
 *     (v5.py:155): bit-exact with the reference's time_step;
 * 1 = fast: the compiled reference's fastmath arithmetic (v5.py:149 is
 *     @njit(fastmath=True): x**2 -> x*x, **0.5 -> sqrt): sqrt(u*u + v*v)
 *     correctly rounded, tau's two divisions on the hardware reciprocal plus
 *     one Newton step (f32; IEEE in f64).  Within 1e-6 relative L-infinity of
 *     mode 0 on u*, v*, tau (tests/test_gpu_predictor.py).
 * The one-thread-per-cell kernel (variant 1, or arrays past 2^31 bytes)
 * always computes mode 0. */
int cfd_set_predictor2d_tau_mode(int mode);
/* The calling thread's current tau mode (0 exact / 1 fast). */
int cfd_get_predictor2d_tau_mode(void);
/* The calling thread's last predictor launch: returns 1 = row march, 0 = one
 * thread per cell, -1 = none yet; *tau_mode (0 exact / 1 fast) and
 * *cells_per_lane of that launch (either pointer may be NULL). */
int cfd_get_last_predictor2d_path(int *tau_mode, int *cells_per_lane);

/* compute_divergence_fast, v5.py:178-187.  absmax (device float*, optional):
 * receives max|div| (the v5.py:410 diagnostic); must be zeroed by the caller. */
int cfd_divergence2d_f32(const float *u, const float *v, float *div, int ny, int nx,
                         double dx, double dy, float *absmax, void *stream);
/* compute_gradient_fast, v5.py:189-200. */
int cfd_gradient2d_f32(const float *phi, float *grad_x, float *grad_y, int ny, int nx,
                       double dx, double dy, void *stream);
/* Gradient + projection, v5.py:413-417: u = u_star - dt*dphi/dx, v likewise.
 * gradmax (optional, zeroed by caller): max sqrt(gx^2+gy^2) (v5.py:414-415). */
int cfd_project2d_f32(const float *phi, const float *u_star, const float *v_star,
                      float *u, float *v, int ny, int nx, double dx, double dy, float dt,
                      float *gradmax, void *stream);

/* ----------------------------------------------------------- step epilogue */

/* clean_divergence_fast, v5.py:239-257, with the serial (lexicographic)
 * Gauss-Seidel order of its phi sweep as the defined semantics (under numba's
 * prange that sweep races).  ws: cfd_clean_divergence_workspace_bytes(ny,nx):
 * the f32 path keeps div and phi in a diagonal-major layout of 64-row blocks
 * (DESIGN.md §5 Round-5), past 4 blocks one block per workgroup with a
 * progress word per block in ws (its waits bounded like the persistent
 * solves', an expired one counted for cfd_persistent_status). */
size_t cfd_clean_divergence_workspace_bytes(int ny, int nx);
int cfd_clean_divergence2d_f32(float *u, float *v, int ny, int nx, double dx, double dy,
                               int iterations, void *ws, void *stream);
/* OptimizedTurbulentSolver.apply_boundary_conditions, v5.py:349-360.
 * y: device float64 (ny) grid coordinates (np.linspace, v5.py:272). */
int cfd_apply_bc2d_f32(float *u, float *v, const double *y, int ny, int nx, double y_max,
                       double v_inf, int step, void *stream);
/* Lid-driven cavity walls (BASELINE config 1, the build's own: the reference
 * has no incompressible cavity): u = v = 0 on the left, right and bottom walls,
 * u = u_lid, v = 0 on the top row (the lid owns the top corners); the
 * assignment pattern of v5.py:349-360. */
int cfd_apply_lid_bc2d_f32(float *u, float *v, int ny, int nx, float u_lid, void *stream);
/* apply_ibm_fast, v5.py:228-237: f *= (1 - ibm_mask*force_strength) where ibm_mask > 0,
 * evaluated in float64 like the reference's float64 mask. */
int cfd_apply_ibm2d_f32(float *u, float *v, const double *ibm_mask, int n, double force_strength,
                        void *stream);
/* np.clip(a, lo, hi, out=a), v5.py:437-438. */
int cfd_clip_f32(float *a, size_t n, float lo, float hi, void *stream);
/* The solver step's fused tails (one launch each; the same results as the
 * separate calls in the reference's order):
 *   apply_boundary_conditions then apply_ibm_fast (v5.py:349-360, :228-237;
 *   ibm_mask may be NULL: BC only), and
 *   the mean kinetic energy (v5.py:431-435) of u, v followed by the two
 *   np.clip calls (v5.py:437-438): the energy is of the unclipped values. */
int cfd_apply_bc_ibm2d_f32(float *u, float *v, const double *y, int ny, int nx, double y_max,
                           double v_inf, int step, const double *ibm_mask, double force_strength,
                           void *stream);
int cfd_energy_mean_clip2d_f32(float *u, float *v, size_t n, double *out, float lo, float hi,
                               void *stream);

/* ------------------------------------------------------------- reductions */
/* Each writes one value to a device scalar; the caller zeroes `out` for the
 * max reductions.  Used by the diagnostics (v5.py:410-435), adaptive dt
 * (v5.py:322) and the health monitor (v5.py:599-613). */
int cfd_absmax_f32(const float *a, size_t n, float *out, void *stream);            /* max|a| */
int cfd_absmax2_f32(const float *a, const float *b, size_t n, float *out, void *stream);
int cfd_energy_mean2d_f32(const float *u, const float *v, size_t n, double *out, void *stream);
int cfd_vorticity_absmax2d_f32(const float *u, const float *v, const uint8_t *mask, int ny, int nx,
                               double dx, double dy, float *out, void *stream);
/* compute_vorticity, v5.py:365-373 (masked cells NaN, boundary ring 0). */
int cfd_vorticity2d_f32(const float *u, const float *v, const uint8_t *mask, float *w, int ny,
                        int nx, double dx, double dy, void *stream);
/* out[i] = NumPy's float32 scalar x[i] ** y, i.e. glibc powf (not correctly
 * rounded): the device restatement the SUPG tau uses for the reference's
 * `(u**2 + v**2) ** 0.5` (v5.py:155).  A parity hook. */
int cfd_numpy_powf_f32(const float *x, float y, float *out, size_t n, void *stream);
/* count of non-finite values in a and b (v5.py:601), into a device int. */
int cfd_nonfinite_count_f32(const float *a, const float *b, size_t n, int *out, void *stream);

/* --------------------------------------------------- float64 fields */
/* memory_efficient=False (v5.py:287-296): every field float64; the kernels
 * below are the *_f32 ones above with float64 arrays, the same argument
 * meaning, and the reference's float64 arithmetic (Python-float constants
 * unrounded).  dt is a double here: the step's dt (np.float32, or the Python
 * float dt_base when adaptive_dt=False) meets float64 fields exactly; the
 * pressure solves keep cfg.dt's float32.  The SUPG tau's
 * |V| is the correctly rounded sqrt(u*u + v*v) where the reference calls
 * glibc pow (1 ulp apart on ~1e-3 of cells, fields.hip file comment): a
 * float64 time_step matches the reference within a relative L-inf of 1e-12
 * instead of bit for bit.  cfd_jacobi2d_f64 is above. */
int cfd_supg_tau2d_f64(const double *u, const double *v, const double *nu_eff, double nu_eff_scalar,
                       double *tau, int ny, int nx, double dx, double dy, double dt, void *stream);
int cfd_convection_supg2d_f64(const double *u, const double *v, const double *phi, const double *tau,
                              double *conv, int ny, int nx, double dx, double dy, void *stream);
int cfd_convection_upwind2d_f64(const double *u, const double *v, const double *phi, double *conv,
                                int ny, int nx, double dx, double dy, void *stream);
int cfd_laplacian2d_f64(const double *phi, const double *nu_eff, double nu_eff_scalar, double *lap,
                        int ny, int nx, double dx, double dy, void *stream);
int cfd_predictor2d_f64(const double *u, const double *v, const double *nu_eff, double nu_eff_scalar,
                        double *u_star, double *v_star, double *tau, int ny, int nx, double dx,
                        double dy, double dt, int use_supg, void *stream);
int cfd_divergence2d_f64(const double *u, const double *v, double *div, int ny, int nx, double dx,
                         double dy, double *absmax, void *stream);
int cfd_gradient2d_f64(const double *phi, double *grad_x, double *grad_y, int ny, int nx, double dx,
                       double dy, void *stream);
int cfd_project2d_f64(const double *phi, const double *u_star, const double *v_star, double *u,
                      double *v, int ny, int nx, double dx, double dy, double dt, double *gradmax,
                      void *stream);
/* ws: cfd_clean_divergence_workspace_bytes(ny, nx) (at least two float64 fields) */
int cfd_clean_divergence2d_f64(double *u, double *v, int ny, int nx, double dx, double dy,
                               int iterations, void *ws, void *stream);
int cfd_apply_bc2d_f64(double *u, double *v, const double *y, int ny, int nx, double y_max,
                       double v_inf, int step, void *stream);
int cfd_apply_lid_bc2d_f64(double *u, double *v, int ny, int nx, double u_lid, void *stream);
int cfd_apply_ibm2d_f64(double *u, double *v, const double *ibm_mask, int n, double force_strength,
                        void *stream);
int cfd_clip_f64(double *a, size_t n, double lo, double hi, void *stream);
/* glibc's double pow elementwise, as NumPy's float64 scalar `**` runs it
 * (the device restatement the float64 SUPG tau uses): out[i] = x[i] ** y. */
int cfd_numpy_pow_f64(const double *x, double y, double *out, size_t n, void *stream);
/* max(|a|, |b|) (b may be NULL) into a zeroed device double */
int cfd_absmax2_f64(const double *a, const double *b, size_t n, double *out, void *stream);
int cfd_energy_mean2d_f64(const double *u, const double *v, size_t n, double *out, void *stream);
int cfd_apply_bc_ibm2d_f64(double *u, double *v, const double *y, int ny, int nx, double y_max,
                           double v_inf, int step, const double *ibm_mask, double force_strength,
                           void *stream);
int cfd_energy_mean_clip2d_f64(double *u, double *v, size_t n, double *out, double lo, double hi,
                               void *stream);
/* compute_vorticity into w (may be NULL) and/or nanmax|w| into a zeroed
 * device double absmax (may be NULL) */
int cfd_vorticity2d_f64(const double *u, const double *v, const uint8_t *mask, double *w,
                        double *absmax, int ny, int nx, double dx, double dy, void *stream);
int cfd_nonfinite_count_f64(const double *a, const double *b, size_t n, int *out, void *stream);
/* solve_pressure_gauss_seidel_fast (v5.py:202-226) on float64 fields: in-place
 * colour passes (two launches per iteration), the device-side stop rule, ws
 * of cfd_rbgs_workspace_bytes(iterations), *iters_done as in cfd_rbgs2d_f32. */
int cfd_rbgs2d_f64(double *phi, const double *div, const uint8_t *mask, int ny, int nx, double dx,
                   double dy, float dt, int iterations, double tolerance, void *ws, int *iters_done,
                   void *stream);

/* ------------------------------------------------- multi-GPU slab Jacobi */
/* One process per GPU.  The global (nz, ny, nx) grid is split on z; rank r
 * holds nz_local owned planes plus `ghost` (1..4) ghost planes on each side:
 * local array (nz_local + 2*ghost, ny, nx), owned planes ghost ..
 * ghost+nz_local-1.  After each pass the ghost planes are refilled from the
 * z-neighbours over xGMI by one of two transports (a `comm` is either):
 *  - copy engines (cfd_comm_init_ipc, the default of the Python side): each
 *    rank maps its neighbours' field buffers through IPC handles and the SDMA
 *    engines write its boundary planes straight into their ghost planes; no CU
 *    is used, so the interior launch keeps the whole chip;
 *  - RCCL send/recv (cfd_comm_init), whose kernel runs on a reserved set of
 *    CUs beside the interior (CFD_SLAB_COMM_CUS). */
int cfd_comm_unique_id(void *out, size_t bytes); /* bytes >= 128 */
int cfd_comm_init(const void *unique_id, int nranks, int rank, void **comm);
/* Copy-engine comm of rank `rank` of nranks (<= 16), no RCCL.  Before a solve
 * every rank attaches its two field buffers: cfd_comm_ipc_export(phi,
 * phi_tmp, n elements each) fills a host blob of cfd_comm_ipc_blob_bytes()
 * bytes; the caller gathers all ranks' blobs (any out-of-band channel, e.g.
 * torch.distributed all_gather_object) and passes them in rank order to
 * cfd_comm_ipc_import, which maps the neighbours' buffers and every rank's
 * flag block.  The slab solves then take exactly those buffers (phi / phi_tmp
 * in either order) and ignore comm_stream (the comm owns one copy stream per
 * direction).  A one-rank comm may name itself as both neighbours: the
 * per-rank rehearsal of scripts/slab_rehearsal.py (its result is not a
 * solve).  Waits for a neighbour are bounded (20 s): cfd_comm_status
 * synchronises the device and returns CFD_E_COMM (timeouts = 1) if one
 * expired, i.e. a rank stopped or the ranks ran different solves. */
int cfd_comm_init_ipc(int nranks, int rank, void **comm);
size_t cfd_comm_ipc_blob_bytes(void);
int cfd_comm_ipc_export(void *comm, const float *phi, const float *phi_tmp, size_t n, void *blob);
/* The same with the pair's ghost size: ghost_elems = ghost planes per side x
 * ny x nx.  A pair whose allocation is 2 GiB or more is never mapped by the
 * peers (hipIpcOpenMemHandle does not return past 2 GiB here, r06): its rank
 * exports a landing buffer of 4 x ghost_elems floats instead, the neighbours'
 * copies land there and the rank's compute stream copies them into the ghost
 * planes after each sync (same bits; CFD_CE_LANDING=1 forces it at any size).
 * cfd_comm_ipc_export (ghost_elems = 0) refuses such a pair. */
int cfd_comm_ipc_export_ghost(void *comm, const float *phi, const float *phi_tmp, size_t n,
                              size_t ghost_elems, void *blob);
int cfd_comm_ipc_import(void *comm, const void *blobs, int nblobs);
int cfd_comm_status(void *comm, int *timeouts);
int cfd_comm_destroy(void *comm);
/* An in-process group of nranks (<= 16) communicators for ONE process driving
 * the ranks from nranks host threads on one GPU (RCCL refuses several ranks per
 * device): the slab drivers below run unchanged, with each send/recv pair
 * replaced by a device copy ordered by HIP events and host barriers, and the
 * max-allreduce by a kernel over all ranks' maxima.  For tests and
 * rehearsals; comms[r] is released with cfd_comm_destroy. */
int cfd_comm_init_local(int nranks, void **comms);
/* Exchange plan, computed and tested on the host (SlabPlan in the package):
 * ghost = ghost planes per side, 1..4: a pass runs min(ghost, levels) sweeps
 * (cfd_set_jacobi3d_blocking), so ghost >= 2 enables the blocked kernels:
 * local array (nz_local + 2*ghost, ny, nx), owned planes ghost ..
 * ghost+nz_local-1.  lo_peer / hi_peer: neighbour ranks or -1.
 * z_update_begin/end: local indices of the owned planes that are updated
 * (global Dirichlet planes excluded).  After each pass the `ghost` owned
 * planes next to a neighbour go into its ghost planes.  rhs_ws: optional
 * same-size workspace (see cfd_jacobi2d_f32).  overlap != 0: the boundary
 * planes are computed first, their exchange runs beside the interior (RCCL:
 * on comm_stream; copy engines: on the comm's own copy streams) while the
 * interior computes on `stream`.  A one-rank comm may name itself (rank 0) as
 * lo_peer and hi_peer: the exchange is then a copy to itself, a timing
 * rehearsal of a middle rank's pass sequence on one GPU; its result is not a
 * solve. */
int cfd_slab_jacobi3d_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                          float *rhs_ws, const uint8_t *mask, int nz_local, int ghost, int ny,
                          int nx, int lo_peer, int hi_peer, int z_update_begin, int z_update_end,
                          double h, float dt, int iters, int overlap, void *stream,
                          void *comm_stream);
/* cfd_slab_jacobi3d_f32 from phi = zeros (v5.py:337; no mask): every rank's
 * phi (ghosts included) is taken as zeros and never read, so there is no
 * fill and no initial ghost exchange; with rhs_ws the first pass of each plane
 * range forms the RHS workspace itself and the last pass lands in phi. */
int cfd_slab_jacobi3d_zero_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                               float *rhs_ws, int nz_local, int ghost, int ny, int nx, int lo_peer,
                               int hi_peer, int z_update_begin, int z_update_end, double h, float dt,
                               int iters, int overlap, void *stream, void *comm_stream);
/* CU partition of an overlapped slab solve (CFD_SLAB_COMM_CUS = reserve,
 * default 16, 0 = off): the drivers run their launches on a stream masked to
 * compute_mask and the RCCL exchange on one masked to exchange_mask, so the
 * exchange kernel finds free CUs beside the one-workgroup-per-CU interior.
 * reserve / 8 CUs per XCD (bits b with b / (ncu/8) == x and b % 8 == x for
 * each XCD x, so the split holds for XCD-major and interleaved bit orders).
 * ncu % 64 == 0, reserve = 8k <= ncu / 8; words >= ceil(ncu / 32).  Host
 * only (no GPU call). */
int cfd_slab_cu_partition(int ncu, int reserve, uint32_t *compute_mask, uint32_t *exchange_mask,
                          int words);
/* Single-sweep building block (also used by the slab tests on one GPU):
 * update planes [z_begin, z_end) of in -> out (local array of nz planes);
 * x/y faces copied through, masked cells -> 0.  resid (optional, device float,
 * zeroed by caller) receives max|out - in|. */
int cfd_jacobi3d_sweep_f32(const float *in, float *out, const float *div, const uint8_t *mask,
                           int nz, int ny, int nx, int z_begin, int z_end, double h, float dt,
                           float *resid, void *stream);
/* Distributed red-black GS (config 5), same plan arguments as
 * cfd_slab_jacobi3d_f32 plus z_global_offset = global index of local plane 0
 * (SlabPlan.z_lo - ghost): colours are global, so the result is bit-identical
 * to cfd_rbgs3d_f32 on the whole grid.  ghost >= 2 + no mask + phi_tmp: fused
 * out-of-place passes, one iteration each, or two with ghost 4 (the default
 * at ghost 4; cfd_set_jacobi3d_blocking(2 or 3, ...) keeps one): boundary
 * planes first, their exchange overlapped with the interior when overlap != 0;
 * otherwise in-place colour passes with a ghost exchange after each colour.
 * The stop rule uses the global max|change| of each iteration (RCCL:
 * ncclAllReduce(max); copy engines: the sync kernel's gather over every
 * rank's flag block; none when tolerance <= 0).  ws / iters_done as in
 * cfd_rbgs3d_f32. */
int cfd_slab_rbgs3d_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                        const uint8_t *mask, int nz_local, int ghost, int ny, int nx, int lo_peer,
                        int hi_peer, int z_update_begin, int z_update_end, int z_global_offset,
                        double dx, double dy, double dz, float dt, int iterations,
                        double tolerance, void *ws, int *iters_done, int overlap, void *stream,
                        void *comm_stream);
/* Fused RB-GS building block (slab tests on one GPU): iteration `iteration`
 * of planes [z_begin, z_end) of in -> out (both colours; local plane 0 =
 * global plane z_global_offset).  fixed_lo/hi: plane z_begin-1 / z_end is a
 * Dirichlet plane (else it is recomputed from the plane beyond it).  Skipped
 * when ws's max|change| of iteration-1 < tolerance.  nx % 4 == 0, 16-byte
 * aligned.  ws is prepared by cfd_rbgs_init and read out by cfd_rbgs_finish:
 * iterations done = 1 + the first iteration whose max|change| < tolerance
 * (else all), into *iters_done; phi <- phi_tmp when that count is odd
 * (phi_tmp may be NULL for in-place solves; n = elements). */
int cfd_rbgs3d_pass_f32(const float *in, float *out, const float *div, int nz, int ny, int nx,
                        int z_begin, int z_end, int fixed_lo, int fixed_hi, int z_global_offset,
                        double dx, double dy, double dz, float dt, double tolerance, int iteration,
                        void *ws, void *stream);
int cfd_rbgs_init(void *ws, int iterations, double tolerance, int *iters_done, void *stream);
int cfd_rbgs_finish(void *ws, float *phi, const float *phi_tmp, size_t n, int *iters_done,
                    void *stream);

/* ------------------------------------------------------------- tuning */
/* The tuning knobs below are PER HOST THREAD: a cfd_set_* call changes the
 * kernels of the solves the calling thread launches, never another thread's.
 * Every thread starts from the process defaults (auto shapes; the CFD_*
 * environment knobs, read once).  cfd_reset_tuning() returns the calling
 * thread to those defaults. */
int cfd_reset_tuning(void);
/* Small-grid 2-D kernels (the v5 cylinder, 600 x 180): Jacobi sweeps per
 * launch j2_k (1..8), output rows per wave j2_rw (1, 2), cells per lane j2_vec
 * (1, or 4 = 16 bytes); red-black GS rows per wave gs_rw (1, 2), cells per lane
 * gs_vec (1, 4), waves per workgroup gs_wpb (4, 16).  0 = the default. */
int cfd_set_small2d_shape(int j2_k, int j2_rw, int j2_vec, int gs_rw, int gs_vec, int gs_wpb);
/* Small-grid red-black GS: iterations (colour-pair levels) fused per launch,
 * 1..5 (0 = the default, 5); a stop inside a launch is rolled back on the
 * device.  The persistent solve takes the most up to this whose tiles all fit
 * on the chip; the launch-per-block path at most 4.
 * shared_rows: 1 = each wave recomputes its halo rows (rbgs2d_small), 2 = the
 * rows of a 16-wave workgroup are shared through LDS (rbgs2d_wg), 0 = default. */
int cfd_set_small2d_gs_iters(int iters_per_launch, int shared_rows);
/* Small-grid GS as one persistent launch (cfd_rbgs2d_f32_ws with a workspace
 * of cfd_rbgs2d_workspace_bytes): 0 = default (on), 1 = off (one launch per
 * block of iterations), 2 = on (one LDS exchange per iteration inside a
 * tile), 3 = on with one exchange per colour level.  Its blocks are the
 * shared-row tile's (iterations per block as cfd_set_small2d_gs_iters). */
int cfd_set_small2d_gs_persistent(int mode);
/* Small-grid float32 Jacobi (cfd_jacobi2d_f32 on a grid the launch-per-pass
 * kernel would take, more sweeps than one block) as one persistent launch:
 * on = 0 default (on), 1 off, 2 on (two sweeps per LDS exchange inside a
 * tile), 3 on with one exchange per sweep; sweeps_per_block 0 = default (10),
 * or 4, 6, 8, 10: the most sweeps per block, up to this, whose tiles all fit
 * on the chip at once.  Its exchange ring lives in a library-owned device
 * buffer. */
int cfd_set_small2d_jacobi_persistent(int on, int sweeps_per_block);
/* Both persistent small-grid solves (the GS above and the Jacobi below) are
 * plain launches after the library's own occupancy check by default
 * (cooperative = 0, r05).  The check assumes no other persistent solve holds
 * CUs, so the library orders a process's persistent launches on a device one
 * after another (each waits on the device for the previous one, whatever its
 * stream or host thread).  Processes sharing a device are not ordered: there,
 * cooperative = 1 makes the HIP runtime guarantee that every tile is resident
 * at once or refuse the launch (a refused launch takes the launch-per-pass
 * path, same bits); it costs ~30 us of queue gap per solve (v5 cylinder step
 * 0.76 -> 0.79 ms).  poll_ticks bounds each wait of a tile for its
 * neighbours, in ticks of the 100 MHz device clock (0 = the default, 20 s; a
 * tiny value forces the failure path in tests).  A solve whose wait expired
 * leaves phi all NaN, the GS's *iters_done = -1, and counts one failure in the
 * failure word of the stream it ran on. */
int cfd_set_persistent_launch(int cooperative, long long poll_ticks);
/* The health check of one stream (the Python solver's
 * monitor_simulation_health, v5.py:599-613): returns in *expired the number
 * of persistent solves run on `stream` (the current device) whose neighbour
 * wait expired since the last read, and clears that count.  An async copy on
 * `stream` followed by a synchronisation of that stream only: other streams
 * keep running, and other streams' failures stay for their own readers. */
int cfd_persistent_status_stream(void *stream, int *expired);
/* The device-wide form: synchronises the current device, then sums and clears
 * the failure counts of every stream on it. */
int cfd_persistent_status(int *expired);
/* Frees the calling thread's library-owned device resources: the persistent
 * Jacobi's exchange rings (24 B per cell of the largest grid the thread
 * solved, one per device) and the timing events, after the work that uses them
 * has finished.  Later calls on the thread allocate them again.  The library
 * makes no HIP call at thread or process exit. */
int cfd_release_thread_resources(void);
/* Diagnostics: the persistent GS writes 4 timestamps (100 MHz device clock)
 * per tile and block into buf -- block start, halo received, tile ready,
 * levels done; layout [block][tile][4] u64 -- when bytes covers the solve
 * (NULL: off, the default).  The persistent Jacobi (r06) writes block start,
 * halo received, levels done, published into the same buffer. */
int cfd_set_small2d_gs_trace(void *buf, size_t bytes);
/* Diagnostics, in a library built with -DCFD_TBR_TRACE (scripts/build_variant.sh;
 * a no-op otherwise): the 3-D tall-tile kernels' workgroup 0 records, per wave,
 * the shader clock at 5 points (step entry, before / after each of the step's
 * two barriers) of z-steps 200..263 into buf, layout [wave][64][5] u64 (40 KiB,
 * 16 waves; NULL: off, the default). */
int cfd_set_tbr_trace(void *buf, size_t bytes);
/* Select the 3-D Jacobi kernel variant (bench / tile sweep):
 * variant 0 = auto, 1 = LDS plane tile, 2 = cache (no LDS); waves = rows per
 * workgroup (1..16); zchunk = planes per workgroup (0 = auto). */
int cfd_set_jacobi3d_config(int variant, int waves, int zchunk);
/* Temporal blocking of the 3-D Jacobi solve (cfd_jacobi3d_f32 without mask
 * or residual): steps = sweeps fused per HBM pass (0 = auto: 4 since r03,
 * 1 = off, 2..4; a remainder of iters % steps runs as a shorter pass, or,
 * from zeros, as the fused first pass); rows = output rows
 * per tile of the 2-sweep kernel (0 auto, 5, 13); zchunk = planes per tile.
 * Fused or not, results are bit-identical.  The red-black GS solves run
 * fused out-of-place passes whenever blocking is not off: steps = their
 * half-sweeps per pass on one GPU (auto 4, see cfd_get_rbgs3d_levels). */
int cfd_set_jacobi3d_blocking(int steps, int rows, int zchunk);
/* Jacobi sweeps per blocked pass currently in effect (2..4). */
int cfd_get_jacobi3d_levels(void);
/* Red-black GS half-sweeps (colour levels) per fused pass of a single-GPU
 * cfd_rbgs3d_f32 solve currently in effect (2..4; auto 4 = two iterations). */
int cfd_get_rbgs3d_levels(void);
/* Prefetch distance of the blocked kernel in planes (0 = auto = 1, 1, 2). */
int cfd_set_jacobi3d_prefetch(int planes);

/* The tile shape of the calling thread's last tall-tile launch (the fused
 * Jacobi / red-black GS passes, jacobi3d_tbr): levels per pass, row waves,
 * rows per row wave (output rows = waves * rows + 2 - 2 * levels) and planes
 * per z-chunk; zeros before the first.  For tests that pin a shape. */
int cfd_get_last_tbr_shape(int *levels, int *row_waves, int *rows_per_wave, int *zchunk);

/* Sweep timing (bench harness): while enabled, every solve records a HIP
 * event pair on its stream around its sweep launches.  cfd_timing_read
 * synchronises on those events and returns the summed elapsed milliseconds
 * and the number of sweeps (Jacobi iterations, or GS colour passes) they
 * cover.  Not for use under graph capture. */
int cfd_timing_enable(int enable);
int cfd_timing_read(double *ms, long long *sweeps, int reset);
/* The same for one channel: 0 = the pressure solves (cfd_timing_read), 1 =
 * the predictor launches (cfd_predictor2d_f32 / _f64, one count per launch),
 * so a timed time_step reports the solve's sweeps without the predictor in
 * them.  reset clears the channel read (the other channel's timings stay). */
int cfd_timing_read_channel(int channel, double *ms, long long *sweeps, int reset);

#ifdef __cplusplus
}
#endif
#endif /* CFDSIM_H */
