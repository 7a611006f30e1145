// fields2d_f64.hip -- the time_step() kernels with float64 fields
// (memory_efficient=False, v5.py:287-296): every field array is float64 and
// the dtype-generic @njit kernels (v5.py:96-257) run in float64.
//
// Arithmetic, as the reference executes it under NumPy 2 (NEP 50): Python
// float constants stay float64 against float64 data (no rounding to float32,
// unlike fields2d.hip).  The step's dt is np.float32 (adaptive_time_step) or
// the Python float dt_base (adaptive_dt=False, v5.py:317-318); either way it
// meets the float64 fields exactly, so the entry points take it as a double
// (tau = dt / 2, v5.py:161, is then exact in both precisions).  The GS's
// dt_inv = 1.0 / cfg.dt is a float32 quotient (cfg.dt is np.float32, v5.py:210).
// Source operation order, nothing fused (-ffp-contract=off).
//
// The SUPG tau's |V| = (u**2 + v**2) ** 0.5 on float64 scalars goes through
// glibc's pow in the reference, which is not correctly rounded (on ~1e-3 of
// random inputs pow(x, 2) != x*x and pow(x, 0.5) != sqrt(x)); it runs here as
// the device restatement of that pow (libm_pow.hpp), so the float64 step is
// bit-exact against the reference's own steps like the float32 one.
//
// These are one-pass-per-cell kernels (the float64 path is the reference's
// secondary configuration: every reference script sets memory_efficient=True,
// v5.py:633); the red-black GS runs as in-place colour passes, two launches
// per iteration, with the device-side stop rule of the float32 path.
#include "common.hpp"
#include "internal.hpp"
#include "libm_pow.hpp"
#include "pred_rows.hpp"

namespace cfd {
namespace {

struct Pred64 {
    double c1x, c1y;  // SUPG first derivative: 0.5 * (0.5/dx)   (v5.py:131,137)
    double c2x, c2y;  // SUPG second derivative: (0.5/dx)^2       (v5.py:141)
    double ux, uy;    // upwind: 1/dx                              (v5.py:116)
    double lx, ly;    // laplacian: 1/(dx*dx)                      (v5.py:168)
    double h;         // min(dx, dy)                               (v5.py:156)
};

Pred64 make_pred64(double dx, double dy) {
    Pred64 k;
    const double sdx = 0.5 / dx, sdy = 0.5 / dy;
    k.c1x = 0.5 * sdx;
    k.c1y = 0.5 * sdy;
    k.c2x = sdx * sdx;
    k.c2y = sdy * sdy;
    k.ux = 1.0 / dx;
    k.uy = 1.0 / dy;
    k.lx = 1.0 / (dx * dx);
    k.ly = 1.0 / (dy * dy);
    k.h = dx < dy ? dx : dy;
    return k;
}

__device__ inline bool interior64(int i, int j, int ny, int nx) {
    return i >= 1 && i < ny - 1 && j >= 1 && j < nx - 1;
}

// compute_supg_stabilization_fast body, v5.py:155-161 (|V| through glibc's
// pow, see the file comment); tau = dt / 2 (exact: dt is float32 or a double)
__device__ inline double supg_tau64(double u, double v, double nu, double dt, const Pred64 &k) {
    const double vm = libm::pow(libm::pow(u, 2.0) + libm::pow(v, 2.0), 0.5);
    if (vm > 1e-10) {
        const double pe = (vm * k.h) / (nu + 1e-10);
        const double half = pe / 2.0;
        const double lim = half < 1.0 ? half : 1.0;  // Python min(1.0, Pe/2.0)
        return (k.h / (2.0 * vm)) * lim;
    }
    return dt / 2.0;
}

// compute_convection_supg_fast body, v5.py:135-146
__device__ inline double conv_supg64(double uc, double vc, double C, double E, double W, double N,
                                     double S, double t, const Pred64 &k) {
    const double ddx = (E - W) * k.c1x;
    const double ddy = (N - S) * k.c1y;
    const double cs = uc * ddx + vc * ddy;
    if (t > 0.0) {
        const double d2x = ((E - 2.0 * C) + W) * k.c2x;
        const double d2y = ((N - 2.0 * C) + S) * k.c2y;
        return cs - t * (uc * d2x + vc * d2y);
    }
    return cs;
}

// compute_convection_fast body (first-order upwind), v5.py:120-124
__device__ inline double conv_upwind64(double uc, double vc, double C, double E, double W, double N,
                                       double S, const Pred64 &k) {
    const double ddx = uc > 0.0 ? (C - W) * k.ux : (E - C) * k.ux;
    const double ddy = vc > 0.0 ? (C - S) * k.uy : (N - C) * k.uy;
    return uc * ddx + vc * ddy;
}

// compute_laplacian_fast body, v5.py:172-175
__device__ inline double laplacian64(double nu, double C, double E, double W, double N, double S,
                                     const Pred64 &k) {
    const double l1 = ((E - 2.0 * C) + W) * k.lx;
    const double l2 = ((N - 2.0 * C) + S) * k.ly;
    return nu * (l1 + l2);
}

#define CFD_2D_INDEX64                                   \
    const int j = blockIdx.x * blockDim.x + threadIdx.x; \
    const int i = blockIdx.y;                            \
    if (j >= nx) return;                                 \
    const size_t c = (size_t)i * nx + j;

// kernel: 0 tau, 1 SUPG convection, 2 upwind convection, 3 laplacian
__global__ void k_component64(int kind, const double *__restrict__ u, const double *__restrict__ v,
                              const double *__restrict__ f, const double *__restrict__ aux, double nu_s,
                              double *__restrict__ out, int ny, int nx, double dt, Pred64 k) {
    CFD_2D_INDEX64
    double r = 0.0;  // np.zeros_like boundary ring
    if (interior64(i, j, ny, nx)) {
        if (kind == 0) r = supg_tau64(u[c], v[c], aux ? aux[c] : nu_s, dt, k);
        if (kind == 1) r = conv_supg64(u[c], v[c], f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], aux[c], k);
        if (kind == 2) r = conv_upwind64(u[c], v[c], f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], k);
        if (kind == 3) r = laplacian64(aux ? aux[c] : nu_s, f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], k);
    }
    out[c] = r;
}

// Fused predictor, v5.py:388-403: u* = u + dt*(-conv_u + lap_u), likewise v
template <bool SUPG>
__global__ __launch_bounds__(256) void k_predictor64(const double *__restrict__ u, const double *__restrict__ v,
                                                     const double *__restrict__ nu_eff, double nu_s,
                                                     double *__restrict__ us, double *__restrict__ vs,
                                                     double *__restrict__ tau_out, int ny, int nx, double dt,
                                                     Pred64 k) {
    CFD_2D_INDEX64
    const double uc = u[c], vc = v[c];
    double cu = 0.0, cv = 0.0, lu = 0.0, lv = 0.0, t = 0.0;
    if (interior64(i, j, ny, nx)) {
        const double nu = nu_eff ? nu_eff[c] : nu_s;
        const double uE = u[c + 1], uW = u[c - 1], uN = u[c + nx], uS = u[c - nx];
        const double vE = v[c + 1], vW = v[c - 1], vN = v[c + nx], vS = v[c - nx];
        if (SUPG) {
            t = supg_tau64(uc, vc, nu, dt, k);
            cu = conv_supg64(uc, vc, uc, uE, uW, uN, uS, t, k);
            cv = conv_supg64(uc, vc, vc, vE, vW, vN, vS, t, k);
        } else {
            cu = conv_upwind64(uc, vc, uc, uE, uW, uN, uS, k);
            cv = conv_upwind64(uc, vc, vc, vE, vW, vN, vS, k);
        }
        lu = laplacian64(nu, uc, uE, uW, uN, uS, k);
        lv = laplacian64(nu, vc, vE, vW, vN, vS, k);
    }
    us[c] = uc + dt * (-cu + lu);
    vs[c] = vc + dt * (-cv + lv);
    if (tau_out) tau_out[c] = t;  // 0 without SUPG (v5.py:292: never assigned without SUPG)
}

// compute_divergence_fast, v5.py:178-187 (+ max|div|, v5.py:410)
__global__ __launch_bounds__(256) void k_divergence64(const double *__restrict__ u, const double *__restrict__ v,
                                                      double *__restrict__ div, int ny, int nx, double cx,
                                                      double cy, double *absmax) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    double m = 0.0;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        double d = 0.0;
        if (interior64(i, j, ny, nx)) d = (u[c + 1] - u[c - 1]) * cx + (v[c + nx] - v[c - nx]) * cy;
        div[c] = d;
        const double a = fabs(d);
        if (a > m) m = a;
    }
    if (absmax) wave_reduce_max_store(m, absmax);
}

// compute_gradient_fast, v5.py:189-200
__global__ void k_gradient64(const double *__restrict__ phi, double *__restrict__ gx, double *__restrict__ gy,
                             int ny, int nx, double cx, double cy) {
    CFD_2D_INDEX64
    double a = 0.0, b = 0.0;
    if (interior64(i, j, ny, nx)) {
        a = (phi[c + 1] - phi[c - 1]) * cx;
        b = (phi[c + nx] - phi[c - nx]) * cy;
    }
    gx[c] = a;
    gy[c] = b;
}

// v5.py:413-417 (+ max sqrt(dpdx^2 + dpdy^2), v5.py:414-415)
__global__ __launch_bounds__(256) void k_project64(const double *__restrict__ phi, const double *__restrict__ us,
                                                   const double *__restrict__ vs, double *__restrict__ u,
                                                   double *__restrict__ v, int ny, int nx, double cx, double cy,
                                                   double dt, double *gradmax) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    double m = 0.0;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        double a = 0.0, b = 0.0;
        if (interior64(i, j, ny, nx)) {
            a = (phi[c + 1] - phi[c - 1]) * cx;
            b = (phi[c + nx] - phi[c - nx]) * cy;
        }
        u[c] = us[c] - dt * a;
        v[c] = vs[c] - dt * b;
        if (gradmax) {
            const double g = sqrt(a * a + b * b);
            if (g > m) m = g;
        }
    }
    if (gradmax) wave_reduce_max_store(m, gradmax);
}

// clean_divergence_fast's phi sweep (v5.py:250-253) in the serial
// lexicographic order (the semantics the float32 path defines; under prange
// the reference races): one workgroup walks anti-diagonals, thread t owns row
// b0 + t of a band and updates column st - t + 1 at step st; W is its own
// last output, S thread t-1's output one step earlier (LDS, by step parity),
// E / N / div are old values read from memory.
__global__ __launch_bounds__(1024) void k_lex_gs_sweep64(double *__restrict__ phi, const double *__restrict__ div,
                                                         int ny, int nx, double cx, double cy, double cd) {
    __shared__ double outb[2][1024];
    const int t = threadIdx.x, nt = blockDim.x;
    const int imax = ny - 2, jmax = nx - 2;
    for (int b0 = 1; b0 <= imax; b0 += nt) {
        __threadfence();  // the previous band's rows are final and visible
        __syncthreads();
        const int nrows = min(nt, imax - b0 + 1);
        const int i = b0 + t;
        const bool rowok = t < nrows;
        const size_t rowc = (size_t)(rowok ? i : 0) * nx;
        double w = rowok ? phi[rowc] : 0.0;  // phi(i, 0): W of column 1
        const int nsteps = nrows - 1 + jmax;
        for (int st = 0; st < nsteps; ++st) {
            const int j = st - t + 1;
            if (rowok && j >= 1 && j <= jmax) {
                const double E = phi[rowc + j + 1];
                const double N = phi[rowc + j + nx];  // old (row i+1 is behind)
                const double S = t == 0 ? phi[rowc + j - nx] : outb[(st + 1) & 1][t - 1];
                const double a = cx * (E + w);
                const double b = cy * (N + S);
                const double val = ((a + b) - div[rowc + j]) * cd;
                phi[rowc + j] = val;
                w = val;
                outb[st & 1][t] = val;
            }
            __syncthreads();
        }
    }
}

// u[1:-1,1:-1] -= grad_x[1:-1,1:-1] (no dt: v5.py:255-256)
__global__ void k_sub_gradient64(const double *__restrict__ phi, double *__restrict__ u, double *__restrict__ v,
                                 int ny, int nx, double cx, double cy) {
    CFD_2D_INDEX64
    if (!interior64(i, j, ny, nx)) return;
    const double a = (phi[c + 1] - phi[c - 1]) * cx;
    const double b = (phi[c + nx] - phi[c - nx]) * cy;
    u[c] = u[c] - a;
    v[c] = v[c] - b;
}

// apply_boundary_conditions, v5.py:349-360 (see k_bc in fields2d.hip; the
// inlet value stays float64 here)
__global__ void k_bc64(double *__restrict__ u, double *__restrict__ v, const double *__restrict__ y, int ny,
                       int nx, double y_max, double v_inf, int step) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nx) {
        u[t] = 0.0;
        v[t] = 0.0;
        u[(size_t)(ny - 1) * nx + t] = 0.0;
        v[(size_t)(ny - 1) * nx + t] = 0.0;
    }
    const int i = t;
    if (i >= 1 && i < ny - 1) {
        const double s = (double)step;
        double scale = s / 1000.0;
        scale = (1.0 < scale ? 1.0 : scale) * 0.01;
        const double two_pi = 2.0 * 3.141592653589793;
        const double pert = scale * sin(two_pi * y[i] / y_max + 0.02 * s);
        const size_t r = (size_t)i * nx;
        u[r] = v_inf * (1.0 + pert);
        v[r] = 0.0;
        u[r + nx - 1] = u[r + nx - 2];
        v[r + nx - 1] = v[r + nx - 2];
    }
}

// lid-driven cavity walls (fields2d.hip k_lid_bc)
__global__ void k_lid_bc64(double *__restrict__ u, double *__restrict__ v, int ny, int nx, double u_lid) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ny - 1) {
        const size_t r = (size_t)t * nx;
        u[r] = 0.0;
        v[r] = 0.0;
        u[r + nx - 1] = 0.0;
        v[r + nx - 1] = 0.0;
    }
    if (t < nx) {
        u[t] = 0.0;
        v[t] = 0.0;
        u[(size_t)(ny - 1) * nx + t] = u_lid;
        v[(size_t)(ny - 1) * nx + t] = 0.0;
    }
}

// apply_ibm_fast, v5.py:228-237
__global__ void k_ibm64(double *__restrict__ u, double *__restrict__ v, const double *__restrict__ m, int n,
                        double fs) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
        const double mv = m[c];
        if (mv > 0.0) {
            u[c] *= (1.0 - mv * fs);
            v[c] *= (1.0 - mv * fs);
        }
    }
}

__global__ void k_clip64(double *__restrict__ a, size_t n, double lo, double hi) {
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n; c += (size_t)gridDim.x * blockDim.x) {
        const double x = a[c];
        a[c] = x < lo ? lo : (x > hi ? hi : x);  // NaN passes through like np.clip
    }
}

__global__ void k_absmax64(const double *__restrict__ a, const double *__restrict__ b, size_t n, double *out) {
    double m = 0.0;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n; c += (size_t)gridDim.x * blockDim.x) {
        double x = fabs(a[c]);
        if (x > m) m = x;
        if (b) {
            x = fabs(b[c]);
            if (x > m) m = x;
        }
    }
    wave_reduce_max_store(m, out);
}

// sum of 0.5*(u^2 + v^2) (v5.py:362-363, :431-432), scaled by 1/n after
__global__ void k_energy_sum64(const double *__restrict__ u, const double *__restrict__ v, size_t n, double *out) {
    double s = 0.0;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n; c += (size_t)gridDim.x * blockDim.x)
        s += 0.5 * (u[c] * u[c] + v[c] * v[c]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

__global__ void k_scale64(double *p, double f) { *p = *p * f; }

// compute_vorticity (v5.py:365-373): w, or (out != NULL) nanmax|w| only
__global__ void k_vorticity64(const double *__restrict__ u, const double *__restrict__ v,
                              const uint8_t *__restrict__ mask, double *__restrict__ w, int ny, int nx,
                              double dx2, double dy2, double *absmax) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    double m = 0.0;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        double r = 0.0;
        if (interior64(i, j, ny, nx)) r = (v[c + 1] - v[c - 1]) / dx2 - (u[c + nx] - u[c - nx]) / dy2;
        const bool masked = mask && mask[c];
        if (w) w[c] = masked ? __builtin_nan("") : r;
        if (!masked && fabs(r) > m) m = fabs(r);
    }
    if (absmax) wave_reduce_max_store(m, absmax);
}

__global__ void k_nonfinite64(const double *__restrict__ a, const double *__restrict__ b, size_t n, int *out) {
    int cnt = 0;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n; c += (size_t)gridDim.x * blockDim.x) {
        cnt += !isfinite(a[c]);
        if (b) cnt += !isfinite(b[c]);
    }
    if (cnt) atomicAdd(out, cnt);
}

// ------------------------------------------------------ red-black GS, fp64
// Workspace (cfd_rbgs_workspace_bytes): int flags[4] (iterations, done,
// unused, unused), then double maxc[iterations] at byte 16.
struct RbgsWs64 {
    int flags[4];
    double maxc[1];
};

__global__ void k_rbgs64_init(RbgsWs64 *ws, int iterations, int *iters_done) {
    for (int k = threadIdx.x; k < iterations; k += blockDim.x) ws->maxc[k] = 0.0;
    if (threadIdx.x == 0) {
        ws->flags[0] = iterations;
        ws->flags[1] = iterations;
        ws->flags[2] = ws->flags[3] = 0;
        if (iters_done) *iters_done = iterations;
    }
}

// One colour of iteration `it`, in place, v5.py:211-222: colour c visits
// j = 1 + (i + c) % 2 step 2, masked cells skipped; max|change| into maxc[it].
// Skipped once an earlier iteration ended below tol (v5.py:224-225; maxc of
// skipped iterations stays 0 < tol, so the stop persists).
template <int C>
__global__ __launch_bounds__(256) void k_rbgs64_color(double *__restrict__ phi, const double *__restrict__ div,
                                                      const uint8_t *__restrict__ mask, int ny, int nx, double cx,
                                                      double cy, double cd, double dt_inv, double tol,
                                                      RbgsWs64 *ws, int it) {
    if (it > 0 && ws->maxc[it - 1] < tol) return;
    const int i = blockIdx.y + 1;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    double mx = 0.0;
    if (j >= 1 && j < nx - 1 && ((i + j + 1 + C) & 1) == 0) {
        const size_t c = (size_t)i * nx + j;
        if (!(mask && mask[c])) {
            const double rhs = -div[c] * dt_inv;
            const double pn = (cx * (phi[c + 1] + phi[c - 1]) + cy * (phi[c + nx] + phi[c - nx]) - rhs) * cd;
            const double ch = fabs(pn - phi[c]);
            if (ch > mx) mx = ch;
            phi[c] = pn;
        }
    }
    wave_reduce_max_store(mx, &ws->maxc[it]);
}

// iterations done = 1 + the first iteration whose max|change| < tol, else all
__global__ void k_rbgs64_count(RbgsWs64 *__restrict__ ws, double tol, int *iters_done) {
    const int n = ws->flags[0];
    int first = n;
    for (int base = 0; base < n; base += 64) {
        const int i = base + (int)threadIdx.x;
        const unsigned long long m = __ballot(i < n && ws->maxc[i] < tol);
        if (m) {
            first = base + __ffsll((long long)m) - 1;
            break;
        }
    }
    if (threadIdx.x == 0) {
        const int c = first < n ? first + 1 : n;
        ws->flags[1] = c;
        if (iters_done) *iters_done = c;
    }
}

dim3 grid2d64(int ny, int nx) { return dim3(ceil_div(nx, 256), ny); }
int grid1d64(size_t n) {
    long b = (long)((n + 255) / 256);
    if (b > 2048) b = 2048;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace
}  // namespace cfd

using namespace cfd;

#define CFD_SHAPE2D64(ny, nx) CFD_REQUIRE((ny) >= 1 && (nx) >= 1, "bad 2-D shape (%d, %d)", ny, nx)

// NumPy float64 scalar power (glibc pow, libm_pow.hpp) elementwise: the
// parity hook for the device pow the float64 SUPG tau uses.
__global__ void k_numpy_pow64(const double *__restrict__ x, double y, double *__restrict__ out, size_t n) {
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n; c += (size_t)gridDim.x * blockDim.x)
        out[c] = libm::pow(x[c], y);
}

extern "C" {

int cfd_supg_tau2d_f64(const double *u, const double *v, const double *nu_eff, double nu_eff_scalar, double *tau,
                       int ny, int nx, double dx, double dy, double dt, void *stream) {
    CFD_REQUIRE(u && v && tau, "supg_tau2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_component64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), 0, u, v,
                       (const double *)nullptr, nu_eff, nu_eff_scalar, tau, ny, nx, dt, make_pred64(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_convection_supg2d_f64(const double *u, const double *v, const double *phi, const double *tau,
                              double *conv, int ny, int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && phi && tau && conv, "convection_supg2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_component64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), 1, u, v, phi, tau, 0.0,
                       conv, ny, nx, 0.0, make_pred64(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_convection_upwind2d_f64(const double *u, const double *v, const double *phi, double *conv, int ny, int nx,
                                double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && phi && conv, "convection_upwind2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_component64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), 2, u, v, phi,
                       (const double *)nullptr, 0.0, conv, ny, nx, 0.0, make_pred64(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_laplacian2d_f64(const double *phi, const double *nu_eff, double nu_eff_scalar, double *lap, int ny, int nx,
                        double dx, double dy, void *stream) {
    CFD_REQUIRE(phi && lap, "laplacian2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_component64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), 3,
                       (const double *)nullptr, (const double *)nullptr, phi, nu_eff, nu_eff_scalar, lap, ny, nx,
                       0.0, make_pred64(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_predictor2d_f64(const double *u, const double *v, const double *nu_eff, double nu_eff_scalar,
                        double *u_star, double *v_star, double *tau, int ny, int nx, double dx, double dy, double dt,
                        int use_supg, void *stream) {
    CFD_REQUIRE(u && v && u_star && v_star, "predictor2d_f64: null pointer");
    CFD_REQUIRE(u_star != u && v_star != v && u_star != v && v_star != u,
                "predictor2d_f64: outputs must not alias inputs");
    CFD_SHAPE2D64(ny, nx);
    hipStream_t s = as_stream(stream);
    // the row march (pred_rows.hpp): cells per lane 2 (16 B) or 1, halved
    // until nx and every array's alignment allow it
    int vec = tuning().pred_vec == 1 ? 1 : 2;
    auto fits = [&](int w) {
        const uintptr_t m = (uintptr_t)(8 * w - 1);
        auto al = [&](const void *p_) { return !p_ || ((uintptr_t)p_ & m) == 0; };
        return nx % w == 0 && al(u) && al(v) && al(u_star) && al(v_star) && al(tau) && al(nu_eff);
    };
    while (vec > 1 && !fits(vec)) vec /= 2;
    const bool rows_ok = (size_t)ny * nx * sizeof(double) < ((size_t)1 << 31) && fits(vec);
    const int tau_mode = use_supg ? tuning().pred_tau : kTauExact;
    const int tk = timing_begin(s, kTimingPredictor);
    if (tuning().pred_variant != 1 && rows_ok) {
        PredRowArgs<double> a;
        a.u = u;
        a.v = v;
        a.nu = nu_eff;
        a.us = u_star;
        a.vs = v_star;
        a.tau = tau;  // zeros without SUPG
        a.nu_s = nu_eff_scalar;
        a.dt = dt;
        a.ny = ny;
        a.nx = nx;
        a.k = make_pred_k<double>(dx, dy);
        CFD_CHECK_HIP(pred_rows_launch<double>(a, use_supg != 0, tau_mode, vec, tuning().pred_rows, s));
        set_last_predictor(1, tau_mode, vec);
    } else {
        const Pred64 k = make_pred64(dx, dy);
        if (use_supg)
            hipLaunchKernelGGL(k_predictor64<true>, grid2d64(ny, nx), dim3(256), 0, s, u, v, nu_eff, nu_eff_scalar,
                               u_star, v_star, tau, ny, nx, dt, k);
        else
            hipLaunchKernelGGL(k_predictor64<false>, grid2d64(ny, nx), dim3(256), 0, s, u, v, nu_eff, nu_eff_scalar,
                               u_star, v_star, tau, ny, nx, dt, k);
        set_last_predictor(0, kTauExact, 1);
    }
    timing_end(tk, s, 1);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_divergence2d_f64(const double *u, const double *v, double *div, int ny, int nx, double dx, double dy,
                         double *absmax, void *stream) {
    CFD_REQUIRE(u && v && div, "divergence2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_divergence64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), u, v, div, ny, nx,
                       0.5 / dx, 0.5 / dy, absmax);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_gradient2d_f64(const double *phi, double *grad_x, double *grad_y, int ny, int nx, double dx, double dy,
                       void *stream) {
    CFD_REQUIRE(phi && grad_x && grad_y, "gradient2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_gradient64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), phi, grad_x, grad_y, ny,
                       nx, 0.5 / dx, 0.5 / dy);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_project2d_f64(const double *phi, const double *u_star, const double *v_star, double *u, double *v, int ny,
                      int nx, double dx, double dy, double dt, double *gradmax, void *stream) {
    CFD_REQUIRE(phi && u_star && v_star && u && v, "project2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_project64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), phi, u_star, v_star, u, v,
                       ny, nx, 0.5 / dx, 0.5 / dy, dt, gradmax);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_clean_divergence2d_f64(double *u, double *v, int ny, int nx, double dx, double dy, int iterations,
                               void *ws, void *stream) {
    CFD_REQUIRE(u && v && ws, "clean_divergence2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipStream_t s = as_stream(stream);
    const size_t n = (size_t)ny * nx;
    double *phi = reinterpret_cast<double *>(ws);
    double *div = phi + n;
    CFD_CHECK_HIP(hipMemsetAsync(phi, 0, n * sizeof(double), s));  // np.zeros_like (v5.py:242)
    const double dx2_inv = 1.0 / (dx * dx), dy2_inv = 1.0 / (dy * dy);
    const double denom_inv = 1.0 / (2.0 * (dx2_inv + dy2_inv));
    for (int it = 0; it < iterations; ++it) {
        hipLaunchKernelGGL(k_divergence64, grid2d64(ny, nx), dim3(256), 0, s, u, v, div, ny, nx, 0.5 / dx,
                           0.5 / dy, (double *)nullptr);
        if (ny > 2 && nx > 2)
            hipLaunchKernelGGL(k_lex_gs_sweep64, dim3(1), dim3(ny - 2 >= 1024 ? 1024 : 64 * ceil_div(ny - 2, 64)),
                               0, s, phi, div, ny, nx, dx2_inv, dy2_inv, denom_inv);
        hipLaunchKernelGGL(k_sub_gradient64, grid2d64(ny, nx), dim3(256), 0, s, phi, u, v, ny, nx, 0.5 / dx,
                           0.5 / dy);
        CFD_LAUNCH_CHECK();
    }
    return CFD_OK;
}

int cfd_apply_bc2d_f64(double *u, double *v, const double *y, int ny, int nx, double y_max, double v_inf,
                       int step, void *stream) {
    CFD_REQUIRE(u && v && y, "apply_bc2d_f64: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_bc2d_f64: grid must be at least 2x2");
    const int n = ny > nx ? ny : nx;
    hipLaunchKernelGGL(k_bc64, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), u, v, y, ny, nx, y_max,
                       v_inf, step);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_apply_lid_bc2d_f64(double *u, double *v, int ny, int nx, double u_lid, void *stream) {
    CFD_REQUIRE(u && v, "apply_lid_bc2d_f64: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_lid_bc2d_f64: grid must be at least 2x2");
    const int n = ny > nx ? ny : nx;
    hipLaunchKernelGGL(k_lid_bc64, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), u, v, ny, nx, u_lid);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_apply_ibm2d_f64(double *u, double *v, const double *ibm_mask, int n, double force_strength,
                        void *stream) {
    CFD_REQUIRE(u && v && ibm_mask && n >= 0, "apply_ibm2d_f64: bad arguments");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_ibm64, dim3(grid1d64(n)), dim3(256), 0, as_stream(stream), u, v, ibm_mask, n,
                       force_strength);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_numpy_pow_f64(const double *x, double y, double *out, size_t n, void *stream) {
    CFD_REQUIRE(x && out, "numpy_pow_f64: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_numpy_pow64, dim3(grid1d64(n)), dim3(256), 0, as_stream(stream), x, y, out, n);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_clip_f64(double *a, size_t n, double lo, double hi, void *stream) {
    CFD_REQUIRE(a, "clip_f64: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_clip64, dim3(grid1d64(n)), dim3(256), 0, as_stream(stream), a, n, lo, hi);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_absmax2_f64(const double *a, const double *b, size_t n, double *out, void *stream) {
    CFD_REQUIRE(a && out, "absmax2_f64: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_absmax64, dim3(grid1d64(n)), dim3(256), 0, as_stream(stream), a, b, n, out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_energy_mean2d_f64(const double *u, const double *v, size_t n, double *out, void *stream) {
    CFD_REQUIRE(u && v && out && n > 0, "energy_mean2d_f64: bad arguments");
    hipStream_t s = as_stream(stream);
    if (n <= kEnergyOneBlock) {
        if (unsigned *ws = energy_scratch(s))
            hipLaunchKernelGGL((k_energy_mean_mb<double, false>), dim3(kEnergyBlocks), dim3(256), 0, s,
                               const_cast<double *>(u), const_cast<double *>(v), n, out, double(0), double(0), ws);
        else
            hipLaunchKernelGGL((k_energy_mean_1blk<double, false>), dim3(1), dim3(1024), 0, s, const_cast<double *>(u),
                               const_cast<double *>(v), n, out, double(0), double(0));
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    CFD_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(double), s));
    hipLaunchKernelGGL(k_energy_sum64, dim3(grid1d64(n)), dim3(256), 0, s, u, v, n, out);
    hipLaunchKernelGGL(k_scale64, dim3(1), dim3(1), 0, s, out, 1.0 / (double)n);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_energy_mean_clip2d_f64(double *u, double *v, size_t n, double *out, double lo, double hi, void *stream) {
    CFD_REQUIRE(u && v && out && n > 0, "energy_mean_clip2d_f64: bad arguments");
    hipStream_t s = as_stream(stream);
    if (n <= kEnergyOneBlock) {
        if (unsigned *ws = energy_scratch(s))
            hipLaunchKernelGGL((k_energy_mean_mb<double, true>), dim3(kEnergyBlocks), dim3(256), 0, s, u, v, n, out,
                               lo, hi, ws);
        else
            hipLaunchKernelGGL((k_energy_mean_1blk<double, true>), dim3(1), dim3(1024), 0, s, u, v, n, out, lo, hi);
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    int rc = cfd_energy_mean2d_f64(u, v, n, out, stream);
    if (!rc) rc = cfd_clip_f64(u, n, lo, hi, stream);
    if (!rc) rc = cfd_clip_f64(v, n, lo, hi, stream);
    return rc;
}

int cfd_apply_bc_ibm2d_f64(double *u, double *v, const double *y, int ny, int nx, double y_max, double v_inf, int step,
                           const double *ibm_mask, double force_strength, void *stream) {
    CFD_REQUIRE(u && v && y, "apply_bc_ibm2d_f64: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_bc_ibm2d_f64: grid must be at least 2x2");
    int blocks = ceil_div(ny > nx ? ny : nx, 256);
    if (ibm_mask) {
        const int g = grid1d64((size_t)ny * nx);
        if (g > blocks) blocks = g;
    }
    hipLaunchKernelGGL(k_bc_ibm<double>, dim3(blocks), dim3(256), 0, as_stream(stream), u, v, y, ibm_mask, ny, nx,
                       y_max, v_inf, step, force_strength);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_vorticity2d_f64(const double *u, const double *v, const uint8_t *mask, double *w, double *absmax, int ny,
                        int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && (w || absmax), "vorticity2d_f64: null pointer");
    CFD_SHAPE2D64(ny, nx);
    hipLaunchKernelGGL(k_vorticity64, grid2d64(ny, nx), dim3(256), 0, as_stream(stream), u, v, mask, w, ny, nx,
                       2.0 * dx, 2.0 * dy, absmax);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_nonfinite_count_f64(const double *a, const double *b, size_t n, int *out, void *stream) {
    CFD_REQUIRE(a && out, "nonfinite_count_f64: null pointer");
    hipStream_t s = as_stream(stream);
    CFD_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(int), s));
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_nonfinite64, dim3(grid1d64(n)), dim3(256), 0, s, a, b, n, out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_rbgs2d_f64(double *phi, const double *div, const uint8_t *mask, int ny, int nx, double dx, double dy,
                   float dt, int iterations, double tolerance, void *ws, int *iters_done, void *stream) {
    CFD_REQUIRE(phi && div && ws, "rbgs2d_f64: null pointer");
    CFD_REQUIRE(ny >= 1 && nx >= 1 && iterations >= 0, "rbgs2d_f64: bad arguments");
    hipStream_t s = as_stream(stream);
    // v5.py:205-210: Python-float constants (float64 against float64 data);
    // dt_inv = 1.0 / np.float32(dt) is a float32 quotient
    const double dx2_inv = 1.0 / (dx * dx), dy2_inv = 1.0 / (dy * dy);
    const double denom_inv = 1.0 / (2.0 * (dx2_inv + dy2_inv));
    const double dt_inv = (double)(1.0f / dt);
    RbgsWs64 *w = reinterpret_cast<RbgsWs64 *>(ws);
    hipLaunchKernelGGL(k_rbgs64_init, dim3(1), dim3(1024), 0, s, w, iterations, iters_done);
    CFD_LAUNCH_CHECK();
    if (ny < 3 || nx < 3 || iterations == 0) return CFD_OK;
    const int tk = timing_begin(s);
    const dim3 grid(ceil_div(nx, 256), ny - 2);
    for (int it = 0; it < iterations; ++it) {
        hipLaunchKernelGGL(k_rbgs64_color<0>, grid, dim3(256), 0, s, phi, div, mask, ny, nx, dx2_inv, dy2_inv,
                           denom_inv, dt_inv, tolerance, w, it);
        hipLaunchKernelGGL(k_rbgs64_color<1>, grid, dim3(256), 0, s, phi, div, mask, ny, nx, dx2_inv, dy2_inv,
                           denom_inv, dt_inv, tolerance, w, it);
        CFD_LAUNCH_CHECK();
    }
    timing_end(tk, s, iterations);
    hipLaunchKernelGGL(k_rbgs64_count, dim3(1), dim3(64), 0, s, w, tolerance, iters_done);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // extern "C"
