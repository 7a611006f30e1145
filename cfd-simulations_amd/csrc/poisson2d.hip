// poisson2d.hip -- 2-D pressure-Poisson kernels for gfx950.
//
//  * Jacobi 5-point (f32 / f64): the reference's NumPy branch of
//    OptimizedTurbulentSolver.solve_pressure_fast, v5.py:336-346, bit-exact.
//  * Red-black Gauss-Seidel (f32): solve_pressure_gauss_seidel_fast,
//    v5.py:202-226, with the serial-execution arithmetic of the reference.
//
// Jacobi design (HBM-bound, 12 B per f32 cell-update / 24 B per f64):
//  one wave owns a 64*VEC-cell x-segment and marches down a chunk of rows,
//  holding rows y-1, y, y+1 in registers (a 3-row register queue, next row
//  prefetched one step ahead), so every phi value is fetched from HBM once per
//  sweep.  x-neighbours come from the adjacent lane through a cross-lane
//  shuffle; only lanes 0 and 63 load one extra scalar per row (L1/L2 hits).
//  Loads and stores are 16 B per lane (float4 / double2).  The RHS
//  (f32(dx^2)*div)/dt is recomputed in-register from div every sweep: the same
//  4 B of traffic as reading a precomputed rhs array, bit-identical to NumPy,
//  and no prologue pass or workspace.
#include "stencil2d.hpp"

namespace cfd {

// One Jacobi sweep over rows [1, ny-1).  Grid: waves = nseg * nchunk.
// PRE: `div` holds the precomputed rhs = (dx2*div)/dt (same bits as in-register)
template <typename T, int VEC, bool RESID, bool PRE>
__global__ __launch_bounds__(256) void jacobi2d_march(const T *__restrict__ in, T *__restrict__ out,
                                                      const T *__restrict__ div,
                                                      const uint8_t *__restrict__ mask, int ny,
                                                      int nx, int nseg, int rows_per_chunk,
                                                      T dx2, T dtv, T *__restrict__ resid) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wpb = blockDim.x / kWave;
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * wpb + threadIdx.x / kWave;
    const int seg = (int)(wave % nseg);
    const int chunk = (int)(wave / nseg);
    const int y0 = 1 + chunk * rows_per_chunk;
    if (y0 >= ny - 1) return;  // wave-uniform
    const int y1 = min(y0 + rows_per_chunk, ny - 1);
    const int x0 = (seg * kWave + lane) * VEC;
    const bool valid = x0 < nx;
    const bool has_left = valid && lane == 0 && x0 > 0;
    const bool has_right = lane == kWave - 1 && x0 + VEC < nx;

    T prv[VEC], cur[VEC], nxt[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) prv[k] = cur[k] = nxt[k] = T(0);
    T cl = T(0), cr = T(0), nl = T(0), nr = T(0);
    if (valid) {
        ld<T, VEC>(in + (size_t)(y0 - 1) * nx + x0, prv);
        ld<T, VEC>(in + (size_t)y0 * nx + x0, cur);
    }
    if (has_left) cl = in[(size_t)y0 * nx + x0 - 1];
    if (has_right) cr = in[(size_t)y0 * nx + x0 + VEC];
    T rmax = T(0);

    for (int y = y0; y < y1; ++y) {
        const size_t row = (size_t)y * nx;
        // prefetch row y+1 (always inside the grid: y <= ny-2)
        if (valid) ld<T, VEC>(in + row + nx + x0, nxt);
        if (has_left) nl = in[row + nx + x0 - 1];
        if (has_right) nr = in[row + nx + x0 + VEC];
        T d[VEC];
        uint8_t m[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) { d[k] = T(0); m[k] = 0; }
        if (valid) {
            ld<T, VEC>(div + row + x0, d);
            if (mask) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) m[k] = mask[row + x0 + k];
            }
        }
        // x-neighbours across lanes: W of element 0 from lane-1, E of the last from lane+1
        T wl = dpp_from_lower(cur[VEC - 1]);
        T er = dpp_from_upper(cur[0]);
        if (lane == 0) wl = cl;
        if (lane == kWave - 1) er = cr;
        T o[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const T E = (k + 1 < VEC) ? cur[k + 1] : er;
            const T W = (k > 0) ? cur[k - 1] : wl;
            const int x = x0 + k;
            T val;
            if (x == 0 || x >= nx - 1) {
                val = cur[k];  // Dirichlet edge: copied (phi_new = phi.copy())
            } else {
                // ((((E + W) + N) + S) - (dx2*div)/dt) * 0.25 -- NumPy's order
                T s = E + W;
                s = s + nxt[k];
                s = s + prv[k];
                const T rhs = PRE ? d[k] : (dx2 * d[k]) / dtv;
                val = T(0.25) * (s - rhs);
            }
            if (m[k]) val = T(0);
            o[k] = val;
            if constexpr (RESID) {
                T c = val - cur[k];
                c = c < T(0) ? -c : c;
                if (c > rmax) rmax = c;
            }
        }
        if (valid) st<T, VEC>(out + row + x0, o);
#pragma unroll
        for (int k = 0; k < VEC; ++k) { prv[k] = cur[k]; cur[k] = nxt[k]; }
        cl = nl;
        cr = nr;
    }
    if constexpr (RESID) wave_reduce_max_store(rmax, resid);
}

// Edge rows the sweep never writes: dst = mask ? 0 : src over [start, start+count).
// Before sweep 1 this builds the output buffer's edges from the input's
// (phi_new = phi.copy(); phi_new[mask] = 0, v5.py:339,345 -- sweep 1 itself
// still reads the unmasked input edges); after sweep 1 it copies them back
// so both ping-pong buffers hold the final edges.
template <typename T>
__global__ void fix_cells(const T *__restrict__ src, T *__restrict__ dst,
                          const uint8_t *__restrict__ mask, size_t start, size_t count) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < count;
         k += (size_t)gridDim.x * blockDim.x) {
        const size_t c = start + k;
        T v = src[c];
        if (mask && mask[c]) v = T(0);
        dst[c] = v;
    }
}
template <typename T>
static int launch_fix_cells(const T *src, T *dst, const uint8_t *mask, size_t start, size_t count,
                            hipStream_t s) {
    if (count == 0) return CFD_OK;
    int blocks = ceil_div((long)count, 256);
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(fix_cells<T>, dim3(blocks), dim3(256), 0, s, src, dst, mask, start, count);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// rows 0 and ny-1: dst = mask ? 0 : src
template <typename T>
static int fix_edge_rows(const T *src, T *dst, const uint8_t *mask, int ny, int nx, hipStream_t s) {
    int rc = launch_fix_cells<T>(src, dst, mask, 0, (size_t)nx, s);
    if (!rc && ny > 1) rc = launch_fix_cells<T>(src, dst, mask, (size_t)(ny - 1) * nx, (size_t)nx, s);
    return rc;
}

template <typename T, int VEC>
static int jacobi2d_sweep(const T *in, T *out, const T *div, const uint8_t *mask, int ny, int nx,
                          T dx2, T dtv, bool pre, T *resid, hipStream_t s) {
    const int nseg = ceil_div(nx, kWave * VEC);
    const int rows = ny - 2;
    if (rows <= 0) return CFD_OK;
    // ~8192 waves (32 per CU) when the grid allows; >= 4 rows per chunk.
    long target = 8192;
    int rpc = ceil_div((long)rows * nseg, target);
    if (rpc < 4) rpc = 4;
    if (rpc > 64) rpc = 64;
    const int nchunk = ceil_div(rows, rpc);
    const long waves = (long)nseg * nchunk;
    const int wpb = 4;
    const int blocks = ceil_div(waves, wpb);
#define CFD_J2(R, PR)                                                                             \
    hipLaunchKernelGGL((jacobi2d_march<T, VEC, R, PR>), dim3(blocks), dim3(wpb * kWave), 0, s, in, \
                       out, div, mask, ny, nx, nseg, rpc, dx2, dtv, resid)
    if (resid) {
        if (pre) CFD_J2(true, true); else CFD_J2(true, false);
    } else {
        if (pre) CFD_J2(false, true); else CFD_J2(false, false);
    }
#undef CFD_J2
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}



// K-level Jacobi for small grids (the v5 cylinder, config 1): each wave owns
// two output rows and loads every row it needs up front (level 0 rows
// y0-K .. y0+1+K, rhs / mask rows y0-(K-1) .. y0+K), so a pass of K sweeps is
// one load latency plus K levels of VALU -- the row march of jacobi2d_tbk is a
// chain of row-step latencies on a grid too small to hide them.  x-segments
// overlap by HL = ceil(K/VEC) halo lanes (erosion), as in jacobi2d_tbk; same
// operation order, fixed rows / columns and mask rule, bit-identical.
template <typename T, int VEC, int K, bool PRE, bool MASK, int RW = 2>
__global__ __launch_bounds__(256) void jacobi2d_small(const T *__restrict__ in, T *__restrict__ out,
                                                      const T *__restrict__ div,
                                                      const uint8_t *__restrict__ mask, int ny, int nx,
                                                      int nseg, T dx2, T dtv) {
    constexpr int HL = (K + VEC - 1) / VEC;
    constexpr int SOUT = (64 - 2 * HL) * VEC;
    constexpr int NR0 = RW + 2 * K;
    constexpr int ND = RW + 2 * K - 2;  // rows y0-(K-1) .. y0+RW-1+K-1
    const int lane = threadIdx.x & 63;
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * 4 + threadIdx.x / 64;
    const int seg = (int)(wave % nseg);
    const int y0 = 1 + RW * (int)(wave / nseg);
    if (y0 >= ny - 1) return;  // wave-uniform
    const int y1 = min(y0 + RW, ny - 1);
    const int x0 = seg * SOUT - HL * VEC + lane * VEC;
    const bool valid = x0 >= 0 && x0 < nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
    T A[NR0][VEC];  // level l in rows [l, NR0 - l) (row i = y0 - K + i)
    T R[ND][VEC];   // rhs row y0 - (K-1) + i
    uint8_t M[ND][VEC];
#pragma unroll
    for (int i = 0; i < NR0; ++i) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) A[i][k] = T(0);
        const int y = y0 - K + i;
        if (valid && y >= 0 && y <= ny - 1) ld<T, VEC>(in + row(y), A[i]);
    }
#pragma unroll
    for (int i = 0; i < ND; ++i) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) { R[i][k] = T(0); M[i][k] = 0; }
        const int y = y0 - (K - 1) + i;
        if (valid && y >= 0 && y <= ny - 1) {
            ld<T, VEC>(div + row(y), R[i]);
            if (MASK) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) M[i][k] = mask[row(y) + k];
            }
        }
    }
#pragma unroll
    for (int l = 1; l <= K; ++l) {
        T B[NR0][VEC];
#pragma unroll
        for (int i = l; i < NR0 - l; ++i) {
            const int p = y0 - K + i;
            const bool fixed = p == 0 || p == ny - 1;
            const int di = i - 1;  // rhs / mask row of row p
            const T wl = dpp_from_lower(A[i][VEC - 1]);
            const T er = dpp_from_upper(A[i][0]);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T E = (k + 1 < VEC) ? A[i][k + 1] : er;
                const T W = (k > 0) ? A[i][k - 1] : wl;
                const int x = x0 + k;
                T val = (fixed || x <= 0 || x >= nx - 1)
                            ? A[i][k]
                            : jac5<T>(E, W, A[i + 1][k], A[i - 1][k], R[di][k], dx2, dtv, PRE);
                if (MASK && M[di][k]) val = T(0);
                B[i][k] = val;
            }
        }
#pragma unroll
        for (int i = l; i < NR0 - l; ++i)
#pragma unroll
            for (int k = 0; k < VEC; ++k) A[i][k] = B[i][k];
    }
    if (writer) {
#pragma unroll
        for (int i = K; i < K + RW; ++i) {
            const int p = y0 - K + i;
            if (p < y1) st<T, VEC>(out + row(p), A[i]);
        }
    }
}

template <typename T, int VEC>
static int jacobi2d_small_pass(int K, const T *in, T *out, const T *div, const uint8_t *mask, int ny,
                               int nx, T dx2, T dtv, bool pre, int rw, hipStream_t s) {
    if (ny - 2 <= 0) return CFD_OK;
#define CFD_J2S(KV, PR, M, RWV)                                                                      \
    do {                                                                                             \
        constexpr int HL_ = (KV + VEC - 1) / VEC;                                                    \
        const int nseg = ceil_div(nx, (64 - 2 * HL_) * VEC);                                         \
        const int blocks = ceil_div((long)nseg * ceil_div(ny - 2, RWV), 4);                          \
        hipLaunchKernelGGL((jacobi2d_small<T, VEC, KV, PR, M, RWV>), dim3(blocks), dim3(256), 0, s, in, \
                           out, div, mask, ny, nx, nseg, dx2, dtv);                                  \
    } while (0)
#define CFD_J2SR(KV, RWV)                                                              \
    do {                                                                               \
        if (mask) {                                                                    \
            if (pre) CFD_J2S(KV, true, true, RWV); else CFD_J2S(KV, false, true, RWV); \
        } else {                                                                       \
            if (pre) CFD_J2S(KV, true, false, RWV); else CFD_J2S(KV, false, false, RWV); \
        }                                                                              \
    } while (0)
#define CFD_J2SK(KV)                       \
    do {                                   \
        if (rw == 2) CFD_J2SR(KV, 2);      \
        else CFD_J2SR(KV, 1);              \
    } while (0)
    switch (K) {
        case 1: CFD_J2SK(1); break;
        case 2: CFD_J2SK(2); break;
        case 3: CFD_J2SK(3); break;
        case 4: CFD_J2SK(4); break;
        case 5: CFD_J2SK(5); break;
        case 6: CFD_J2SK(6); break;
        case 7: CFD_J2SK(7); break;
        default: CFD_J2SK(8); break;
    }
#undef CFD_J2SK
#undef CFD_J2SR
#undef CFD_J2S
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// r01 at 8192^2 f64 (Gcell/s): K=2 368, 3 554, 4 752, 5 876, 6 1051, 8 1232,
// 10 1228, 12 1155 (the pass turns latency-bound past 8 levels)
constexpr int kDefaultLevels2d = 8;
// Auto depth: 8 levels when the grid fills the chip with long row chunks
// (at least 16 rows per wave with ~12 resident waves per CU), else 2 -- on a
// small grid a pass is a chain of row-step latencies, 2(K-1) of them wasted
// per chunk.  r01 on the 600 x 180 cylinder (f32, masked): K = 1 / 2 / 3 / 4
// / 6 / 8 -> 5.0 / 2.7 / 3.1 / 3.7 / 4.8 / 5.8 us per sweep.
template <typename T>
static int auto_levels2d(int ny, int nx) {
    constexpr int V = 16 / sizeof(T);
    const int sout = (64 - 2 * ((kDefaultLevels2d + V - 1) / V)) * V;
    const long work = (long)(ny - 2) * ceil_div(nx, sout);
    return work >= 16L * 12 * 256 ? kDefaultLevels2d : 2;
}

template <typename T>
__global__ void k_rhs2d(const T *__restrict__ div, T *__restrict__ rhs, size_t n, T dx2, T dtv) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
         k += (size_t)gridDim.x * blockDim.x)
        rhs[k] = (dx2 * div[k]) / dtv;
}

// the last 2-D Jacobi solve of this thread: which path ran and its sweeps
// per launch (cfd_get_last_jacobi2d_path, for the bench's per-launch roofline)
thread_local int g_j2_last[2] = {0, 0};

template <typename T>
static int jacobi2d_solve(const T *div, T *phi, T *tmp, T *rhs_ws, const uint8_t *mask, int ny,
                          int nx, T dx2, T dtv, int iters, int resid_every, T *resid_out,
                          hipStream_t s, bool zero = false) {
    CFD_REQUIRE(div && phi && tmp, "jacobi2d: null array pointer");
    CFD_REQUIRE(ny >= 1 && nx >= 1, "jacobi2d: bad shape (%d, %d)", ny, nx);
    CFD_REQUIRE(iters >= 0, "jacobi2d: iters < 0");
    CFD_REQUIRE(resid_every <= 0 || resid_out, "jacobi2d: resid_every > 0 needs resid_out");
    if (iters == 0) return CFD_OK;
    int rc;
    if constexpr (std::is_same_v<T, float>) {
        // small f32 grids (those the launch-per-pass kernel would take): the
        // whole solve as one persistent launch, any row length.  It keeps the
        // edge rows itself and forms dx2 * div / dt per cell, so neither the
        // edge-row copy nor the RHS prologue below runs.
        if (tuning().j2_blocking == 0 && resid_every <= 0 && ny >= 3 &&
            auto_levels2d<T>(ny, nx) != kDefaultLevels2d) {
            int prc = CFD_OK;
            const int tk = timing_begin(s);
            if (jacobi2d_persist_solve(phi, div, false, mask, ny, nx, dx2, dtv, iters, s, &prc, zero)) {
                if (prc) return prc;
                g_j2_last[0] = 1;
                g_j2_last[1] = iters;
                timing_end(tk, s, iters);
                return CFD_OK;
            }
            timing_cancel(tk);
        }
    }
    if (zero) CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(T) * (size_t)ny * nx, s));  // v5.py:337
    // Dirichlet rows 0 and ny-1 of the first output buffer (masked -> 0)
    if ((rc = fix_edge_rows<T>(phi, tmp, mask, ny, nx, s))) return rc;
    const int nres = resid_every > 0 ? iters / resid_every : 0;
    if (nres > 0) CFD_CHECK_HIP(hipMemsetAsync(resid_out, 0, sizeof(T) * nres, s));
    // RHS prologue: with a workspace the sweeps read rhs instead of dividing
    const bool pre = rhs_ws != nullptr;
    const T *src = div;
    if (pre) {
        const size_t n = (size_t)ny * nx;
        long blocks = (long)((n + 255) / 256);
        if (blocks > 4096) blocks = 4096;
        hipLaunchKernelGGL(k_rhs2d<T>, dim3(blocks), dim3(256), 0, s, div, rhs_ws, n, dx2, dtv);
        CFD_LAUNCH_CHECK();
        src = rhs_ws;
    }
    constexpr int V = 16 / sizeof(T);
    const bool vec_ok = (nx % V == 0) && aligned16(src) && aligned16(phi) && aligned16(tmp);
    T *a = phi, *b = tmp;
    const int tk = timing_begin(s);
    if (tuning().j2_blocking != 1 && vec_ok && resid_every <= 0 && iters >= 2 && ny >= 3) {
        // temporally blocked: passes of K sweeps, the remainder last
        // small grids (auto depth 2) take the preloaded kernel, 4 sweeps a pass
        const bool small = tuning().j2_blocking == 0 && auto_levels2d<T>(ny, nx) != kDefaultLevels2d;
        // the preloaded kernel's shape: sweeps per launch (1..8), output rows per
        // wave (1 or 2), cells per lane (1 or 16 B) -- Tuning, cfd_set_small2d_shape
        const int ks = tuning().j2s_k, srw = tuning().j2s_rw, svec = tuning().j2s_vec;
        const int K = small ? ks : tuning().j2_blocking >= 2 ? tuning().j2_blocking : auto_levels2d<T>(ny, nx);
        g_j2_last[0] = 0;
        g_j2_last[1] = K < iters ? K : iters;
        int done = 0;
        while (done < iters) {
            int k = iters - done < K ? iters - done : K;
            if (!small && (k == 7 || k == 9 || k == 11)) --k;  // tbk depths: 2..6, 8, 10, 12
            rc = small    ? (svec == 1 ? jacobi2d_small_pass<T, 1>(k, a, b, src, mask, ny, nx, dx2, dtv, pre, srw, s)
                                       : jacobi2d_small_pass<T, V>(k, a, b, src, mask, ny, nx, dx2, dtv, pre, srw, s))
                 : k == 1 ? jacobi2d_sweep<T, V>(a, b, src, mask, ny, nx, dx2, dtv, pre, nullptr, s)
                          : jacobi2d_tbk_pass<T, V>(k, a, b, src, mask, ny, nx, dx2, dtv, pre, s);
            if (rc) return rc;
            if (done == 0 && (rc = fix_edge_rows<T>(tmp, phi, nullptr, ny, nx, s))) return rc;
            done += k;
            T *t = a; a = b; b = t;
        }
        timing_end(tk, s, iters);
        if (a != phi) CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(T) * (size_t)ny * nx, hipMemcpyDeviceToDevice, s));
        return CFD_OK;
    }
    g_j2_last[0] = 0;
    g_j2_last[1] = 1;
    for (int it = 0; it < iters; ++it) {
        T *r = (resid_every > 0 && (it + 1) % resid_every == 0) ? resid_out + ((it + 1) / resid_every - 1)
                                                                 : nullptr;
        rc = vec_ok ? jacobi2d_sweep<T, V>(a, b, src, mask, ny, nx, dx2, dtv, pre, r, s)
                    : jacobi2d_sweep<T, 1>(a, b, src, mask, ny, nx, dx2, dtv, pre, r, s);
        if (rc) return rc;
        // after sweep 1, give the other buffer the final edge rows too
        if (it == 0 && iters > 1 && (rc = fix_edge_rows<T>(tmp, phi, nullptr, ny, nx, s))) return rc;
        T *t = a; a = b; b = t;
    }
    timing_end(tk, s, iters);
    if (a != phi) CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(T) * (size_t)ny * nx, hipMemcpyDeviceToDevice, s));
    return CFD_OK;
}

// ----------------------------------------------------------- red-black GS
// Workspace layout (RbgsWs, internal.hpp): flags[1] = iterations done by the
// fused path, then float maxc[iterations] at byte 16.

// Colour pass, in place.  Each thread owns a 4-cell x-vector of one row and
// rewrites it whole (cells of the other colour unchanged; nobody else writes
// them in this pass).  Stop rule (v5.py:224-225) is evaluated on device: the
// pass of iteration `it` runs only if no earlier iteration ended with
// max_change < tol; the first pass to see that records `it` in iters_done.
__device__ inline bool rbgs_stopped(const RbgsWs *ws, int it, float tol) {
    return it > 0 && ws->maxc[it - 1] < tol;
}

__global__ void rbgs_init(RbgsWs *ws, int iterations, float tol, int *iters_done) {
    for (int k = threadIdx.x; k < iterations; k += blockDim.x) ws->maxc[k] = 0.0f;
    if (threadIdx.x == 0) {
        ws->flags[0] = iterations;
        ws->flags[1] = iterations;
        ws->flags[2] = __float_as_int(tol);
        ws->flags[3] = 0;
        if (iters_done) *iters_done = iterations;
    }
}

int launch_rbgs_init(RbgsWs *ws, int iterations, float tol, int *iters_done, hipStream_t s) {
    hipLaunchKernelGGL(rbgs_init, dim3(1), dim3(1024), 0, s, ws, iterations, tol, iters_done);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// Iterations done = 1 + the first iteration whose max|change| < tol (the
// reference's break, v5.py:224-225), else all: iterations after a stop never
// write maxc, which stays 0 (< tol whenever a stop is possible at all).  One
// wave scans maxc; the count goes to flags[1] and *iters_done.
__global__ void rbgs_count(RbgsWs *__restrict__ ws, int *iters_done) {
    const int n = ws->flags[0];
    const float tol = __int_as_float(ws->flags[2]);
    int first = n;
    for (int base = 0; base < n; base += 64) {
        const int i = base + (int)threadIdx.x;
        const bool hit = i < n && ws->maxc[i] < tol;
        const unsigned long long m = __ballot(hit);
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

int launch_rbgs_count(RbgsWs *ws, int *iters_done, hipStream_t s) {
    hipLaunchKernelGGL(rbgs_count, dim3(1), dim3(64), 0, s, ws, iters_done);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// The fused paths ping-pong phi / phi_tmp, one buffer per pass; where the
// last iteration landed depends on the device-side stop, so the copy-back is
// decided on device too (no host sync in the solve): after c iterations at
// `hpp` half-sweeps per pass the result is in buffer ceil(2c / hpp) & 1.
__global__ void rbgs_copy(const RbgsWs *__restrict__ ws, float *__restrict__ phi,
                          const float *__restrict__ tmp, size_t n, int hpp) {
    const int c = ws->flags[1];
    if (!(((2 * c + hpp - 1) / hpp) & 1)) return;
    const size_t n4 = n / 4;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (size_t k = t0; k < n4; k += stride)
        reinterpret_cast<float4 *>(phi)[k] = reinterpret_cast<const float4 *>(tmp)[k];
    for (size_t k = 4 * n4 + t0; k < n; k += stride) phi[k] = tmp[k];
}

int launch_rbgs_copy(const RbgsWs *ws, float *phi, const float *phi_tmp, size_t n, int hpp,
                     hipStream_t s) {
    if (!phi_tmp) return CFD_OK;
    long blocks = (long)((n / 4 + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(rbgs_copy, dim3(blocks), dim3(256), 0, s, ws, phi, phi_tmp, n, hpp);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int launch_rbgs_finish(RbgsWs *ws, float *phi, const float *phi_tmp, size_t n, int *iters_done,
                       hipStream_t s) {
    int rc = launch_rbgs_count(ws, iters_done, s);
    return rc ? rc : launch_rbgs_copy(ws, phi, phi_tmp, n, 2, s);
}

// Fused red-black iteration, 2-D: the overlapped-segment row march of
// jacobi2d_tb2 with the colour-0 half-sweep as the first level and the
// colour-1 half-sweep as the second, out of place (12 B per cell per
// iteration instead of ~2 x 12 B for two in-place colour passes).  Masked
// cells keep their value (v5.py:216).  Bit-identical to rbgs2d_color<0/1>.
__device__ inline float gs5(float E, float W, float N, float S, float d, float cx, float cy,
                            float cd, float dt_inv) {
    const float rhs = -d * dt_inv;
    const float a = cx * (E + W);
    const float b = cy * (N + S);
    return ((a + b) - rhs) * cd;
}

template <bool MASK>
__global__ __launch_bounds__(256) void rbgs2d_tb(const float *__restrict__ in,
                                                 float *__restrict__ out,
                                                 const float *__restrict__ div,
                                                 const uint8_t *__restrict__ mask, int ny, int nx,
                                                 int nseg, int rows_per_chunk, float cx, float cy,
                                                 float cd, float dt_inv, float tol, RbgsWs *ws,
                                                 int it) {
    constexpr int VEC = 4;
    constexpr int SOUT = 64 * VEC - 2 * VEC;
    // the stop test (a global load) is read here but acted on after the first
    // row loads are issued, so the two latencies overlap (small grids run a
    // pass in a few microseconds)
    const float prev = it > 0 ? *reinterpret_cast<volatile float *>(&ws->maxc[it - 1]) : 0.f;
    const bool stopped = it > 0 && prev < tol;
    if (stopped && blockIdx.x == 0 && threadIdx.x == 0) atomicMin(&ws->flags[1], it);
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x / 64;
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * wpb + threadIdx.x / 64;
    const int seg = (int)(wave % nseg);
    const int chunk = (int)(wave / nseg);
    const int y0 = 1 + chunk * rows_per_chunk;
    float mx = 0.f;
    if (y0 < ny - 1) {  // wave-uniform
        const int y1 = min(y0 + rows_per_chunk, ny - 1);
        const int xs = seg * SOUT;
        const int x0 = xs - VEC + lane * VEC;
        const bool valid = x0 >= 0 && x0 < nx;
        const bool writer = lane >= 1 && lane <= 62 && valid;
        float am[VEC], ac[VEC], ap[VEC], app[VEC];  // level 0 rows r-1, r, r+1, r+2
        float bm[VEC], bc[VEC];                     // level 1 rows r-2, r-1
        float dm[VEC], dc[VEC], dn[VEC];            // div rows r-1, r, r+1
        uint8_t mm[VEC], mc[VEC], mn[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            am[k] = ac[k] = ap[k] = app[k] = bm[k] = bc[k] = dm[k] = dc[k] = dn[k] = 0.f;
            mm[k] = mc[k] = mn[k] = 0;
        }
        const int rs = y0 - 1;
        auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
        if (valid) {
            if (rs - 1 >= 0) ld<float, VEC>(in + row(rs - 1), am);
            ld<float, VEC>(in + row(rs), ac);
            ld<float, VEC>(in + row(rs + 1), ap);
            ld<float, VEC>(div + row(rs), dc);
            ld<float, VEC>(div + row(rs + 1), dn);
            if (MASK) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) { mc[k] = mask[row(rs) + k]; mn[k] = mask[row(rs + 1) + k]; }
            }
        }
        if (stopped) return;  // an earlier iteration met the tolerance (v5.py:224-225)
        for (int r = rs; r <= y1; ++r) {
            if (valid && r + 1 <= y1 && r + 2 <= ny - 1) ld<float, VEC>(in + row(r + 2), app);
            // level 1 (colour 0) of row r
            const bool edge = r == 0 || r == ny - 1;
            const float wl = dpp_from_lower(ac[VEC - 1]);
            const float er = dpp_from_upper(ac[0]);
            float l1[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const int x = x0 + k;
                l1[k] = ac[k];
                if (!edge && x >= 1 && x < nx - 1 && ((r + x + 1) & 1) == 0 && !(MASK && mc[k])) {
                    const float E = (k + 1 < VEC) ? ac[k + 1] : er;
                    const float W = (k > 0) ? ac[k - 1] : wl;
                    l1[k] = gs5(E, W, ap[k], am[k], dc[k], cx, cy, cd, dt_inv);
                    // halo lanes 0 / 63 duplicate neighbour segments' cells, and
                    // their outer cell sees no true x-neighbour: not counted
                    const float ch = fabsf(l1[k] - ac[k]);
                    if (writer && ch > mx) mx = ch;
                }
            }
            // level 2 (colour 1) of row r-1
            const float wl1 = dpp_from_lower(bc[VEC - 1]);
            const float er1 = dpp_from_upper(bc[0]);
            if (r >= y0 + 1 && writer) {
                float o[VEC];
#pragma unroll
                for (int k = 0; k < VEC; ++k) {
                    const int x = x0 + k;
                    o[k] = bc[k];
                    if (x >= 1 && x < nx - 1 && ((r - 1 + x + 2) & 1) == 0 && !(MASK && mm[k])) {
                        const float E = (k + 1 < VEC) ? bc[k + 1] : er1;
                        const float W = (k > 0) ? bc[k - 1] : wl1;
                        o[k] = gs5(E, W, l1[k], bm[k], dm[k], cx, cy, cd, dt_inv);
                        const float ch = fabsf(o[k] - bc[k]);
                        if (ch > mx) mx = ch;
                    }
                }
                st<float, VEC>(out + row(r - 1), o);
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                am[k] = ac[k]; ac[k] = ap[k]; ap[k] = app[k];
                bm[k] = bc[k]; bc[k] = l1[k];
                dm[k] = dc[k]; dc[k] = dn[k];
                if (MASK) { mm[k] = mc[k]; mc[k] = mn[k]; }
            }
            if (valid && r + 2 <= y1 && r + 2 <= ny - 1) {
                ld<float, VEC>(div + row(r + 2), dn);
                if (MASK) {
#pragma unroll
                    for (int k = 0; k < VEC; ++k) mn[k] = mask[row(r + 2) + k];
                }
            }
        }
    }
    if (stopped) return;
    wave_reduce_max_store(mx, &ws->maxc[it]);
}

// rbgs2d_tb for small grids: each wave owns TWO output rows and loads every
// row it needs up front, so a pass is one load latency, the colour levels and
// the stores -- no row march with a load per step.  NI = 2 fuses two
// iterations (four colour levels: level 0 rows y0-4 .. y0+5, div / mask rows
// y0-3 .. y0+4; the halo lane of 4 cells absorbs the 4-cell x-erosion).  A
// stop after the first iteration of a pair is undone after the loop by a
// rollback run of that iteration alone (NI = 1, rollback != 0: it reads the
// count and re-runs iteration 2m from the pair's input buffer, which no later
// pass overwrote), as the 3-D pair passes do.  Same cells, operation order
// and max|change| accounting as rbgs2d_tb (own rows; halo rows repeat a
// neighbour chunk's values).
constexpr int kGsSlots = 16;  // per-iteration maxima slots of rbgs2d_small

// maxc[k] = max over the slots of iteration k (before rbgs_count)
__global__ void rbgs_fold_slots(RbgsWs *ws, int niters) {
    const float *slots = ws->maxc + niters;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < niters; k += gridDim.x * blockDim.x) {
        float m = 0.f;
#pragma unroll
        for (int q = 0; q < kGsSlots; ++q) m = fmaxf(m, slots[(size_t)q * niters + k]);
        ws->maxc[k] = m;
    }
}

template <bool MASK, int NI, int VEC = 4, int RW = 2, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void rbgs2d_small(const float *__restrict__ in,
                                                    float *__restrict__ out,
                                                    const float *__restrict__ div,
                                                    const uint8_t *__restrict__ mask, int ny, int nx,
                                                    int nseg, float cx, float cy, float cd,
                                                    float dt_inv, float tol, RbgsWs *ws, int it,
                                                    int rollback, int niters) {
    // per-iteration maxima go to kGsSlots slot rows (slot-major, after
    // maxc[niters]) instead of one word: the workgroups' device-scope atomics
    // spread over kGsSlots addresses in different lines (same-address ones
    // serialise, ~10 ns each); rbgs_fold_slots folds them into maxc
    float *slots = ws->maxc + niters;
    constexpr int L = 2 * NI;                    // colour levels
    constexpr int HL = (L + VEC - 1) / VEC;      // halo lanes per side (erosion)
    constexpr int SOUT = (64 - 2 * HL) * VEC;    // output cells per wave
    constexpr int NR0 = RW + 2 * L;              // level-0 rows y0-L .. y0+RW-1+L
    constexpr int ND = RW + 2 * (L - 1);         // div / mask rows y0-(L-1) .. y0+RW-1+L-1
    bool stopped = false;
    if (rollback) {
        // rollback = P, the iterations per launch of the solve: the stop fell
        // inside launch g = (c - 1) / P when it ends before the launch's last
        // iteration; re-run its first need = c - P g iterations from the
        // launch's input buffer (no later launch overwrote it) into its
        // output.  One rollback launch per possible need; this one does NI.
        const int P = rollback, c = ws->flags[1], g = (c - 1) / P, need = c - P * g;
        const int len = min(P, niters - P * g);  // iterations launch g ran
        if (need != NI || need >= len) return;  // grid-uniform
        it = P * g;
        if (g & 1) {  // launch g read phi_tmp
            float *t_ = const_cast<float *>(in);
            in = out;
            out = t_;
        }
    } else {
        // the stop test's loads are issued here but acted on after the row
        // loads, so the latencies overlap; a launch skips when any of the last
        // four iterations met the tolerance (the previous launch's: a stop
        // earlier than those already skipped that launch)
        // lane l reads slot l % kGsSlots of iteration it - 1 - l / kGsSlots
        static_assert(4 * kGsSlots == 64, "one lane per (slot, iteration)");
        const int ln = threadIdx.x & 63, sl = ln % kGsSlots, back = 1 + ln / kGsSlots;
        const bool rd = it - back >= 0;
        const float pv = rd ? *reinterpret_cast<volatile float *>(&slots[(size_t)sl * niters + it - back]) : 0.f;
#pragma unroll
        for (int b = 1; b <= 4; ++b) {
            const float pb = wave_max(back == b ? pv : 0.f);
            stopped = stopped || (it >= b && pb < tol);
        }
        // grid-uniform (every lane read the same words): a scalar branch, so the
        // level arrays below need no exec-masked copies (584 v_mov without it)
        stopped = __builtin_amdgcn_readfirstlane((int)stopped) != 0;
        if (stopped && blockIdx.x == 0 && threadIdx.x == 0) atomicMin(&ws->flags[1], it);
    }
    const int lane = threadIdx.x & 63;
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * WPB + threadIdx.x / 64;
    const int seg = (int)(wave % nseg);
    const int y0 = 1 + RW * (int)(wave / nseg);
    float mx[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) mx[q] = 0.f;
    if (y0 < ny - 1) {  // wave-uniform
        const int y1 = min(y0 + RW, ny - 1);
        const int x0 = seg * SOUT - HL * VEC + lane * VEC;
        const bool valid = x0 >= 0 && x0 < nx;
        const bool writer = lane >= HL && lane < 64 - HL && valid;
        auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
        float A[NR0][VEC];  // level l lives in rows [l, NR0 - l) of A (row i = y0 - L + i)
        float D[ND][VEC];   // div row y0 - (L-1) + i
        uint8_t Mk[ND][VEC];
        // unconditional loads from clamped rows, then selects: a load under a
        // branch makes the compiler copy the whole row array at every merge
        // (584 v_mov at one cell per lane)
#pragma unroll
        for (int i = 0; i < NR0; ++i) {
            const int y = y0 - L + i;
            const bool in_ = valid && y >= 0 && y <= ny - 1;
            ld<float, VEC>(in + row(min(max(y, 0), ny - 1)), A[i]);
#pragma unroll
            for (int k = 0; k < VEC; ++k) A[i][k] = in_ ? A[i][k] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const int y = y0 - (L - 1) + i;
            const bool in_ = valid && y >= 0 && y <= ny - 1;
            const size_t rc = row(min(max(y, 0), ny - 1));
            ld<float, VEC>(div + rc, D[i]);
            uint32_t m4 = 0;
            if (MASK && VEC == 4) {  // 4 mask bytes in one load (nx % 4 == 0, x0 % 4 == 0)
                m4 = *reinterpret_cast<const uint32_t *>(mask + rc);
            } else if (MASK) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) m4 |= (uint32_t)mask[rc + k] << (8 * k);
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                D[i][k] = in_ ? D[i][k] : 0.f;
                Mk[i][k] = in_ ? (uint8_t)(m4 >> (8 * k)) : 0;
            }
        }
        // level-invariant per cell, computed once: the rhs (-div * dt_inv, the
        // same product gs5 forms) and which colour updates the cell (none for
        // edges, masked cells and x outside [1, nx-2]); colour c updates cells
        // with (r + x + 1 + c) even
        float RH[ND][VEC];
        bool U0[ND][VEC], U1[ND][VEC];  // updated by colour 0 / colour 1
#pragma unroll
        for (int i = 0; i < ND; ++i) {
            const int r = y0 - (L - 1) + i;
            const bool edge = r <= 0 || r >= ny - 1;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const int x = x0 + k;
                RH[i][k] = -D[i][k] * dt_inv;
                const bool ok = !edge && x >= 1 && x < nx - 1 && !(MASK && Mk[i][k]);
                const bool even = ((r + x + 1) & 1) == 0;
                U0[i][k] = ok && even;
                U1[i][k] = ok && !even;
            }
        }
        if (!stopped) {
#pragma unroll
            for (int l = 1; l <= L; ++l) {
                const int par = (l - 1) & 1;  // colour of this level
                float B[NR0][VEC];
                // rows [l, NR0 - l): level l from level l-1 (rows i-1, i, i+1)
#pragma unroll
                for (int i = l; i < NR0 - l; ++i) {
                    const int r = y0 - L + i;
                    const float *ac = A[i];
                    const float wl = dpp_from_lower(ac[VEC - 1]);
                    const float er = dpp_from_upper(ac[0]);
                    const int di = i - 1;  // div / mask row index of row r
#pragma unroll
                    for (int k = 0; k < VEC; ++k) {
                        // branch-free: every lane computes, selects keep the old value
                        // (same bits as the conditional update; fmaxf ignores a NaN
                        // change like the `ch > mx` test did)
                        const bool upd = par ? U1[di][k] : U0[di][k];
                        const float E = (k + 1 < VEC) ? ac[k + 1] : er;
                        const float W = (k > 0) ? ac[k - 1] : wl;
                        const float nv = ((cx * (E + W) + cy * (A[i + 1][k] + A[i - 1][k])) - RH[di][k]) * cd;
                        B[i][k] = upd ? nv : ac[k];
                        const float ch = upd ? fabsf(nv - ac[k]) : 0.f;
                        if (writer && r >= y0 && r < y1) mx[(l - 1) / 2] = fmaxf(mx[(l - 1) / 2], ch);
                    }
                }
#pragma unroll
                for (int i = l; i < NR0 - l; ++i)
#pragma unroll
                    for (int k = 0; k < VEC; ++k) A[i][k] = B[i][k];
            }
            if (writer) {
#pragma unroll
                for (int i = L; i < L + RW; ++i) {
                    const int p = y0 - L + i;
                    if (p < y1) st<float, VEC>(out + row(p), A[i]);
                }
            }
        }
    }
    if (rollback) return;
    // one atomic per workgroup and iteration, no read-first guard (a
    // dependent load at the end of a few-microsecond kernel)
    __shared__ float red[NI][WPB];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
        const float m = wave_max(mx[q]);
        if (lane == 0) red[q][threadIdx.x / 64] = m;
    }
    __syncthreads();
    if (threadIdx.x < NI && !stopped) {
        const int q = threadIdx.x;
        float b = red[q][0];
#pragma unroll
        for (int w = 1; w < WPB; ++w) b = fmaxf(b, red[q][w]);
        if (b > 0.0f) atomic_max_nonneg(&slots[(size_t)(blockIdx.x % kGsSlots) * niters + it + q], b);
    }
}

// rbgs2d_small with the rows shared inside a workgroup: 16 waves stack in y,
// each holding two rows of a 32-row tile (level 0 rows y0 - L .. y0 + 31 - L,
// L = 2 NI colour levels), so a level is one LDS exchange of the waves' edge
// rows and one barrier instead of every wave recomputing 2L halo rows of its
// own (rbgs2d_small: sum over levels of 2 + 2(L - l) rows per wave).  A tile
// writes its 32 - 2L inner rows.  x as in rbgs2d_small (one cell per lane by
// default, HL = ceil(L / VEC) halo lanes per side).  Stop test, max|change|
// slots, rollback: as rbgs2d_small, so the two kernels are interchangeable
// launch for launch (same cells, operation order, counts).
template <bool MASK, int NI, int VEC>
__global__ __launch_bounds__(1024) void rbgs2d_wg(const float *__restrict__ in, float *__restrict__ out,
                                                  const float *__restrict__ div,
                                                  const uint8_t *__restrict__ mask, int ny, int nx,
                                                  int nseg, float cx, float cy, float cd, float dt_inv,
                                                  float tol, RbgsWs *ws, int it, int rollback,
                                                  int niters) {
    constexpr int WPB = 16, RW = 2, T0 = WPB * RW;
    constexpr int L = 2 * NI;                // colour levels
    constexpr int OUT = T0 - 2 * L;          // output rows per tile
    constexpr int HL = (L + VEC - 1) / VEC;  // halo lanes per side
    constexpr int SOUT = (64 - 2 * HL) * VEC;
    constexpr int RS = 64 * VEC;  // LDS row
    static_assert(OUT >= 2, "too many levels for the tile");
    __shared__ float S[2][T0][RS];  // level parity, tile row
    __shared__ float red[NI][WPB];
    float *slots = ws->maxc + niters;
    bool stopped = false;
    if (rollback) {
        const int P = rollback, c = ws->flags[1], g = (c - 1) / P, need = c - P * g;
        const int len = min(P, niters - P * g);
        if (need != NI || need >= len) return;  // grid-uniform
        it = P * g;
        if (g & 1) {
            float *t_ = const_cast<float *>(in);
            in = out;
            out = t_;
        }
    }
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = bid % nseg, tile = bid / nseg;
    const int ytop = 1 + tile * OUT - L;  // global row of tile row 0
    const int x0 = seg * SOUT - HL * VEC + lane * VEC;
    const bool valid = x0 >= 0 && x0 < nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
    float A[RW][VEC], RH[RW][VEC];
    bool U0[RW][VEC], U1[RW][VEC];
    float mx[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) mx[q] = 0.f;
#pragma unroll
    for (int j = 0; j < RW; ++j) {
        const int y = ytop + RW * w + j;
        const bool in_ = valid && y >= 0 && y <= ny - 1;
        const size_t rc = row(min(max(y, 0), ny - 1));
        float D[VEC];
        ld<float, VEC>(in + rc, A[j]);
        ld<float, VEC>(div + rc, D);
        uint32_t m4 = 0;
        if (MASK && VEC == 4) {
            m4 = *reinterpret_cast<const uint32_t *>(mask + rc);
        } else if (MASK) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) m4 |= (uint32_t)mask[rc + k] << (8 * k);
        }
        const bool edge = y <= 0 || y >= ny - 1;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            A[j][k] = in_ ? A[j][k] : 0.f;
            RH[j][k] = -(in_ ? D[k] : 0.f) * dt_inv;
            const int x = x0 + k;
            const bool ok = in_ && !edge && x >= 1 && x < nx - 1 && !(MASK && ((m4 >> (8 * k)) & 0xff));
            const bool even = ((y + x + 1) & 1) == 0;
            U0[j][k] = ok && even;
            U1[j][k] = ok && !even;
        }
    }
    if (!rollback) {
        // the stop test, issued behind the row loads so that the two latencies
        // overlap; a launch skips when any of the last four iterations met the
        // tolerance (grid-uniform: every wave leaves before the first barrier)
        const int ln = threadIdx.x & 63, sl = ln % kGsSlots, back = 1 + ln / kGsSlots;
        const bool rd = it - back >= 0;
        const float pv = rd ? *reinterpret_cast<volatile float *>(&slots[(size_t)sl * niters + it - back]) : 0.f;
        bool stopped = false;
#pragma unroll
        for (int b = 1; b <= 4; ++b) {
            const float pb = wave_max(back == b ? pv : 0.f);
            stopped = stopped || (it >= b && pb < tol);
        }
        if (__builtin_amdgcn_readfirstlane((int)stopped) != 0) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicMin(&ws->flags[1], it);
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int k = 0; k < VEC; ++k) S[0][RW * w + j][lane * VEC + k] = A[j][k];
    __syncthreads();
#pragma unroll
    for (int l = 1; l <= L; ++l) {
        const int par = (l - 1) & 1;  // colour of this level
        const int rb = (l - 1) & 1, wb = l & 1;
        float B[RW][VEC];
#pragma unroll
        for (int j = 0; j < RW; ++j) {
            const int i = RW * w + j;  // tile row
            // rows i - 1 / i + 1 of level l - 1: this wave's own in registers,
            // the neighbour waves' from LDS (tile rows outside are never read:
            // rows 0 and T0 - 1 are not updated at any level >= 1)
            float Nn[VEC], Sv[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                Nn[k] = j + 1 < RW ? A[j + 1][k] : (i + 1 < T0 ? S[rb][i + 1][lane * VEC + k] : 0.f);
                Sv[k] = j > 0 ? A[j - 1][k] : (i > 0 ? S[rb][i - 1][lane * VEC + k] : 0.f);
            }
            const float wl = dpp_from_lower(A[j][VEC - 1]);
            const float er = dpp_from_upper(A[j][0]);
            const bool live = i >= l && i < T0 - l;  // rows level l is defined on
            const bool own = i >= L && i < T0 - L && ytop + i <= ny - 2;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const bool upd = live && (par ? U1[j][k] : U0[j][k]);
                const float E = (k + 1 < VEC) ? A[j][k + 1] : er;
                const float W = (k > 0) ? A[j][k - 1] : wl;
                const float nv = ((cx * (E + W) + cy * (Nn[k] + Sv[k])) - RH[j][k]) * cd;
                B[j][k] = upd ? nv : A[j][k];
                const float ch = upd ? fabsf(nv - A[j][k]) : 0.f;
                if (writer && own) mx[(l - 1) / 2] = fmaxf(mx[(l - 1) / 2], ch);
            }
        }
#pragma unroll
        for (int j = 0; j < RW; ++j)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                A[j][k] = B[j][k];
                S[wb][RW * w + j][lane * VEC + k] = B[j][k];
            }
        __syncthreads();
    }
    if (!stopped && writer) {
#pragma unroll
        for (int j = 0; j < RW; ++j) {
            const int i = RW * w + j, y = ytop + i;
            if (i >= L && i < T0 - L && y <= ny - 2) st<float, VEC>(out + row(y), A[j]);
        }
    }
    if (rollback) return;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
        const float m = wave_max(mx[q]);
        if (lane == 0) red[q][w] = m;
    }
    __syncthreads();
    if (threadIdx.x < NI && !stopped) {
        const int q = threadIdx.x;
        float b = red[q][0];
#pragma unroll
        for (int v = 1; v < WPB; ++v) b = fmaxf(b, red[q][v]);
        if (b > 0.0f) atomic_max_nonneg(&slots[(size_t)(blockIdx.x % kGsSlots) * niters + it + q], b);
    }
}

// Small grid: launch rbgs2d_small (NI = 1..4 iterations from `it`; rollback
// = P != 0: re-run the iterations of the launch of P the stop fell in).
static void rbgs2d_small_launch(int NI, const float *in, float *out, const float *div,
                                const uint8_t *mask, int ny, int nx, float cx, float cy, float cd,
                                float dt_inv, float tol, RbgsWs *ws, int it, int rollback, int niters,
                                hipStream_t s) {
    // shape: output rows per wave (1 or 2) and cells per lane (1 or 4); r01 at
    // 600 x 180, us per iteration: (1, 2) 2.36, (1, 1) 2.42, (4, 2) 3.38
    const int rw = tuning().gs_rw, vec = tuning().gs_vec, wpb = tuning().gs_wpb;
    if (tuning().gs_wg) {  // rows shared in the workgroup (rbgs2d_wg), one cell per lane
#define CFD_GSW(M, N)                                                                              \
    do {                                                                                           \
        constexpr int HL_ = 2 * N, OUT_ = 32 - 4 * N;                                              \
        const int nseg = ceil_div(nx, 64 - 2 * HL_);                                               \
        const int blocks = nseg * ceil_div(ny - 2, OUT_);                                          \
        hipLaunchKernelGGL((rbgs2d_wg<M, N, 1>), dim3(blocks), dim3(1024), 0, s, in, out, div, mask, \
                           ny, nx, nseg, cx, cy, cd, dt_inv, tol, ws, it, rollback, niters);       \
    } while (0)
#define CFD_GSW_N(M)                                  \
    do {                                              \
        switch (NI) {                                 \
            case 4: CFD_GSW(M, 4); break;             \
            case 3: CFD_GSW(M, 3); break;             \
            case 2: CFD_GSW(M, 2); break;             \
            default: CFD_GSW(M, 1); break;            \
        }                                             \
    } while (0)
        if (mask) CFD_GSW_N(true); else CFD_GSW_N(false);
#undef CFD_GSW_N
#undef CFD_GSW
        return;
    }
#define CFD_GSS_W(M, N, V, R, W)                                                                     \
    do {                                                                                             \
        constexpr int HL_ = (2 * N + V - 1) / V;                                                     \
        const int nseg = ceil_div(nx, (64 - 2 * HL_) * V);                                           \
        const int blocks = ceil_div((long)nseg * ceil_div(ny - 2, R), W);                            \
        hipLaunchKernelGGL((rbgs2d_small<M, N, V, R, W>), dim3(blocks), dim3(64 * W), 0, s, in, out, \
                           div, mask, ny, nx, nseg, cx, cy, cd, dt_inv, tol, ws, it, rollback, niters); \
    } while (0)
#define CFD_GSS(M, N, V, R)                              \
    do {                                                 \
        if (wpb == 16) CFD_GSS_W(M, N, V, R, 16);        \
        else CFD_GSS_W(M, N, V, R, 4);                   \
    } while (0)
#define CFD_GSS_VR(M, N)                                       \
    do {                                                       \
        if (vec == 1) {                                        \
            if (rw == 1) CFD_GSS(M, N, 1, 1); else CFD_GSS(M, N, 1, 2); \
        } else {                                               \
            if (rw == 1) CFD_GSS(M, N, 4, 1); else CFD_GSS(M, N, 4, 2); \
        }                                                      \
    } while (0)
#define CFD_GSS_N(M)                                   \
    do {                                               \
        switch (NI) {                                  \
            case 4: CFD_GSS_VR(M, 4); break;           \
            case 3: CFD_GSS_VR(M, 3); break;           \
            case 2: CFD_GSS_VR(M, 2); break;           \
            default: CFD_GSS_VR(M, 1); break;          \
        }                                              \
    } while (0)
    if (mask) CFD_GSS_N(true); else CFD_GSS_N(false);
#undef CFD_GSS_N
#undef CFD_GSS_VR
#undef CFD_GSS
#undef CFD_GSS_W
}

// rbgs2d_small serves grids whose row march would use chunks of <= 2 rows
static bool rbgs2d_small_grid(int ny, int nx) {
    const int nseg = ceil_div(nx, 64 * 4 - 2 * 4);
    return ceil_div((long)(ny - 2) * nseg, 8192) <= 2;
}

static int rbgs2d_tb_pass(const float *in, float *out, const float *div, const uint8_t *mask,
                          int ny, int nx, float cx, float cy, float cd, float dt_inv, float tol,
                          RbgsWs *ws, int it, hipStream_t s) {
    constexpr int SOUT = 64 * 4 - 2 * 4;
    const int nseg = ceil_div(nx, SOUT);
    const int rows = ny - 2;
    // (grids with chunks of <= 2 rows take rbgs2d_small in the solve instead)
    int rpc = ceil_div((long)rows * nseg, 8192);
    if (rpc > 64) rpc = 64;
    const int nchunk = ceil_div(rows, rpc);
    const int wpb = 4;
    const int blocks = ceil_div((long)nseg * nchunk, wpb);
    if (mask)
        hipLaunchKernelGGL(rbgs2d_tb<true>, dim3(blocks), dim3(wpb * 64), 0, s, in, out, div, mask,
                           ny, nx, nseg, rpc, cx, cy, cd, dt_inv, tol, ws, it);
    else
        hipLaunchKernelGGL(rbgs2d_tb<false>, dim3(blocks), dim3(wpb * 64), 0, s, in, out, div, mask,
                           ny, nx, nseg, rpc, cx, cy, cd, dt_inv, tol, ws, it);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

template <int C, int VEC>
__global__ __launch_bounds__(256) void rbgs2d_color(float *__restrict__ phi,
                                                    const float *__restrict__ div,
                                                    const uint8_t *__restrict__ mask, int ny,
                                                    int nx, float cx, float cy, float cd,
                                                    float dt_inv, float tol, RbgsWs *ws, int it,
                                                    int *iters_done) {
    // maxc[it-1] is final once iteration it-1's two passes completed in-stream.
    // After a stop, later iterations never write maxc, so it stays 0 < tol and
    // the stop persists (tol <= 0 never stops, like the reference).
    if (rbgs_stopped(ws, it, tol)) {
        if (C == 0 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && iters_done)
            atomicMin(iters_done, it);
        return;
    }
    const int i = blockIdx.y + 1;  // rows 1..ny-2
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * VEC;
    float mx = 0.0f;
    if (x0 < nx) {
        const size_t row = (size_t)i * nx;
        float c[VEC], n[VEC], sv[VEC], d[VEC];
        ld<float, VEC>(phi + row + x0, c);
        ld<float, VEC>(phi + row + nx + x0, n);
        ld<float, VEC>(phi + row - nx + x0, sv);
        ld<float, VEC>(div + row + x0, d);
        const float wl = x0 > 0 ? phi[row + x0 - 1] : 0.0f;
        const float er = x0 + VEC < nx ? phi[row + x0 + VEC] : 0.0f;
        float o[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            o[k] = c[k];
            const int j = x0 + k;
            // colour c visits j = 1 + (i + c) % 2 step 2  <=>  (i + j + 1 + c) even
            if (j >= 1 && j < nx - 1 && ((i + j + 1 + C) & 1) == 0 && !(mask && mask[row + j])) {
                const float E = (k + 1 < VEC) ? c[k + 1] : er;
                const float W = (k > 0) ? c[k - 1] : wl;
                const float rhs = -d[k] * dt_inv;
                const float a = cx * (E + W);
                const float b = cy * (n[k] + sv[k]);
                const float pn = ((a + b) - rhs) * cd;
                float ch = fabsf(pn - c[k]);
                if (ch > mx) mx = ch;
                o[k] = pn;
            }
        }
        st<float, VEC>(phi + row + x0, o);
    }
    wave_reduce_max_store(mx, &ws->maxc[it]);
}

template <int VEC>
static int rbgs2d_iter(float *phi, const float *div, const uint8_t *mask, int ny, int nx, float cx,
                       float cy, float cd, float dt_inv, float tol, RbgsWs *ws, int it,
                       int *iters_done, hipStream_t s) {
    const int threads = 256;
    dim3 grid(ceil_div(ceil_div(nx, VEC), threads), ny - 2);
    hipLaunchKernelGGL((rbgs2d_color<0, VEC>), grid, dim3(threads), 0, s, phi, div, mask, ny, nx,
                       cx, cy, cd, dt_inv, tol, ws, it, iters_done);
    hipLaunchKernelGGL((rbgs2d_color<1, VEC>), grid, dim3(threads), 0, s, phi, div, mask, ny, nx,
                       cx, cy, cd, dt_inv, tol, ws, it, iters_done);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // namespace cfd

using namespace cfd;

extern "C" {

int cfd_jacobi2d_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                     const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                     int resid_every, float *resid_out, void *stream) {
    // `cfg.dx**2` is a Python float; NEP 50 rounds it to float32 against the
    // float32 array (v5.py:343).
    return jacobi2d_solve<float>(div, phi, phi_tmp, rhs_ws, mask, ny, nx, (float)(dx * dx), dt,
                                 iters, resid_every, resid_out, as_stream(stream));
}

int cfd_jacobi2d_f64(const double *div, double *phi, double *phi_tmp, double *rhs_ws,
                     const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                     int resid_every, double *resid_out, void *stream) {
    return jacobi2d_solve<double>(div, phi, phi_tmp, rhs_ws, mask, ny, nx, dx * dx, (double)dt,
                                  iters, resid_every, resid_out, as_stream(stream));
}

int cfd_jacobi2d_zero_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                          const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                          int resid_every, float *resid_out, void *stream) {
    if (iters == 0 && phi && ny >= 1 && nx >= 1)
        CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(float) * (size_t)ny * nx, as_stream(stream)));
    return jacobi2d_solve<float>(div, phi, phi_tmp, rhs_ws, mask, ny, nx, (float)(dx * dx), dt, iters, resid_every,
                                 resid_out, as_stream(stream), true);
}

int cfd_jacobi2d_zero_f64(const double *div, double *phi, double *phi_tmp, double *rhs_ws,
                          const uint8_t *mask, int ny, int nx, double dx, float dt, int iters,
                          int resid_every, double *resid_out, void *stream) {
    if (iters == 0 && phi && ny >= 1 && nx >= 1)
        CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(double) * (size_t)ny * nx, as_stream(stream)));
    return jacobi2d_solve<double>(div, phi, phi_tmp, rhs_ws, mask, ny, nx, dx * dx, (double)dt, iters, resid_every,
                                  resid_out, as_stream(stream), true);
}

int cfd_get_jacobi2d_levels(void) { return tuning().j2_blocking >= 2 ? tuning().j2_blocking : kDefaultLevels2d; }

int cfd_set_jacobi2d_blocking(int steps) {
    CFD_REQUIRE((steps >= 0 && steps <= 6) || steps == 8 || steps == 10 || steps == 12,
                "blocking steps must be 0 (auto), 1 (off), 2..6, 8, 10 or 12");
    tuning().j2_blocking = steps;
    return CFD_OK;
}

int cfd_set_jacobi2d_staging(int rows_ahead) {
    CFD_REQUIRE(rows_ahead == 0 || rows_ahead == 4 || rows_ahead == 6,
                "2-D staging depth must be 0 (register prefetch), 4 or 6 rows");
    tuning().j2_dma = rows_ahead;
    return CFD_OK;
}

int cfd_get_last_jacobi2d_path(int *sweeps_per_launch) {
    if (sweeps_per_launch) *sweeps_per_launch = g_j2_last[1];
    return g_j2_last[0];
}

size_t cfd_rbgs_workspace_bytes(int iterations) {
    // flags, maxc[iterations], then the small-grid kernel's kGsSlots slot rows
    static_assert(kGsSlots == kGsSlotRows, "one slot-row count");
    return rbgs_base_bytes(iterations);
}

size_t cfd_rbgs2d_workspace_bytes(int ny, int nx, int iterations) {
    // the base workspace, then (small grids) the persistent solve's exchange rings
    const size_t base = rbgs_base_bytes(iterations);
    if (ny < 3 || nx < 3 || !rbgs2d_small_grid(ny, nx)) return base;
    return ((base + 255) & ~(size_t)255) + rbgs2d_persist_extra_bytes(ny, nx);
}

int cfd_rbgs2d_f32(float *phi, const float *div, const uint8_t *mask, int ny, int nx, double dx,
                   double dy, float dt, int iterations, double tolerance, float *phi_tmp, void *ws,
                   int *iters_done, void *stream) {
    return cfd_rbgs2d_f32_ws(phi, div, mask, ny, nx, dx, dy, dt, iterations, tolerance, phi_tmp, ws,
                             cfd_rbgs_workspace_bytes(iterations), iters_done, stream);
}

static int rbgs2d_f32_solve(float *phi, const float *div, const uint8_t *mask, int ny, int nx, double dx,
                            double dy, float dt, int iterations, double tolerance, float *phi_tmp, void *ws,
                            size_t ws_bytes, int *iters_done, void *stream, bool zero) {
    CFD_REQUIRE(phi && div && ws, "rbgs2d: null pointer");
    CFD_REQUIRE(ny >= 1 && nx >= 1 && iterations >= 0, "rbgs2d: bad arguments");
    hipStream_t s = as_stream(stream);
    // v5.py:205-210: Python-float constants, rounded to f32 where they meet f32
    const double dx2_inv = 1.0 / (dx * dx), dy2_inv = 1.0 / (dy * dy);
    const double denom_inv = 1.0 / (2.0 * (dx2_inv + dy2_inv));
    const float cx = (float)dx2_inv, cy = (float)dy2_inv, cd = (float)denom_inv;
    const float dt_inv = 1.0f / dt;  // 1.0 / np.float32 -> float32
    const float tol = (float)tolerance;
    RbgsWs *w = reinterpret_cast<RbgsWs *>(ws);
    int rc = CFD_OK;
    const bool vec_ok = (nx % 4 == 0) && aligned16(phi) && aligned16(div);
    const bool fused = phi_tmp && tuning().j2_blocking != 1 && vec_ok && aligned16(phi_tmp);
    if (ny >= 3 && nx >= 3 && iterations > 0 && fused && rbgs2d_small_grid(ny, nx)) {
        // small grid (the v5 cylinder): one persistent launch when the
        // workspace holds its rings and every tile is resident at once.  It
        // needs neither the workspace init (its failure word lives in the
        // rings, reset with them; it writes the count) nor phi_tmp's edge
        // rows (its finish copies rows 1 .. ny - 2 back): two launches fewer
        const int tk = timing_begin(s);
        if (rbgs2d_persist_solve(phi, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, phi_tmp, w, ws_bytes, iterations,
                                 iters_done, s, &rc, zero)) {
            timing_end(tk, s, iterations);
            return rc;
        }
        timing_cancel(tk);  // (the fallback below times itself)
    }
    if (zero) CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(float) * (size_t)ny * nx, s));
    rc = launch_rbgs_init(w, iterations, tol, iters_done, s);
    if (rc) return rc;
    if (ny < 3 || nx < 3 || iterations == 0) return CFD_OK;
    const int tk = timing_begin(s);
    if (fused) {
        // fused: one out-of-place pass per iteration (both colours), ping-pong
        if ((rc = fix_edge_rows<float>(phi, phi_tmp, nullptr, ny, nx, s))) return rc;
        float *a = phi, *b = phi_tmp;
        if (rbgs2d_small_grid(ny, nx)) {
            // else P iterations per launch (the last
            // launch shorter), then the rollback of a stop inside a launch
            const int P = tuning().gs_ni < 4 ? tuning().gs_ni : 4;
            CFD_CHECK_HIP(hipMemsetAsync(w->maxc + iterations, 0, sizeof(float) * kGsSlots * (size_t)iterations, s));
            for (int it = 0; it < iterations;) {
                const int m = iterations - it >= P ? P : iterations - it;
                rbgs2d_small_launch(m, a, b, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, w, it, 0, iterations, s);
                CFD_LAUNCH_CHECK();
                it += m;
                float *t = a; a = b; b = t;
            }
            timing_end(tk, s, iterations);
            hipLaunchKernelGGL(rbgs_fold_slots, dim3(ceil_div(iterations, 256)), dim3(256), 0, s, w, iterations);
            CFD_LAUNCH_CHECK();
            if ((rc = launch_rbgs_count(w, iters_done, s))) return rc;
            // one launch per possible remainder (none when no stop is possible)
            for (int need = 1; need < P && need < iterations && tol > 0.f; ++need) {
                rbgs2d_small_launch(need, phi, phi_tmp, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, w, 0, P,
                                    iterations, s);
                CFD_LAUNCH_CHECK();
            }
            return launch_rbgs_copy(w, phi, phi_tmp, (size_t)ny * nx, 2 * P, s);
        }
        for (int it = 0; it < iterations; ++it) {
            if ((rc = rbgs2d_tb_pass(a, b, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, w, it, s)))
                return rc;
            float *t = a; a = b; b = t;
        }
        timing_end(tk, s, iterations);
        return launch_rbgs_finish(w, phi, phi_tmp, (size_t)ny * nx, iters_done, s);
    }
    for (int it = 0; it < iterations; ++it) {
        rc = vec_ok ? rbgs2d_iter<4>(phi, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, w, it, iters_done, s)
                        : rbgs2d_iter<1>(phi, div, mask, ny, nx, cx, cy, cd, dt_inv, tol, w, it, iters_done, s);
        if (rc) return rc;
    }
    timing_end(tk, s, iterations);
    return CFD_OK;
}

int cfd_rbgs2d_f32_ws(float *phi, const float *div, const uint8_t *mask, int ny, int nx, double dx,
                      double dy, float dt, int iterations, double tolerance, float *phi_tmp, void *ws,
                      size_t ws_bytes, int *iters_done, void *stream) {
    return rbgs2d_f32_solve(phi, div, mask, ny, nx, dx, dy, dt, iterations, tolerance, phi_tmp, ws, ws_bytes,
                            iters_done, stream, false);
}

int cfd_rbgs2d_zero_f32_ws(float *phi, const float *div, const uint8_t *mask, int ny, int nx, double dx,
                           double dy, float dt, int iterations, double tolerance, float *phi_tmp, void *ws,
                           size_t ws_bytes, int *iters_done, void *stream) {
    return rbgs2d_f32_solve(phi, div, mask, ny, nx, dx, dy, dt, iterations, tolerance, phi_tmp, ws, ws_bytes,
                            iters_done, stream, true);
}

}  // extern "C"
