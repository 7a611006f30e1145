// jacobi3d_tb.hip -- temporally blocked 7-point sweeps: TWO levels per HBM pass.
//
// MODE_JACOBI: two Jacobi sweeps per pass.  The single-sweep kernel
// (poisson3d.hip) moves 12 B per cell-update (read phi, read div, write phi').
// This kernel fuses sweeps k+1 and k+2 in one z-march: one pass reads phi^k
// and div once and writes phi^(k+2), so 12 B of traffic buys TWO
// cell-updates.  The intermediate level phi^(k+1) never leaves the CU.
//
// MODE_RBGS: one full red-black Gauss-Seidel iteration per pass (the 3-D
// generalisation of solve_pressure_gauss_seidel_fast, v5.py:202-226).  The
// colour-0 half-sweep is the first level: colour-0 cells are updated from old
// values, colour-1 cells are copied.  The colour-1 half-sweep is the second
// level.  Out of place, 12 B per cell per iteration instead of ~24 B for two
// in-place colour passes.  The per-iteration max|change| reduces on device,
// and the stop rule (v5.py:224-225) is checked by every launch without a host
// sync.
//
// Per z-step (front plane z) a workgroup:
//   1. publishes level 0 of plane z into LDS tile A: its W+4 rows (2 halo
//      rows) plus 4-float x-halo chunks;
//   2. computes level 1 of plane z for W+2 rows (1 halo row each side) and
//      the two x-halo columns into LDS tile B.  z-neighbours come from a
//      register queue, y-neighbours from A, x-neighbours by lane shuffle;
//   3. computes level 2 of plane z-1 for its W rows from B (plane z-1, the
//      previous step's buffer) and the level-1 register queue, and stores it.
// A and B are double-buffered by plane parity: one barrier per step.  Both
// neighbouring tiles recompute the halo rows/columns of level 1.  That is the
// same arithmetic, so the result is bit-identical to the unfused sweeps
// (tests: tests/test_gpu_parity.py against the oracle).
//
// Scope: no mask, no per-sweep residual (callers fall back to the unfused
// kernels for those), nx % 4 == 0, 16-byte aligned arrays.
#include "internal.hpp"

namespace cfd {

// explicit global address space (never flat_load / flat_store)
typedef float gv4f __attribute__((ext_vector_type(4)));
__device__ inline float4 ldg4(const float *p) {
    const gv4f r = *(const __attribute__((address_space(1))) gv4f *)p;
    return make_float4(r.x, r.y, r.z, r.w);
}
__device__ inline void stg4(float *p, float4 v) {
    const gv4f r = {v.x, v.y, v.z, v.w};
    *(__attribute__((address_space(1))) gv4f *)p = r;
}

// Zero unless c.  A `c ? ldg4(p) : zero` with the zero vector captured by
// reference (an addressable local) was folded into a load from a select of
// addresses, i.e. a flat_load from scratch or HBM.
__device__ inline float4 ldg4_if(bool c, const float *p) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c) v = ldg4(p);
    return v;
}
__device__ inline float4 lds4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ inline void sts4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

enum { MODE_JACOBI = 0, MODE_RBGS = 1 };

struct Tb2Args {
    const float *in;
    float *out;
    const float *div;  // div, or the precomputed Jacobi rhs (PRE)
    int nz, ny, nx, nseg, ntile_y, zb, ze, zchunk, fixed_lo, fixed_hi;
    float h2, dt;                      // Jacobi
    float cx, cy, cz, cd, dt_inv, tol; // red-black GS
    int zoff;                          // global z of local plane 0 (colour parity)
    int it;                            // GS iteration index of this pass
    float *maxc;                       // GS: per-iteration max|change| (device)
    int *iters_done;                   // GS: iteration count (device, optional)
};

// the 7-point update of one cell; d is div (or the Jacobi rhs when PRE)
template <int MODE, bool PRE>
__device__ inline float upd7(float E, float W, float N, float S, float U, float D, float d,
                             const Tb2Args &a) {
    if (MODE == MODE_JACOBI) {
        float s = E + W;
        s = s + N;
        s = s + S;
        s = s + U;
        s = s + D;
        const float rhs = PRE ? d : (a.h2 * d) / a.dt;
        return (1.0f / 6.0f) * (s - rhs);
    } else {
        // v5.py:217-219 generalised: rhs = -div/dt, (cx(E+W) + cy(N+S) + cz(U+D) - rhs)*denom_inv
        const float rhs = -d * a.dt_inv;
        const float p = a.cx * (E + W);
        const float q = a.cy * (N + S);
        const float r = a.cz * (U + D);
        return (((p + q) + r) - rhs) * a.cd;
    }
}

// does level `lev` (0 = first) update this cell?  Jacobi: always; red-black:
// colour lev updates cells with (z + y + x + 1 + lev) even (colour 0 = odd sum,
// v5.py:213-215)
template <int MODE>
__device__ inline bool updates(int zg, int y, int x, int lev) {
    return MODE == MODE_JACOBI || ((zg + y + x + 1 + lev) & 1) == 0;
}

// PD: prefetch distance in planes (1 or 2): how many steps ahead the next
// planes' loads are issued.
//
// Roles: waves 0..G-1 ("row waves") each own one level-1 row of the tile
// (rows y0-1 .. y0+W), 64 lanes x float4 = 256 columns.  Wave G (the "halo
// wave") owns everything outside that 256 x (W+2) block: the two extra
// level-0 rows (y0-2, y0+W+1), the 4-float x-halo chunks of all W+4 rows, and
// the level-1 values of the two halo columns (x0-1, x0+256), one lane per
// (row, side).  The row waves therefore run identical, branch-free code.
template <int W, int MODE, bool PRE, int PD>
__global__ __launch_bounds__((W + 3) * 64) void jacobi3d_tb2(Tb2Args a) {
    constexpr int G = W + 2;  // row waves
    constexpr int RS = 264;   // LDS row: 4 halo | 256 | 4 halo floats
    static_assert(2 * (W + 4) <= 64, "halo wave: one lane per (row, side)");
    __shared__ __attribute__((aligned(16))) float A[2][W + 4][RS];  // level 0, rows y0-2 .. y0+W+1
    __shared__ __attribute__((aligned(16))) float B[2][G][RS];      // level 1, rows y0-1 .. y0+W

    if (MODE == MODE_RBGS && a.it > 0 && a.maxc[a.it - 1] < a.tol) {
        // the previous iteration converged (v5.py:224-225): nothing more runs
        if (blockIdx.x == 0 && threadIdx.x == 0 && a.iters_done) atomicMin(a.iters_done, a.it);
        return;
    }
    const int nz = a.nz, ny = a.ny, nx = a.nx;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = t % a.nseg;
    const int ty = (t / a.nseg) % a.ntile_y;
    const int zc = t / (a.nseg * a.ntile_y);
    const int z0 = a.zb + zc * a.zchunk;
    if (z0 >= a.ze) return;  // workgroup-uniform
    const int z1 = min(z0 + a.zchunk, a.ze);
    const int y0 = 1 + ty * W;
    const int xs = seg * 256;
    const int x = xs + 4 * lane;
    const bool xin = x < nx;
    const size_t plane = (size_t)ny * nx;
    const int zs = z0 - 1;  // first front plane
    const float *in = a.in;
    const float *div = a.div;
    auto P = [&](int p) { return in + (size_t)p * plane; };
    auto R = [&](int p) { return div + (size_t)p * plane; };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float rmax = 0.f;  // red-black: max|change| over this lane's updates

    if (wv < G) {
        // ------------------------------------------------------------ row wave
        const int g = wv;
        const int y = y0 - 1 + g;
        const bool rowin = y >= 0 && y <= ny - 1;
        const bool ld_ok = xin && rowin;
        const bool int_row = y >= 1 && y <= ny - 2;
        const bool out_row = g >= 1 && g <= W && y <= ny - 2;
        const size_t rofs = (size_t)(rowin ? y : 0) * nx + (xin ? x : 0);
        float4 cm = z4, cc = z4, cp = z4, cpp = z4, c3 = z4;  // level 0 centre, planes z-1 .. z+3
        float4 dprev = z4, dcur = z4, dnext = z4, d2 = z4;    // div/rhs, planes z-1 .. z+2
        float4 l1m2 = z4, l1m1 = z4, l1c = z4;                // level 1, planes z-2 .. z
        if (ld_ok) {
            if (zs - 1 >= 0) cm = ldg4(P(zs - 1) + rofs);
            cc = ldg4(P(zs) + rofs);
            if (zs + 1 <= nz - 1) cp = ldg4(P(zs + 1) + rofs);
            dcur = ldg4(R(zs) + rofs);
            if (PD == 2 && zs + 1 <= z1) {
                if (zs + 2 <= nz - 1) cpp = ldg4(P(zs + 2) + rofs);
                dnext = ldg4(R(zs + 1) + rofs);
            }
        }
        for (int z = zs; z <= z1; ++z) {
            const int zp = z + PD - 1;  // this step fetches what step zp+1 needs
            if (ld_ok && zp + 1 <= z1) {
                const float4 nc = ldg4_if(zp + 2 <= nz - 1, P(zp + 2) + rofs);
                const float4 nd = ldg4(R(zp + 1) + rofs);
                if constexpr (PD == 2) { c3 = nc; d2 = nd; } else { cpp = nc; dnext = nd; }
            }
            const int b = z & 1;
            if (ld_ok) sts4(&A[b][g + 1][4 + 4 * lane], cc);
            __syncthreads();
            // level 1 of plane z, row y
            const bool fixed = (z == a.zb - 1 && a.fixed_lo) || (z == a.ze && a.fixed_hi);
            float wl = __shfl_up(cc.w, 1, 64);
            float er = __shfl_down(cc.x, 1, 64);
            const float wl_l = A[b][g + 1][3], er_l = A[b][g + 1][260];
            if (lane == 0) wl = wl_l;
            if (lane == 63) er = er_l;
            float4 l1 = cc;
            if (ld_ok && int_row && !fixed) {
                const float4 N = lds4(&A[b][g + 2][4 + 4 * lane]);
                const float4 S = lds4(&A[b][g][4 + 4 * lane]);
                const float c[4] = {cc.x, cc.y, cc.z, cc.w};
                const float n[4] = {N.x, N.y, N.z, N.w};
                const float sv[4] = {S.x, S.y, S.z, S.w};
                const float u[4] = {cp.x, cp.y, cp.z, cp.w};
                const float dd[4] = {cm.x, cm.y, cm.z, cm.w};
                const float dv[4] = {dcur.x, dcur.y, dcur.z, dcur.w};
                float o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int xk = x + k;
                    const float E = k < 3 ? c[k + 1] : er;
                    const float Wv = k > 0 ? c[k - 1] : wl;
                    o[k] = c[k];
                    if (xk != 0 && xk != nx - 1 && updates<MODE>(a.zoff + z, y, xk, 0)) {
                        o[k] = upd7<MODE, PRE>(E, Wv, n[k], sv[k], u[k], dd[k], dv[k], a);
                        if (MODE == MODE_RBGS) {
                            const float ch = fabsf(o[k] - c[k]);
                            if (ch > rmax) rmax = ch;
                        }
                    }
                }
                l1 = make_float4(o[0], o[1], o[2], o[3]);
            }
            l1c = l1;
            if (ld_ok) sts4(&B[b][g][4 + 4 * lane], l1);
            // level 2 of plane z-1 (B[b^1]: last step's, behind this step's barrier)
            float wl1 = __shfl_up(l1m1.w, 1, 64);
            float er1 = __shfl_down(l1m1.x, 1, 64);
            if (z >= z0 + 1 && out_row && xin) {
                const int pb = b ^ 1;
                if (lane == 0) wl1 = B[pb][g][3];
                if (lane == 63) er1 = B[pb][g][260];
                const float4 N = lds4(&B[pb][g + 1][4 + 4 * lane]);
                const float4 S = lds4(&B[pb][g - 1][4 + 4 * lane]);
                const float c[4] = {l1m1.x, l1m1.y, l1m1.z, l1m1.w};
                const float n[4] = {N.x, N.y, N.z, N.w};
                const float sv[4] = {S.x, S.y, S.z, S.w};
                const float u[4] = {l1c.x, l1c.y, l1c.z, l1c.w};
                const float dd[4] = {l1m2.x, l1m2.y, l1m2.z, l1m2.w};
                const float dv[4] = {dprev.x, dprev.y, dprev.z, dprev.w};
                float o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int xk = x + k;
                    const float E = k < 3 ? c[k + 1] : er1;
                    const float Wv = k > 0 ? c[k - 1] : wl1;
                    o[k] = c[k];
                    if (xk != 0 && xk != nx - 1 && updates<MODE>(a.zoff + z - 1, y, xk, 1)) {
                        o[k] = upd7<MODE, PRE>(E, Wv, n[k], sv[k], u[k], dd[k], dv[k], a);
                        if (MODE == MODE_RBGS) {
                            const float ch = fabsf(o[k] - c[k]);
                            if (ch > rmax) rmax = ch;
                        }
                    }
                }
                stg4(a.out + (size_t)(z - 1) * plane + rofs, make_float4(o[0], o[1], o[2], o[3]));
            }
            cm = cc; cc = cp; cp = cpp;
            dprev = dcur; dcur = dnext;
            if constexpr (PD == 2) { cpp = c3; dnext = d2; }
            l1m2 = l1m1; l1m1 = l1c;
        }
    } else {
        // ------------------------------------------------------------ halo wave
        // extra level-0 rows (all lanes): tile row 0 = y0-2, tile row W+3 = y0+W+1
        const int ylo = y0 - 2, yhi = y0 + W + 1;
        const bool elo = xin && ylo >= 0 && ylo <= ny - 1;
        const bool ehi = xin && yhi >= 0 && yhi <= ny - 1;
        const size_t olo = (size_t)(elo ? ylo : 0) * nx + (xin ? x : 0);
        const size_t ohi = (size_t)(ehi ? yhi : 0) * nx + (xin ? x : 0);
        // halo chunks: lane -> tile row r (y0-2+r), side (0: x0-4..x0-1, 1: x0+256..x0+259)
        const int r = lane >> 1, side = lane & 1;
        const int yr = y0 - 2 + r;
        const bool hon = lane < 2 * (W + 4) && yr >= 0 && yr <= ny - 1 &&
                         (side ? xs + 256 < nx : xs > 0);
        const int hx = side ? xs + 256 : xs - 4;
        const size_t hofs = (size_t)(hon ? yr : 0) * nx + (hon ? hx : 0);
        const size_t rhofs = hofs + (side ? 0 : 3);  // the cell next to the tile
        const bool l1row = r >= 1 && r <= W + 2;     // level-1 rows y0-1 .. y0+W
        const bool hint = hon && l1row && yr >= 1 && yr <= ny - 2;
        const int col = side ? 260 : 0;               // chunk position in an LDS row
        const int px = side ? xs + 256 : xs - 1;      // the halo column's x
        float4 lo = z4, lon = z4, lo2 = z4, hi = z4, hin = z4, hi2 = z4;
        float4 hm = z4, hc = z4, hp = z4, hpp = z4, h3 = z4;
        float rh = 0.f, rhn = 0.f, rh2 = 0.f;
        if (elo) lo = ldg4(P(zs) + olo);
        if (ehi) hi = ldg4(P(zs) + ohi);
        if (hon) {
            if (zs - 1 >= 0) hm = ldg4(P(zs - 1) + hofs);
            hc = ldg4(P(zs) + hofs);
            if (zs + 1 <= nz - 1) hp = ldg4(P(zs + 1) + hofs);
            if (l1row) rh = R(zs)[rhofs];
        }
        if (PD == 2 && zs + 1 <= z1) {
            if (elo) lon = ldg4(P(zs + 1) + olo);
            if (ehi) hin = ldg4(P(zs + 1) + ohi);
            if (hon) {
                if (zs + 2 <= nz - 1) hpp = ldg4(P(zs + 2) + hofs);
                if (l1row) rhn = R(zs + 1)[rhofs];
            }
        }
        for (int z = zs; z <= z1; ++z) {
            const int zp = z + PD - 1;
            if (zp + 1 <= z1) {
                const float4 nlo = ldg4_if(elo, P(zp + 1) + olo);
                const float4 nhi = ldg4_if(ehi, P(zp + 1) + ohi);
                const float4 nh = ldg4_if(hon && zp + 2 <= nz - 1, P(zp + 2) + hofs);
                const float nr = (hon && l1row) ? R(zp + 1)[rhofs] : 0.f;
                if constexpr (PD == 2) { lo2 = nlo; hi2 = nhi; h3 = nh; rh2 = nr; }
                else { lon = nlo; hin = nhi; hpp = nh; rhn = nr; }
            }
            const int b = z & 1;
            if (elo) sts4(&A[b][0][4 + 4 * lane], lo);
            if (ehi) sts4(&A[b][W + 3][4 + 4 * lane], hi);
            if (hon) sts4(&A[b][r][col], hc);
            __syncthreads();
            // level 1 of the halo columns (x0-1 / x0+256) for rows y0-1 .. y0+W
            if (hon && l1row) {
                const bool fixed = (z == a.zb - 1 && a.fixed_lo) || (z == a.ze && a.fixed_hi);
                const float C = side ? hc.x : hc.w;
                float v = C;
                if (hint && !fixed && px != 0 && px != nx - 1 && updates<MODE>(a.zoff + z, yr, px, 0)) {
                    const float E = side ? hc.y : A[b][r][4];
                    const float Wn = side ? A[b][r][259] : hc.z;
                    const int cc_ = side ? 260 : 3;
                    v = upd7<MODE, PRE>(E, Wn, A[b][r + 1][cc_], A[b][r - 1][cc_], side ? hp.x : hp.w,
                                        side ? hm.x : hm.w, rh, a);
                }
                B[b][r - 1][side ? 260 : 3] = v;
            }
            lo = lon; hi = hin;
            hm = hc; hc = hp; hp = hpp;
            rh = rhn;
            if constexpr (PD == 2) { lon = lo2; hin = hi2; hpp = h3; rhn = rh2; }
        }
    }
    if (MODE == MODE_RBGS) {
        __shared__ float red[W + 3];
        block_reduce_max_store(rmax, a.maxc + a.it, red);
    }
}

// Launch one fused pass of mode MODE over planes [zb, ze) of `out`.
template <int MODE>
static int tb2_launch(Tb2Args a, int W, bool pre, hipStream_t s) {
    const int pd = jacobi3d_tb_prefetch();
    if (a.ze <= a.zb || a.ny < 3) return CFD_OK;
    a.nseg = ceil_div(a.nx, 256);
    a.ntile_y = ceil_div(a.ny - 2, W);
    const int L = a.ze - a.zb;
    int zchunk = a.zchunk;
    if (zchunk <= 0) {
        // >= ~1024 workgroups (4 per CU) when the grid allows; 16..128 planes
        // per march (r01 sweep at 1024^3: 64-128 best on one GPU)
        const long tiles = (long)a.nseg * a.ntile_y;
        int nzc = (int)((1024 + tiles - 1) / tiles);
        if (nzc < 1) nzc = 1;
        zchunk = ceil_div(L, nzc);
        if (zchunk > 128) zchunk = 128;
        if (zchunk < 16) zchunk = 16;
    }
    if (zchunk > L) zchunk = L;
    a.zchunk = zchunk;
    const int blocks = a.nseg * a.ntile_y * ceil_div(L, zchunk);
#define CFD_TB2_L(WV, PR, PDV) \
    hipLaunchKernelGGL((jacobi3d_tb2<WV, MODE, PR, PDV>), dim3(blocks), dim3((WV + 3) * 64), 0, s, a)
#define CFD_TB2(WV)                                                      \
    case WV:                                                             \
        if (pd == 2) {                                                   \
            if (pre) CFD_TB2_L(WV, true, 2); else CFD_TB2_L(WV, false, 2); \
        } else {                                                         \
            if (pre) CFD_TB2_L(WV, true, 1); else CFD_TB2_L(WV, false, 1); \
        }                                                                \
        break;
    switch (W) {
        CFD_TB2(5)
        CFD_TB2(13)
        default:
            set_error("jacobi3d_tb2: unsupported rows per tile %d (5, 13)", W);
            return CFD_E_INVALID;
    }
#undef CFD_TB2
#undef CFD_TB2_L
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// One fused Jacobi pass: planes [zb, ze) of `out` receive phi after two sweeps
// of `in`.  Planes zb-1 and ze must be readable; fixed_lo / fixed_hi say that
// they are Dirichlet planes (their intermediate level equals their input),
// otherwise they are updated too (2-deep ghost planes, slab mode).
int jacobi3d_tb2_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                      int ze, int fixed_lo, int fixed_hi, float h2, float dt, int W, int zchunk,
                      bool pre, hipStream_t s) {
    Tb2Args a{};
    a.in = in; a.out = out; a.div = div;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze; a.zchunk = zchunk;
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi; a.h2 = h2; a.dt = dt;
    return tb2_launch<MODE_JACOBI>(a, W, pre, s);
}

// One fused red-black GS iteration (`it`): planes [zb, ze) of `out` receive
// both colour half-sweeps of `in`; max|change| lands in ws->maxc[it].
int rbgs3d_tb_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                   int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int it,
                   RbgsWs *ws, hipStream_t s) {
    Tb2Args a{};
    a.in = in; a.out = out; a.div = div;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze; a.zchunk = jacobi3d_tb_zchunk();
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi;
    a.cx = k.cx; a.cy = k.cy; a.cz = k.cz; a.cd = k.cd; a.dt_inv = k.dt_inv; a.tol = k.tol;
    a.zoff = zoff; a.it = it; a.maxc = ws->maxc; a.iters_done = &ws->flags[1];
    return tb2_launch<MODE_RBGS>(a, jacobi3d_tb_rows(), false, s);
}

}  // namespace cfd
