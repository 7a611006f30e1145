// jacobi3d_tb.hip -- temporally blocked 7-point Jacobi: TWO sweeps per HBM pass.
//
// The single-sweep kernel (poisson3d.hip) moves 12 B per cell-update: read
// phi, read div, write phi'.  That is the floor for one sweep.  This kernel
// fuses sweeps k+1 and k+2 in one z-march, so one pass reads phi^k and div
// once and writes phi^(k+2): 12 B of traffic per TWO cell-updates.  The
// intermediate level phi^(k+1) never leaves the CU.
//
// Per z-step (front plane z) a workgroup:
//   1. publishes phi^k of plane z (its W+4 rows with 2 halo rows, and
//      256+8 columns with x-halo chunks) into LDS tile A;
//   2. computes phi^(k+1) of plane z for W+2 rows (1 halo row each side, and
//      the two x-halo columns) into LDS tile B: z-neighbours come from a
//      register queue, y-neighbours from A, x-neighbours by lane shuffle;
//   3. computes phi^(k+2) of plane z-1 for its W rows from B (plane z-1, the
//      previous step's buffer) and the phi^(k+1) register queue, and stores it.
// A and B are double-buffered by plane parity: one barrier per step.  The
// halo rows/columns of phi^(k+1) are recomputed by both neighbouring tiles.
// That redundant work is identical arithmetic, so the result is bit-identical
// to two single sweeps (checked against the oracle in tests).
//
// Scope: no mask, no residual (the solver falls back to single sweeps for
// those), nx % 4 == 0, 16-byte aligned arrays.
#include "internal.hpp"

namespace cfd {

__device__ inline float4 ldg4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ inline void stg4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
__device__ inline float4 lds4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ inline void sts4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// d is div (PRE = false: rhs = (h2*div)/dt here) or the precomputed rhs
template <bool PRE>
__device__ inline float jac7(float E, float W, float N, float S, float U, float D, float d, float h2,
                             float dt) {
    float s = E + W;
    s = s + N;
    s = s + S;
    s = s + U;
    s = s + D;
    const float rhs = PRE ? d : (h2 * d) / dt;
    return (1.0f / 6.0f) * (s - rhs);
}

template <int W, bool PRE>
__global__ __launch_bounds__((W + 2) * 64) void jacobi3d_tb2(
    const float *__restrict__ in, float *__restrict__ out, const float *__restrict__ div, int nz,
    int ny, int nx, int nseg, int ntile_y, int zb, int ze, int zchunk, int fixed_lo, int fixed_hi,
    float h2, float dt) {
    constexpr int G = W + 2;    // waves: phi^(k+1) rows y0-1 .. y0+W
    constexpr int RS = 264;     // LDS row: 4 halo | 256 | 4 halo floats
    __shared__ __attribute__((aligned(16))) float A[2][W + 4][RS];  // phi^k rows y0-2 .. y0+W+1
    __shared__ __attribute__((aligned(16))) float B[2][G][RS];      // phi^(k+1) rows y0-1 .. y0+W

    const int lane = threadIdx.x & 63;
    const int g = threadIdx.x >> 6;
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = t % nseg;
    const int ty = (t / nseg) % ntile_y;
    const int zc = t / (nseg * ntile_y);
    const int z0 = zb + zc * zchunk;
    if (z0 >= ze) return;  // workgroup-uniform
    const int z1 = min(z0 + zchunk, ze);
    const int y0 = 1 + ty * W;
    const int y = y0 - 1 + g;
    const int xs = seg * 256;
    const int x = xs + 4 * lane;
    const bool xin = x < nx;
    const bool rowin = y >= 0 && y <= ny - 1;
    const bool ld_ok = xin && rowin;
    const bool int_row = y >= 1 && y <= ny - 2;
    const bool out_row = g >= 1 && g <= W && y <= ny - 2;
    // extra phi^k rows: wave 0 -> y0-2, last wave -> y0+W+1
    const bool has_extra = g == 0 || g == G - 1;
    const int ye = g == 0 ? y0 - 2 : y0 + W + 1;
    const bool extra_ok = has_extra && xin && ye >= 0 && ye <= ny - 1;
    const int arow_extra = g == 0 ? 0 : W + 3;
    // x-halo chunks: lane 0 -> [xs-4, xs), lane 63 -> [xs+256, xs+260)
    const bool halo_lane = (lane == 0 && xs > 0) || (lane == 63 && xs + 256 < nx);
    const int hx = lane == 0 ? xs - 4 : xs + 256;
    const int hcol = lane == 0 ? 0 : 260;
    const bool hal_ok = halo_lane && rowin;
    const bool ehal_ok = halo_lane && has_extra && ye >= 0 && ye <= ny - 1;

    const size_t plane = (size_t)ny * nx;
    const size_t rofs = (size_t)(rowin ? y : 0) * nx + (xin ? x : 0);
    const size_t eofs = (size_t)(extra_ok ? ye : 0) * nx + (xin ? x : 0);
    const size_t hofs = (size_t)(rowin ? y : 0) * nx + (halo_lane ? hx : 0);
    const size_t ehofs = (size_t)(ehal_ok ? ye : 0) * nx + (halo_lane ? hx : 0);
    const int hd = lane == 0 ? 3 : 0;  // the halo cell next to the tile

    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 cm = z4, cc = z4, cp = z4, cpp = z4;  // phi^k centre, planes z-1 .. z+2
    float4 hm = z4, hc = z4, hp = z4, hpp = z4;  // phi^k x-halo chunk
    float4 ec = z4, ecn = z4, ehc = z4, ehcn = z4;
    float4 dcur = z4, dnext = z4, dprev = z4;
    float dh = 0.f, dhn = 0.f;
    float4 l1m2 = z4, l1m1 = z4, l1c = z4;  // phi^(k+1) centre, planes z-2 .. z

    const int zs = z0 - 1;  // first front plane
    auto P = [&](int p) { return in + (size_t)p * plane; };
    if (ld_ok) {
        if (zs - 1 >= 0) cm = ldg4(P(zs - 1) + rofs);
        cc = ldg4(P(zs) + rofs);
        if (zs + 1 <= nz - 1) cp = ldg4(P(zs + 1) + rofs);
        dcur = ldg4(div + (size_t)zs * plane + rofs);
    }
    if (hal_ok) {
        if (zs - 1 >= 0) hm = ldg4(P(zs - 1) + hofs);
        hc = ldg4(P(zs) + hofs);
        if (zs + 1 <= nz - 1) hp = ldg4(P(zs + 1) + hofs);
        dh = div[(size_t)zs * plane + hofs + hd];
    }
    if (extra_ok) ec = ldg4(P(zs) + eofs);
    if (ehal_ok) ehc = ldg4(P(zs) + ehofs);

    for (int z = zs; z <= z1; ++z) {
        const bool more = z < z1;
        if (more) {  // prefetch for the next step
            if (z + 2 <= nz - 1) {
                if (ld_ok) cpp = ldg4(P(z + 2) + rofs);
                if (hal_ok) hpp = ldg4(P(z + 2) + hofs);
            }
            if (extra_ok) ecn = ldg4(P(z + 1) + eofs);
            if (ehal_ok) ehcn = ldg4(P(z + 1) + ehofs);
            if (ld_ok) dnext = ldg4(div + (size_t)(z + 1) * plane + rofs);
            if (hal_ok) dhn = div[(size_t)(z + 1) * plane + hofs + hd];
        }
        const int b = z & 1;
        // 1. publish phi^k of plane z
        if (ld_ok) sts4(&A[b][g + 1][4 + 4 * lane], cc);
        if (hal_ok) sts4(&A[b][g + 1][hcol], hc);
        if (extra_ok) sts4(&A[b][arow_extra][4 + 4 * lane], ec);
        if (ehal_ok) sts4(&A[b][arow_extra][hcol], ehc);
        __syncthreads();

        // 2. phi^(k+1) of plane z
        const bool fixed = (z == zb - 1 && fixed_lo) || (z == ze && fixed_hi);
        float wl = __shfl_up(cc.w, 1, 64);
        float er = __shfl_down(cc.x, 1, 64);
        if (lane == 0) wl = hc.w;
        if (lane == 63) er = hc.x;
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
                o[k] = (xk == 0 || xk == nx - 1) ? c[k] : jac7<PRE>(E, Wv, n[k], sv[k], u[k], dd[k], dv[k], h2, dt);
            }
            l1 = make_float4(o[0], o[1], o[2], o[3]);
        }
        l1c = l1;
        if (ld_ok) sts4(&B[b][g][4 + 4 * lane], l1);
        if (hal_ok) {  // the halo column next to the tile
            float v;
            if (lane == 0) {
                v = hc.w;  // x = xs-1
                if (int_row && !fixed)
                    v = jac7<PRE>(cc.x, hc.z, A[b][g + 2][3], A[b][g][3], hp.w, hm.w, dh, h2, dt);
                B[b][g][3] = v;
            } else {
                v = hc.x;  // x = xs+256
                if (int_row && !fixed && xs + 256 != nx - 1)
                    v = jac7<PRE>(hc.y, cc.w, A[b][g + 2][260], A[b][g][260], hp.x, hm.x, dh, h2, dt);
                B[b][g][260] = v;
            }
        }

        // 3. phi^(k+2) of plane z-1 (B[b^1] was written last step, behind this step's barrier)
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
                o[k] = (xk == 0 || xk == nx - 1) ? c[k] : jac7<PRE>(E, Wv, n[k], sv[k], u[k], dd[k], dv[k], h2, dt);
            }
            stg4(out + (size_t)(z - 1) * plane + rofs, make_float4(o[0], o[1], o[2], o[3]));
        }
        // rotate the queues
        cm = cc; cc = cp; cp = cpp;
        hm = hc; hc = hp; hp = hpp;
        ec = ecn; ehc = ehcn;
        dprev = dcur; dcur = dnext; dh = dhn;
        l1m2 = l1m1; l1m1 = l1c;
    }
}

// One fused pass: planes [zb, ze) of `out` receive phi after two sweeps of
// `in`.  Planes zb-1 and ze must be readable; fixed_lo / fixed_hi say that
// they are Dirichlet planes (their intermediate level equals their input),
// otherwise they are updated too (2-deep ghost planes, slab mode).
int jacobi3d_tb2_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                      int ze, int fixed_lo, int fixed_hi, float h2, float dt, int W, int zchunk,
                      bool pre, hipStream_t s) {
    if (ze <= zb || ny < 3) return CFD_OK;
    const int nseg = ceil_div(nx, 256);
    const int ntile_y = ceil_div(ny - 2, W);
    const int L = ze - zb;
    if (zchunk <= 0) {
        const long tiles = (long)nseg * ntile_y;
        int nzc = (int)((1024 + tiles - 1) / tiles);
        if (nzc < 1) nzc = 1;
        zchunk = ceil_div(L, nzc);
        if (zchunk < 16) zchunk = 16;
    }
    if (zchunk > L) zchunk = L;
    const int blocks = nseg * ntile_y * ceil_div(L, zchunk);
#define CFD_TB2(WV)                                                                             \
    case WV:                                                                                    \
        if (pre)                                                                                \
            hipLaunchKernelGGL((jacobi3d_tb2<WV, true>), dim3(blocks), dim3((WV + 2) * 64), 0, s, in, \
                               out, div, nz, ny, nx, nseg, ntile_y, zb, ze, zchunk, fixed_lo,      \
                               fixed_hi, h2, dt);                                               \
        else                                                                                    \
            hipLaunchKernelGGL((jacobi3d_tb2<WV, false>), dim3(blocks), dim3((WV + 2) * 64), 0, s, in, \
                               out, div, nz, ny, nx, nseg, ntile_y, zb, ze, zchunk, fixed_lo,      \
                               fixed_hi, h2, dt);                                               \
        break;
    switch (W) {
        CFD_TB2(2)
        CFD_TB2(6)
        CFD_TB2(14)
        default:
            set_error("jacobi3d_tb2: unsupported rows per tile %d (2, 6, 14)", W);
            return CFD_E_INVALID;
    }
#undef CFD_TB2
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // namespace cfd
