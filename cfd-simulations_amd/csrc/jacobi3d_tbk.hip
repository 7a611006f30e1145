// jacobi3d_tbk.hip -- K Jacobi sweeps per HBM pass (K = 2, 3, 4), 7-point, fp32.
//
// The generalisation of jacobi3d_tb2 (jacobi3d_tb.hip) to K levels: one pass
// reads phi^k and the rhs once and writes phi^(k+K).  At 12 B of algorithmic
// traffic per cell and pass, K = 3 / 4 cost 4 / 3 B per cell-update, against
// 6 B for two levels.  The price is a deeper halo: a tile of W output rows
// loads W + 2K rows of phi^k (its neighbours' rows are re-read, mostly from
// HBM: the L2 seldom still holds them).
//
// Workgroup = one 256-column x-segment x W rows, marching a z-chunk; W + 2K - 1
// waves (16 for the shipped shapes: K=2 W=13, K=3 W=11, K=4 W=9):
//  * row waves g = 0 .. W+2K-3 own tile row r = g + 1 (y = y0 - K + r) and
//    compute level l (1..K) of their row when l <= r < W+2K-l;
//  * the halo wave loads the two outermost rows (r = 0, W+2K-1) and, one lane
//    per (row, side), the 4-float x-halo chunks of all W+2K rows, and computes
//    levels 1..K-1 of those chunks (a chunk of 4 columns covers the K-l halo
//    columns level l needs, for K <= 4).
// Per z-step (front plane z):
//    level 0 of plane z -> LDS tile T_0;  barrier;
//    for l = 1..K: level l of plane p = z-l+1 from T_(l-1)[p&1] (y), the
//    level-(l-1) register queue (z) and lane shuffles (x); into T_l[p&1] and
//    the level-l queue, or (l = K) to HBM.
// T_l[p&1] written at step p+l-1 is read at step p+l only, and overwritten at
// step p+l+1: one barrier per step suffices.  Every level is computed with the
// unfused sweep's operation order, so the result is bit-identical to K single
// sweeps.  Cells outside the domain and eroded halo cells hold garbage that
// never reaches a valid cell: Dirichlet planes/rows/columns are copied through
// at every level (tests/test_gpu_parity.py).
#include "internal.hpp"

namespace cfd {

namespace {

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

struct TbkArgs {
    const float *in;
    float *out;
    const float *div;  // div, or the precomputed rhs (PRE)
    int nz, ny, nx, nseg, ntile_y, zb, ze, zchunk, fixed_lo, fixed_hi;
    float h2, dt;
};

template <bool PRE>
__device__ inline float jac7(float E, float W, float N, float S, float U, float D, float d,
                             float h2, float dt) {
    float s = E + W;
    s = s + N;
    s = s + S;
    s = s + U;
    s = s + D;
    const float rhs = PRE ? d : (h2 * d) / dt;
    return (1.0f / 6.0f) * (s - rhs);
}

// one level on a float4 of cells x .. x+3; `upd` = row and plane are updated
template <bool PRE>
__device__ inline float4 level4(float4 c, float wl, float er, float4 N, float4 S, float4 U,
                                float4 D, float4 d, int x, int nx, bool upd, float h2, float dt) {
    if (!upd) return c;
    const float cv[4] = {c.x, c.y, c.z, c.w};
    const float nv[4] = {N.x, N.y, N.z, N.w};
    const float sv[4] = {S.x, S.y, S.z, S.w};
    const float uv[4] = {U.x, U.y, U.z, U.w};
    const float dv[4] = {D.x, D.y, D.z, D.w};
    const float rv[4] = {d.x, d.y, d.z, d.w};
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float E = k < 3 ? cv[k + 1] : er;
        const float Wv = k > 0 ? cv[k - 1] : wl;
        const int xk = x + k;
        o[k] = (xk != 0 && xk != nx - 1) ? jac7<PRE>(E, Wv, nv[k], sv[k], uv[k], dv[k], rv[k], h2, dt)
                                         : cv[k];
    }
    return make_float4(o[0], o[1], o[2], o[3]);
}

}  // namespace

// PD: planes of prefetch (loads for step z + PD are issued at step z)
template <int K, int W, bool PRE, int PD>
__global__ __launch_bounds__((W + 2 * K - 1) * 64) void jacobi3d_tbk(TbkArgs a) {
    constexpr int NR = W + 2 * K;  // level-0 rows per tile
    constexpr int RS = 264;        // LDS row: 4 halo | 256 | 4 halo floats
    constexpr int NRW = NR - 2;    // row waves
    static_assert(K >= 2 && K <= 4, "a 4-float halo chunk covers K <= 4 levels");
    static_assert(2 * NR <= 64, "halo wave: one lane per (row, side)");
    // level l keeps rows [l, NR - l), double-buffered by plane parity
    constexpr int TOTAL = [] {
        int t = 0;
        for (int l = 0; l < K; ++l) t += 2 * (NR - 2 * l) * RS;
        return t;
    }();
    __shared__ __attribute__((aligned(16))) float smem[TOTAL];
    auto T = [&](int l, int b, int r) -> float * {
        int base = 0;
#pragma unroll
        for (int m = 0; m < K; ++m)
            if (m < l) base += 2 * (NR - 2 * m) * RS;
        return smem + base + (b * (NR - 2 * l) + (r - l)) * RS;
    };

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
    const int zs = z0 - K + 1;       // first front plane
    const int zl = z1 + K - 2;       // last front plane
    const float h2 = a.h2, dt = a.dt;
    auto P = [&](int p) { return a.in + (size_t)p * plane; };
    auto R = [&](int p) { return a.div + (size_t)p * plane; };
    auto fixedp = [&](int p) { return (p == a.zb - 1 && a.fixed_lo) || (p == a.ze && a.fixed_hi); };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);

    if (wv < NRW) {
        // ------------------------------------------------------------ row wave
        const int r = wv + 1;
        const int y = y0 - K + r;
        const bool rowin = y >= 0 && y <= ny - 1;
        const bool ld = xin && rowin;
        const bool int_row = y >= 1 && y <= ny - 2;
        const bool out_row = r >= K && r < NR - K && y <= ny - 2;
        const size_t rofs = (size_t)(rowin ? y : 0) * nx + (xin ? x : 0);
        auto ldp = [&](int p) { return ldg4_if(ld && p >= 0 && p <= nz - 1, P(p) + rofs); };
        auto ldr = [&](int p) { return ldg4_if(ld && p >= 0 && p <= nz - 1, R(p) + rofs); };
        float4 Q[K][3];   // Q[l][j] = level l of plane (z - l) - 1 + j, for the level-(l+1) update
        float4 Rq[K];     // Rq[j] = rhs of plane z - j
#pragma unroll
        for (int l = 0; l < K; ++l) Q[l][0] = Q[l][1] = Q[l][2] = z4;
        Q[0][0] = ldp(zs - 1);
        Q[0][1] = ldp(zs);
        Q[0][2] = ldp(zs + 1);
#pragma unroll
        for (int j = 0; j < K; ++j) Rq[j] = ldr(zs - j);
        float4 Cq[PD], Rn[PD];  // in flight: level 0 of planes z+2.., rhs of planes z+1..
#pragma unroll
        for (int j = 0; j + 1 < PD; ++j) {
            Cq[j] = ldp(zs + 2 + j);
            Rn[j] = ldr(zs + 1 + j);
        }
        for (int z = zs; z <= zl; ++z) {
            Cq[PD - 1] = ldp(z + 1 + PD);
            Rn[PD - 1] = ldr(z + PD);
            const int b = z & 1;
            if (ld) sts4(T(0, b, r) + 4 + 4 * lane, Q[0][1]);
            __syncthreads();
#pragma unroll
            for (int l = 1; l <= K; ++l) {
                const int p = z - l + 1;
                const int pb = p & 1;
                if (r >= l && r < NR - l) {
                    const float4 c = Q[l - 1][1];
                    float wl = __shfl_up(c.w, 1, 64);
                    float er = __shfl_down(c.x, 1, 64);
                    const float *row = T(l - 1, pb, r);
                    const float wl_l = row[3], er_l = row[260];
                    if (lane == 0) wl = wl_l;
                    if (lane == 63) er = er_l;
                    float4 v = c;
                    if (xin) {
                        const float4 N = lds4(T(l - 1, pb, r + 1) + 4 + 4 * lane);
                        const float4 S = lds4(T(l - 1, pb, r - 1) + 4 + 4 * lane);
                        v = level4<PRE>(c, wl, er, N, S, Q[l - 1][2], Q[l - 1][0], Rq[l - 1], x, nx,
                                        int_row && !fixedp(p), h2, dt);
                    }
                    if (l < K) {
                        if (xin) sts4(T(l, pb, r) + 4 + 4 * lane, v);
                        Q[l][0] = Q[l][1];
                        Q[l][1] = Q[l][2];
                        Q[l][2] = v;
                    } else if (out_row && xin && p >= z0 && p < z1) {
                        stg4(a.out + (size_t)p * plane + rofs, v);
                    }
                }
            }
            Q[0][0] = Q[0][1];
            Q[0][1] = Q[0][2];
            Q[0][2] = Cq[0];
#pragma unroll
            for (int j = K - 1; j > 0; --j) Rq[j] = Rq[j - 1];
            Rq[0] = Rn[0];
#pragma unroll
            for (int j = 0; j + 1 < PD; ++j) {
                Cq[j] = Cq[j + 1];
                Rn[j] = Rn[j + 1];
            }
        }
    } else {
        // ------------------------------------------------------------ halo wave
        const int ylo = y0 - K, yhi = y0 - K + NR - 1;
        const bool elo = xin && ylo >= 0 && ylo <= ny - 1;
        const bool ehi = xin && yhi >= 0 && yhi <= ny - 1;
        const size_t olo = (size_t)(elo ? ylo : 0) * nx + (xin ? x : 0);
        const size_t ohi = (size_t)(ehi ? yhi : 0) * nx + (xin ? x : 0);
        // halo chunks: lane -> tile row hr, side (0: x0-4..x0-1, 1: x0+256..x0+259)
        const int hr = lane >> 1, side = lane & 1;
        const int yr = y0 - K + hr;
        const bool hon = lane < 2 * NR && yr >= 0 && yr <= ny - 1 &&
                         (side ? xs + 256 < nx : xs > 0);
        const bool hint = hon && yr >= 1 && yr <= ny - 2;
        const int hx = side ? xs + 256 : xs - 4;
        const size_t hofs = (size_t)(hon ? yr : 0) * nx + (hon ? hx : 0);
        const int col = side ? 260 : 0;  // chunk position in an LDS row
        auto ldh = [&](const float *base, int p) {
            return ldg4_if(hon && p >= 0 && p <= nz - 1, base + (size_t)p * plane + hofs);
        };
        auto ldlo = [&](int p) { return ldg4_if(elo && p >= 0 && p <= nz - 1, P(p) + olo); };
        auto ldhi = [&](int p) { return ldg4_if(ehi && p >= 0 && p <= nz - 1, P(p) + ohi); };
        float4 lo = ldlo(zs), hi = ldhi(zs);
        float4 H[K][3];
        float4 Hr[K];
#pragma unroll
        for (int l = 0; l < K; ++l) H[l][0] = H[l][1] = H[l][2] = z4;
        H[0][0] = ldh(a.in, zs - 1);
        H[0][1] = ldh(a.in, zs);
        H[0][2] = ldh(a.in, zs + 1);
#pragma unroll
        for (int j = 0; j < K; ++j) Hr[j] = ldh(a.div, zs - j);
        // in flight: rows 0 / NR-1 of planes z+1.., chunks of z+2.., rhs chunks of z+1..
        float4 Lq[PD], Uq[PD], Hq[PD], Rn[PD];
#pragma unroll
        for (int j = 0; j + 1 < PD; ++j) {
            Lq[j] = ldlo(zs + 1 + j);
            Uq[j] = ldhi(zs + 1 + j);
            Hq[j] = ldh(a.in, zs + 2 + j);
            Rn[j] = ldh(a.div, zs + 1 + j);
        }
        for (int z = zs; z <= zl; ++z) {
            Lq[PD - 1] = ldlo(z + PD);
            Uq[PD - 1] = ldhi(z + PD);
            Hq[PD - 1] = ldh(a.in, z + 1 + PD);
            Rn[PD - 1] = ldh(a.div, z + PD);
            const int b = z & 1;
            if (elo) sts4(T(0, b, 0) + 4 + 4 * lane, lo);
            if (ehi) sts4(T(0, b, NR - 1) + 4 + 4 * lane, hi);
            if (hon) sts4(T(0, b, hr) + col, H[0][1]);
            __syncthreads();
#pragma unroll
            for (int l = 1; l < K; ++l) {
                const int p = z - l + 1;
                const int pb = p & 1;
                if (lane < 2 * NR && hr >= l && hr < NR - l) {
                    const float4 c = H[l - 1][1];
                    // the tile column next to the chunk; the far side is eroded
                    const float inner = T(l - 1, pb, hr)[side ? 259 : 4];
                    float4 v = c;
                    if (hon) {
                        const float4 N = lds4(T(l - 1, pb, hr + 1) + col);
                        const float4 S = lds4(T(l - 1, pb, hr - 1) + col);
                        v = level4<PRE>(c, side ? inner : 0.f, side ? 0.f : inner, N, S, H[l - 1][2],
                                        H[l - 1][0], Hr[l - 1], hx, nx, hint && !fixedp(p), h2, dt);
                        sts4(T(l, pb, hr) + col, v);
                    }
                    H[l][0] = H[l][1];
                    H[l][1] = H[l][2];
                    H[l][2] = v;
                }
            }
            lo = Lq[0];
            hi = Uq[0];
            H[0][0] = H[0][1];
            H[0][1] = H[0][2];
            H[0][2] = Hq[0];
#pragma unroll
            for (int j = K - 1; j > 0; --j) Hr[j] = Hr[j - 1];
            Hr[0] = Rn[0];
#pragma unroll
            for (int j = 0; j + 1 < PD; ++j) {
                Lq[j] = Lq[j + 1];
                Uq[j] = Uq[j + 1];
                Hq[j] = Hq[j + 1];
                Rn[j] = Rn[j + 1];
            }
        }
    }
}

// One K-level pass over planes [zb, ze) of `out`.  Needs K readable planes on
// each non-fixed side (slab ghosts), one on a fixed side.
int jacobi3d_tbk_pass(int K, const float *in, float *out, const float *div, int nz, int ny, int nx,
                      int zb, int ze, int fixed_lo, int fixed_hi, float h2, float dt, int zchunk,
                      bool pre, hipStream_t s) {
    if (ze <= zb || ny < 3) return CFD_OK;
    TbkArgs a{};
    a.in = in; a.out = out; a.div = div;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze;
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi; a.h2 = h2; a.dt = dt;
    const int pd = jacobi3d_tb_prefetch();
    const int W = K == 2 ? 13 : K == 3 ? 11 : 9;
    a.nseg = ceil_div(nx, 256);
    a.ntile_y = ceil_div(ny - 2, W);
    const int L = ze - zb;
    if (zchunk <= 0) {
        const long tiles = (long)a.nseg * a.ntile_y;
        int nzc = (int)((1024 + tiles - 1) / tiles);
        if (nzc < 1) nzc = 1;
        zchunk = ceil_div(L, nzc);
        // each chunk re-marches 2K-2 planes: longer chunks for more levels
        if (zchunk > 256) zchunk = 256;
        if (zchunk < 16) zchunk = 16;
    }
    if (zchunk > L) zchunk = L;
    a.zchunk = zchunk;
    const int blocks = a.nseg * a.ntile_y * ceil_div(L, zchunk);
#define CFD_TBK_L(KV, WV, PR, PDV) \
    hipLaunchKernelGGL((jacobi3d_tbk<KV, WV, PR, PDV>), dim3(blocks), dim3((WV + 2 * KV - 1) * 64), 0, s, a)
#define CFD_TBK(KV, WV)                                                            \
    do {                                                                           \
        if (pd == 2) {                                                             \
            if (pre) CFD_TBK_L(KV, WV, true, 2); else CFD_TBK_L(KV, WV, false, 2); \
        } else {                                                                   \
            if (pre) CFD_TBK_L(KV, WV, true, 1); else CFD_TBK_L(KV, WV, false, 1); \
        }                                                                          \
    } while (0)
    switch (K) {
        case 2: CFD_TBK(2, 13); break;
        case 3: CFD_TBK(3, 11); break;
        case 4: CFD_TBK(4, 9); break;
        default:
            set_error("jacobi3d_tbk: unsupported levels per pass %d (2..4)", K);
            return CFD_E_INVALID;
    }
#undef CFD_TBK
#undef CFD_TBK_L
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // namespace cfd
