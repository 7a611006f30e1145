// poisson3d.hip -- 3-D 7-point pressure-Poisson kernels for gfx950.
//
// The reference is 2-D only; the 3-D path generalises its Jacobi template
// (v5.py:336-346) to 7 points:
//     phi_new = f32(1/6) * (((((E+W)+N)+S)+U)+D - f32(h*h)*div/dt)
// and its red-black Gauss-Seidel (v5.py:202-226) to (z+i+j) parity colours.
//
// Jacobi sweep design ("2.5-D z-march"; HBM-bound, 12 B per cell-update):
//  * a workgroup owns an x-segment of 256 cells (64 lanes x float4) by W rows
//    (one wave per row) and marches a chunk of z-planes;
//  * z-neighbours live in a 3-plane register queue (the plane after next is
//    prefetched one step ahead), so each phi value is read from HBM once;
//  * y-neighbours: variant LDS stages the current plane's W rows plus two halo
//    rows in a double-buffered LDS tile (one barrier per plane); variant CACHE
//    loads them straight from global (they are the rows the neighbouring
//    waves just fetched: L1/L2 hits);
//  * x-neighbours come from the adjacent lane by cross-lane shuffle; lanes 0
//    and 63 fetch one scalar each per row;
//  * the RHS (h^2*div)/dt is recomputed in-register from div (4 B either way);
//  * the workgroup -> tile map is XCD-aware: each XCD gets a contiguous run of
//    y-tiles so the halo rows two tiles share stay in that XCD's L2.
#include "internal.hpp"

namespace cfd {

// Dirichlet faces the sweep never writes, planes [za, zb) of an (nz, ny, nx)
// array: every cell of the planes full_lo / full_hi, rows y = 0 and ny-1 of
// the others (x faces are copied through by the sweep itself):
//     dst = mask ? 0 : src        (phi_new[mask] = 0 hits faces too)
// Before sweep 1 this builds the output buffer's faces (sweep 1 still reads
// the unmasked input faces, like the reference); after sweep 1 it copies them
// back so both ping-pong buffers hold the final faces.
__global__ void fix_faces3d(const float *__restrict__ src, float *__restrict__ dst,
                            const uint8_t *__restrict__ mask, int ny, int nx, int za, int zb,
                            int full_lo, int full_hi) {
    const size_t plane = (size_t)ny * nx;
    for (int z = za + blockIdx.y; z < zb; z += gridDim.y) {
        const bool full = z == full_lo || z == full_hi;
        const size_t n = full ? plane : 2 * (size_t)nx;
        for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
             k += (size_t)gridDim.x * blockDim.x) {
            size_t c;
            if (full) c = (size_t)z * plane + k;
            else c = (size_t)z * plane + (k < (size_t)nx ? k : (size_t)(ny - 1) * nx + (k - nx));
            float v = src ? src[c] : 0.f;  // src NULL: zero the faces
            if (mask && mask[c]) v = 0.f;
            dst[c] = v;
        }
    }
}

int launch_fix_faces3d(const float *src, float *dst, const uint8_t *mask, int ny, int nx, int za,
                       int zb, int full_lo, int full_hi, hipStream_t s) {
    if (zb <= za) return CFD_OK;
    int gy = zb - za;
    if (gy > 1024) gy = 1024;
    hipLaunchKernelGGL(fix_faces3d, dim3(16, gy), dim3(256), 0, s, src, dst, mask, ny, nx, za, zb,
                       full_lo, full_hi);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// Zero the Dirichlet faces the blocked passes never write (planes 0 and nz-1,
// rows 0 and ny-1 of every plane) in both arrays of the ping-pong pair: the
// boundary of phi = zeros (v5.py:337) for a solve that starts from zero.
// This kernel does rows 0 and ny-1 of planes 1 .. nz-2 (grid-stride in y);
// the two full planes are memsets.  float4: nx % 4 == 0, aligned arrays.
__global__ void zero_rows3d(float *__restrict__ a, float *__restrict__ b, int nz, int ny, int nx) {
    const size_t plane = (size_t)ny * nx;
    const size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (4 * k >= 2 * (size_t)nx) return;
    const size_t r = 4 * k < (size_t)nx ? 4 * k : (size_t)(ny - 2) * nx + 4 * k;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t z = blockIdx.y + 1; z + 1 < (size_t)nz; z += gridDim.y) {
        *reinterpret_cast<float4 *>(a + z * plane + r) = z4;
        *reinterpret_cast<float4 *>(b + z * plane + r) = z4;
    }
}

int launch_zero_faces3d(float *a, float *b, int nz, int ny, int nx, hipStream_t s) {
    const size_t plane = (size_t)ny * nx;
    for (float *p : {a, b}) {
        CFD_CHECK_HIP(hipMemsetAsync(p, 0, plane * sizeof(float), s));
        CFD_CHECK_HIP(hipMemsetAsync(p + (size_t)(nz - 1) * plane, 0, plane * sizeof(float), s));
    }
    if (nz > 2) {
        hipLaunchKernelGGL(zero_rows3d, dim3(ceil_div(2 * nx / 4, 256), nz - 2 < 4096 ? nz - 2 : 4096),
                           dim3(256), 0, s, a, b, nz, ny, nx);
        CFD_LAUNCH_CHECK();
    }
    return CFD_OK;
}

// Jacobi sweeps per pass when tb_steps == 0 (r01 sweep at 1024^3: K=2 855,
// K=3 1010-1030, K=4 1000 Gcell/s; r03, nt stores and the packed K = 4
// level, three runs each on one box: 1024^3 K=3 1462-1466 / K=4 1490-1494,
// 512^3 1380-1385 / 1435-1443, channel 1450-1465 / 1490-1492)
constexpr int kDefaultLevels = 4;

// planes per tile of the blocked kernels (0 = the launcher's cost model)
int jacobi3d_tb_zchunk() { return tuning().tb_zchunk; }
bool jacobi3d_tb_enabled() { return tuning().tb_steps != 1; }
int jacobi3d_tb_levels() { return tuning().tb_steps >= 2 ? tuning().tb_steps : kDefaultLevels; }
bool rbgs3d_fused_ok(const float *phi, const float *phi_tmp, const float *div, const uint8_t *mask,
                     int nx) {
    return phi_tmp && jacobi3d_tb_enabled() && !mask && nx % 4 == 0 && aligned16(phi) &&
           aligned16(phi_tmp) && aligned16(div);
}
int jacobi3d_tb_prefetch() { return tuning().tb_prefetch == 2 ? 2 : 1; }

__device__ inline float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ inline void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// PRE: `div` holds the precomputed rhs = (h2*div)/dt (cfd_rhs prologue);
// otherwise the rhs is formed in-register (same bits, one fp32 division).
template <int W, bool USE_LDS, bool RESID, bool MASK, bool PRE>
__global__ __launch_bounds__(W * 64) void jacobi3d_march(
    const float *__restrict__ in, float *__restrict__ out, const float *__restrict__ div,
    const uint8_t *__restrict__ mask, int ny, int nx, int nseg, int ntile_y, int zb, int ze,
    int zchunk, float h2, float dt, float *__restrict__ resid) {
    __shared__ float4 lds[USE_LDS ? 2 : 1][USE_LDS ? W + 2 : 1][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    // logical tile: seg fastest, then y-tile, then z-chunk; XCD-contiguous runs
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = t % nseg;
    const int ty = (t / nseg) % ntile_y;
    const int zc = t / (nseg * ntile_y);
    const int z0 = zb + zc * zchunk;
    if (z0 >= ze) return;  // workgroup-uniform
    const int z1 = min(z0 + zchunk, ze);
    const int y = 1 + ty * W + w;
    const int x0 = (seg * 64 + lane) * 4;
    const bool xin = x0 < nx;
    const bool ok = y < ny - 1 && xin;      // this lane updates cells
    const bool live = y <= ny - 1 && xin;   // this lane's row is read by a neighbour (LDS)
    const bool has_left = ok && lane == 0 && x0 > 0;
    const bool has_right = ok && lane == 63 && x0 + 4 < nx;
    const size_t plane = (size_t)ny * nx;
    const size_t rofs = (size_t)y * nx + x0;
    // LDS halo rows: row y-1 for wave 0, row y+1 for the last wave
    const bool lo_ok = USE_LDS && w == 0 && xin && y <= ny - 1;
    const bool hi_ok = USE_LDS && w == W - 1 && xin && y + 1 <= ny - 1;

    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 dn = zero4, cur = zero4, up = zero4, up2 = zero4;
    float4 nn = zero4, ss = zero4, nn_next = zero4, ss_next = zero4;  // CACHE variant
    float4 hlo = zero4, hhi = zero4, hlo_next = zero4, hhi_next = zero4;  // LDS variant
    float cl = 0.f, cr = 0.f, nl = 0.f, nr = 0.f;

    const float *pz = in + (size_t)z0 * plane;
    if (ok) {
        dn = ld4(pz - plane + rofs);
        if (!USE_LDS) {
            nn = ld4(pz + rofs + nx);
            ss = ld4(pz + rofs - nx);
        }
    }
    if (ok || (USE_LDS && live)) {
        cur = ld4(pz + rofs);
        up = ld4(pz + plane + rofs);
    }
    if (lo_ok) hlo = ld4(pz + rofs - nx);
    if (hi_ok) hhi = ld4(pz + rofs + nx);
    if (has_left) cl = pz[rofs - 1];
    if (has_right) cr = pz[rofs + 4];
    float rmax = 0.f;
    const float sixth = 1.0f / 6.0f;

    for (int z = z0; z < z1; ++z) {
        const float *p = in + (size_t)z * plane;
        const bool more = z + 1 < z1;
        // prefetch for plane z+1: its upper neighbour (z+2), y-rows, x-edges
        if (more) {
            if (ok) {
                up2 = ld4(p + 2 * plane + rofs);
                if (!USE_LDS) {
                    nn_next = ld4(p + plane + rofs + nx);
                    ss_next = ld4(p + plane + rofs - nx);
                }
            } else if (USE_LDS && live) {
                up2 = ld4(p + 2 * plane + rofs);  // boundary row: feeds a neighbour only
            }
            if (lo_ok) hlo_next = ld4(p + plane + rofs - nx);
            if (hi_ok) hhi_next = ld4(p + plane + rofs + nx);
            if (has_left) nl = p[plane + rofs - 1];
            if (has_right) nr = p[plane + rofs + 4];
        }
        float4 d = zero4;
        uchar4 m = make_uchar4(0, 0, 0, 0);
        if (ok) {
            d = ld4(div + (size_t)z * plane + rofs);
            if (MASK) m = *reinterpret_cast<const uchar4 *>(mask + (size_t)z * plane + rofs);
        }
        if constexpr (USE_LDS) {
            const int buf = z & 1;
            lds[buf][w + 1][lane] = cur;
            if (w == 0) lds[buf][0][lane] = hlo;
            if (w == W - 1) lds[buf][W + 1][lane] = hhi;
            __syncthreads();
            nn = lds[buf][w + 2][lane];
            ss = lds[buf][w][lane];
        }
        float wl = __shfl_up(cur.w, 1, 64);
        float er = __shfl_down(cur.x, 1, 64);
        if (lane == 0) wl = cl;
        if (lane == 63) er = cr;
        const float c[4] = {cur.x, cur.y, cur.z, cur.w};
        const float N[4] = {nn.x, nn.y, nn.z, nn.w};
        const float S[4] = {ss.x, ss.y, ss.z, ss.w};
        const float U[4] = {up.x, up.y, up.z, up.w};
        const float D[4] = {dn.x, dn.y, dn.z, dn.w};
        const float dv[4] = {d.x, d.y, d.z, d.w};
        const unsigned char mk[4] = {m.x, m.y, m.z, m.w};
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float E = k < 3 ? c[k + 1] : er;
            const float Wv = k > 0 ? c[k - 1] : wl;
            const int x = x0 + k;
            float val;
            if (x == 0 || x >= nx - 1) {
                val = c[k];
            } else {
                float s = E + Wv;
                s = s + N[k];
                s = s + S[k];
                s = s + U[k];
                s = s + D[k];
                val = sixth * (s - (PRE ? dv[k] : (h2 * dv[k]) / dt));
            }
            if (MASK && mk[k]) val = 0.f;
            o[k] = val;
            if (RESID && ok) {  // only cells this lane owns
                const float ch = fabsf(val - c[k]);
                if (ch > rmax) rmax = ch;
            }
        }
        if (ok) st4(out + (size_t)z * plane + rofs, make_float4(o[0], o[1], o[2], o[3]));
        dn = cur;
        cur = up;
        up = up2;
        if (!USE_LDS) {
            nn = nn_next;
            ss = ss_next;
        }
        hlo = hlo_next;
        hhi = hhi_next;
        cl = nl;
        cr = nr;
    }
    if (RESID) wave_reduce_max_store(rmax, resid);
}

// Scalar fallback for nx % 4 != 0 or unaligned arrays (small parity cases):
// one thread per cell, all 7 neighbours from global.
template <bool MASK>
__global__ __launch_bounds__(256) void jacobi3d_scalar(const float *__restrict__ in,
                                                       float *__restrict__ out,
                                                       const float *__restrict__ div,
                                                       const uint8_t *__restrict__ mask, int ny,
                                                       int nx, int zb, float h2, float dt, int pre,
                                                       float *__restrict__ resid) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y + 1;
    const int z = blockIdx.z + zb;
    float ch = 0.f;
    if (x < nx) {
        const size_t plane = (size_t)ny * nx;
        const size_t c = (size_t)z * plane + (size_t)y * nx + x;
        float val;
        if (x == 0 || x == nx - 1) {
            val = in[c];
        } else {
            float s = in[c + 1] + in[c - 1];
            s = s + in[c + nx];
            s = s + in[c - nx];
            s = s + in[c + plane];
            s = s + in[c - plane];
            val = (1.0f / 6.0f) * (s - (pre ? div[c] : (h2 * div[c]) / dt));
        }
        if (MASK && mask[c]) val = 0.f;
        out[c] = val;
        ch = fabsf(val - in[c]);
        if (!(ch > 0.f)) ch = 0.f;
    }
    if (resid) wave_reduce_max_store(ch, resid);
}

template <int W, bool USE_LDS, bool PRE>
static void launch_march(const float *in, float *out, const float *div, const uint8_t *mask,
                         int ny, int nx, int zb, int ze, int zchunk, float h2, float dt,
                         float *resid, hipStream_t s) {
    const int nseg = ceil_div(nx, 256);
    const int ntile_y = ceil_div(ny - 2, W);
    const int nzc = ceil_div(ze - zb, zchunk);
    const int blocks = nseg * ntile_y * nzc;
#define CFD_J3_LAUNCH(R, M)                                                                    \
    hipLaunchKernelGGL((jacobi3d_march<W, USE_LDS, R, M, PRE>), dim3(blocks), dim3(W * 64), 0, s, \
                       in, out, div, mask, ny, nx, nseg, ntile_y, zb, ze, zchunk, h2, dt, resid)
    if (resid) {
        if (mask) CFD_J3_LAUNCH(true, true); else CFD_J3_LAUNCH(true, false);
    } else {
        if (mask) CFD_J3_LAUNCH(false, true); else CFD_J3_LAUNCH(false, false);
    }
#undef CFD_J3_LAUNCH
}

// Sweep planes [zb, ze) of in -> out (local array of nz planes).  pre: `div`
// is the precomputed rhs (launch_rhs), else the divergence.
int jacobi3d_sweep(const float *in, float *out, const float *div, const uint8_t *mask, int nz,
                   int ny, int nx, int zb, int ze, float h2, float dt, bool pre, float *resid,
                   hipStream_t s) {
    if (ze <= zb || ny < 3) return CFD_OK;
    CFD_REQUIRE(zb >= 1 && ze <= nz - 1, "jacobi3d sweep: z range [%d,%d) outside 1..%d", zb, ze,
                nz - 1);
    const bool vec_ok = nx % 4 == 0 && aligned16(in) && aligned16(out) && aligned16(div) &&
                        (!mask || (reinterpret_cast<uintptr_t>(mask) & 3u) == 0);
    if (!vec_ok) {
        dim3 grid(ceil_div(nx, 256), ny - 2, ze - zb);
        if (mask)
            hipLaunchKernelGGL(jacobi3d_scalar<true>, grid, dim3(256), 0, s, in, out, div, mask, ny,
                               nx, zb, h2, dt, (int)pre, resid);
        else
            hipLaunchKernelGGL(jacobi3d_scalar<false>, grid, dim3(256), 0, s, in, out, div, mask,
                               ny, nx, zb, h2, dt, (int)pre, resid);
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    // defaults from the r01 tile sweep (1024^3): LDS tile, 16 rows, 64 planes
    int variant = tuning().j3_variant ? tuning().j3_variant : 1;
    int W = tuning().j3_waves ? tuning().j3_waves : 16;
    const int nseg = ceil_div(nx, 256);
    const int L = ze - zb;
    int zchunk = tuning().j3_zchunk;
    if (zchunk <= 0) {
        // >= ~1024 workgroups when the grid allows, 64 planes per march otherwise
        const long tiles = (long)nseg * ceil_div(ny - 2, W);
        int nzc = (int)((1024 + tiles - 1) / tiles);
        if (nzc < 1) nzc = 1;
        zchunk = ceil_div(L, nzc);
        if (zchunk > 64) zchunk = 64;
        if (zchunk < 16) zchunk = 16;
    }
    if (zchunk > L) zchunk = L;
#define CFD_J3_W(WV)                                                                                 \
    case WV:                                                                                         \
        if (variant == 2) {                                                                          \
            if (pre) launch_march<WV, false, true>(in, out, div, mask, ny, nx, zb, ze, zchunk, h2, dt, resid, s); \
            else launch_march<WV, false, false>(in, out, div, mask, ny, nx, zb, ze, zchunk, h2, dt, resid, s); \
        } else {                                                                                     \
            if (pre) launch_march<WV, true, true>(in, out, div, mask, ny, nx, zb, ze, zchunk, h2, dt, resid, s); \
            else launch_march<WV, true, false>(in, out, div, mask, ny, nx, zb, ze, zchunk, h2, dt, resid, s); \
        }                                                                                            \
        break;
    switch (W) {
        CFD_J3_W(1)
        CFD_J3_W(2)
        CFD_J3_W(4)
        CFD_J3_W(8)
        CFD_J3_W(16)
        default:
            set_error("jacobi3d: unsupported waves-per-workgroup %d", W);
            return CFD_E_INVALID;
    }
#undef CFD_J3_W
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// rhs = (f32(h*h) * div) / dt over n cells (the Poisson RHS prologue; the
// same bits the sweep kernels form in-register when no workspace is given).
__global__ void k_rhs_f32(const float *__restrict__ div, float *__restrict__ rhs, size_t n4,
                          size_t n, float h2, float dt) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n4; k += stride) {
        float4 d = reinterpret_cast<const float4 *>(div)[k];
        d.x = (h2 * d.x) / dt;
        d.y = (h2 * d.y) / dt;
        d.z = (h2 * d.z) / dt;
        d.w = (h2 * d.w) / dt;
        reinterpret_cast<float4 *>(rhs)[k] = d;
    }
    for (size_t k = 4 * n4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n; k += stride)
        rhs[k] = (h2 * div[k]) / dt;
}

int launch_rhs_f32(const float *div, float *rhs, size_t n, float h2, float dt, hipStream_t s) {
    const size_t n4 = (aligned16(div) && aligned16(rhs)) ? n / 4 : 0;
    long blocks = (long)((n / 4 + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_rhs_f32, dim3(blocks), dim3(256), 0, s, div, rhs, n4, n, h2, dt);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// ----------------------------------------------------------- red-black GS 3-D
// In-place colour pass over planes [z0, z0 + gridDim.z) of a local array whose
// plane 0 is global plane zoff (colour parity is global, so a slab's cells get
// the colours they have in the whole grid).  The fused out-of-place pass is
// jacobi3d_tb2<.., MODE_RBGS, ..> (jacobi3d_tb.hip); this one serves masks.
template <int C>
__global__ __launch_bounds__(256) void rbgs3d_color(float *__restrict__ phi,
                                                    const float *__restrict__ div,
                                                    const uint8_t *__restrict__ mask, int ny,
                                                    int nx, int z0, int zoff, float cx, float cy,
                                                    float cz, float cd, float dt_inv, float tol,
                                                    RbgsWs *ws, int it) {
    if (it > 0 && ws->maxc[it - 1] < tol) {
        if (C == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
            atomicMin(&ws->flags[1], it);
        return;
    }
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y + 1;
    const int z = z0 + blockIdx.z;
    float mx = 0.f;
    // colour c: (zg + i + j + 1 + c) even
    if (x < nx - 1 && x >= 1 && ((zoff + z + i + x + 1 + C) & 1) == 0) {
        const size_t plane = (size_t)ny * nx;
        const size_t c = (size_t)z * plane + (size_t)i * nx + x;
        if (!(mask && mask[c])) {
            const float rhs = -div[c] * dt_inv;
            const float a = cx * (phi[c + 1] + phi[c - 1]);
            const float b = cy * (phi[c + nx] + phi[c - nx]);
            const float e = cz * (phi[c + plane] + phi[c - plane]);
            const float pn = (((a + b) + e) - rhs) * cd;
            const float ch = fabsf(pn - phi[c]);
            if (ch > mx) mx = ch;
            phi[c] = pn;
        }
    }
    wave_reduce_max_store(mx, &ws->maxc[it]);
}

int rbgs3d_colour_pass(int colour, float *phi, const float *div, const uint8_t *mask, int ny,
                       int nx, int z0, int z1, int zoff, const RbgsConsts &k, RbgsWs *ws, int it,
                       hipStream_t s) {
    if (z1 <= z0 || ny < 3 || nx < 3) return CFD_OK;
    dim3 grid(ceil_div(nx, 256), ny - 2, z1 - z0);
    if (colour == 0)
        hipLaunchKernelGGL(rbgs3d_color<0>, grid, dim3(256), 0, s, phi, div, mask, ny, nx, z0, zoff,
                           k.cx, k.cy, k.cz, k.cd, k.dt_inv, k.tol, ws, it);
    else
        hipLaunchKernelGGL(rbgs3d_color<1>, grid, dim3(256), 0, s, phi, div, mask, ny, nx, z0, zoff,
                           k.cx, k.cy, k.cz, k.cd, k.dt_inv, k.tol, ws, it);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// v5.py:205-210 generalised to 3-D: Python-float constants, rounded to f32
// where they meet f32 data; 1.0 / np.float32(dt) stays float32
RbgsConsts rbgs3d_consts(double dx, double dy, double dz, float dt, double tolerance) {
    const double dx2_inv = 1.0 / (dx * dx), dy2_inv = 1.0 / (dy * dy), dz2_inv = 1.0 / (dz * dz);
    const double denom_inv = 1.0 / (2.0 * (dx2_inv + dy2_inv + dz2_inv));
    RbgsConsts k;
    k.cx = (float)dx2_inv;
    k.cy = (float)dy2_inv;
    k.cz = (float)dz2_inv;
    k.cd = (float)denom_inv;
    k.dt_inv = 1.0f / dt;
    k.tol = (float)tolerance;
    return k;
}

// Red-black GS iterations per fused pass of a slab solve: 2 when the blocking
// depth is set to 4 levels (then a stop inside a pair is rolled back after the
// loop), else 1.
// Slab GS iterations per fused pass where the ghosts allow two (ghost 4):
// 2 unless the blocking depth is set to 2 or 3 (or off).
int rbgs3d_iters_per_pass() { return tuning().tb_steps == 4 || tuning().tb_steps == 0 ? 2 : 1; }
// Half-sweeps (colour levels) per fused pass of a single-GPU solve: the
// blocking depth, 2..4; auto = 4 (two iterations per HBM pass on the K = 4
// tall tiles: 2.86 ms per pass at 1024^3 = 745 Gcell/s, against 2.19 ms per
// 1.5 iterations = 730 at 3 levels, same box; r02).
int rbgs3d_half_per_pass() { return tuning().tb_steps >= 2 ? tuning().tb_steps : 4; }

// One fused GS pass of `iters` (1, 2) iterations: the tuned 2-level kernel
// when its rows are set explicitly (5, 13), the tall-tile kernel otherwise
// (always for a lagged stop test, which only the tall-tile kernel has).
int rbgs3d_fused_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                      int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int it,
                      int iters, RbgsWs *ws, hipStream_t s, int lag) {
    return rbgs3d_half_pass(in, out, div, nz, ny, nx, zb, ze, fixed_lo, fixed_hi, zoff, k, 2 * it,
                            2 * iters, ws, s, lag);
}

// A fused GS pass of `levels` half-sweeps from half-sweep h0, on the tile rows
// set for that depth (2: 16, 18, 20, 28; 3: 16, 18; 4: 15, 16), else auto.
int rbgs3d_half_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                     int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int h0,
                     int levels, RbgsWs *ws, hipStream_t s, int lag) {
    const int r = tuning().tb_rows;
    const bool shape_ok = levels == 2   ? (r == 16 || r == 18 || r == 20 || r == 28)
                          : levels == 3 ? (r == 16 || r == 18)
                          : levels == 4 ? (r == 15 || r == 16)
                                        : false;
    return rbgs3d_tbr_pass(in, out, div, nz, ny, nx, zb, ze, fixed_lo, fixed_hi, zoff, k, h0, levels,
                           ws, 0, 0, shape_ok ? r : 0, s, lag);
}

// One pass of k Jacobi sweeps over planes [zb, ze) (k = 1..4): the single
// sweep for k = 1, else the tall-tile jacobi3d_tbr with the tile shape
// cfd_set_jacobi3d_blocking selected (16, 18, 20 or 28 rows for k = 2; 16, 17
// or 18 for k = 3; 14, 15 or 16 for k = 4; 0 = chosen by its cost model).
int jacobi3d_blocked_pass(int k, const float *in, float *out, const float *src, int nz, int ny,
                          int nx, int zb, int ze, int fixed_lo, int fixed_hi, float h2, float dt,
                          bool pre, hipStream_t s) {
    // the configured rows apply to passes of the configured depth; a shorter
    // remainder pass picks its own tile
    const int rows = k == jacobi3d_tb_levels() ? tuning().tb_rows : 0, zc = tuning().tb_zchunk;
    if (k == 1) return jacobi3d_sweep(in, out, src, nullptr, nz, ny, nx, zb, ze, h2, dt, pre, nullptr, s);
    return jacobi3d_tbr_pass(k, rows, in, out, src, nz, ny, nx, zb, ze,
                             fixed_lo, fixed_hi, h2, dt, zc, pre, s);
}

// Whether a solve can start with a fused first pass (jacobi3d_tbr_first_pass:
// the RHS workspace formed by the pass itself, and, from zero, no phi read):
// the blocked path, a workspace, the LDS-DMA kernel (prefetch 1).
static bool jacobi3d_first_ok(const float *rhs_ws, bool vec_ok, int nz, int ny, int iters) {
    return rhs_ws && vec_ok && jacobi3d_tb_enabled() && jacobi3d_tb_prefetch() == 1 && nz >= 3 &&
           ny >= 3 && iters >= 2 && aligned16(rhs_ws);
}

// The blocked solve with a fused first pass of k1 = 2..4 sweeps (k1 =
// iters mod K when that is 2 or 3, K when it is 0, so the passes of K that
// follow need no shorter remainder pass), then passes of K, any remainder last.  zero: phi
// starts as zeros (its boundary ring zeroed here in both arrays; nothing of
// phi is read), and the first pass writes the array that makes the last
// pass land in phi -- no zero fill, no RHS prologue, no final copy.  Else phi
// holds the initial guess (faces copied to phi_tmp, the first pass reads phi).
static int jacobi3d_blocked_solve(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                                  int nz, int ny, int nx, float h2, float dt, int iters, bool zero,
                                  hipStream_t s) {
    int rc;
    const int K = jacobi3d_tb_levels();
    const int r = iters % K;
    int k1 = (r == 2 || r == 3) ? r : r == 0 ? K : (K < 3 ? K : 3);
    if (k1 > iters) k1 = iters;
    const int rest = iters - k1;
    const int npass = 1 + (rest + K - 1) / K;
    float *first_out = zero && npass % 2 == 1 ? phi : phi_tmp;
    if (zero) {
        if ((rc = launch_zero_faces3d(phi, phi_tmp, nz, ny, nx, s))) return rc;
    } else if ((rc = launch_fix_faces3d(phi, phi_tmp, nullptr, ny, nx, 0, nz, 0, nz - 1, s))) {
        return rc;
    }
    const int tk = timing_begin(s);
    if ((rc = jacobi3d_tbr_first_pass(k1, first_out, div, rhs_ws, phi, nz, ny, nx, 1, nz - 1, 1, 1, h2,
                                      dt, tuning().tb_zchunk, zero, s)))
        return rc;
    float *a = first_out, *b = first_out == phi ? phi_tmp : phi;
    for (int done = k1; done < iters;) {
        const int k = iters - done < K ? iters - done : K;
        if ((rc = jacobi3d_blocked_pass(k, a, b, rhs_ws, nz, ny, nx, 1, nz - 1, 1, 1, h2, dt, true, s)))
            return rc;
        done += k;
        float *t = a;
        a = b;
        b = t;
    }
    timing_end(tk, s, iters);
    if (a != phi)
        CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(float) * (size_t)nz * ny * nx, hipMemcpyDeviceToDevice, s));
    return CFD_OK;
}

}  // namespace cfd

using namespace cfd;

extern "C" {

int cfd_set_jacobi3d_prefetch(int planes) {
    CFD_REQUIRE(planes >= 0 && planes <= 2, "prefetch planes must be 0 (auto), 1 or 2");
    tuning().tb_prefetch = planes;
    return CFD_OK;
}

int cfd_set_jacobi3d_blocking(int steps, int rows, int zchunk) {
    CFD_REQUIRE(steps >= 0 && steps <= 4, "blocking steps must be 0 (auto), 1 (off) or 2..4");
    CFD_REQUIRE(rows == 0 || rows == 14 || rows == 15 || rows == 16 || rows == 17 || rows == 18 || rows == 20 ||
                    rows == 28,
                "blocking rows must be 0 (auto), 16, 18, 20, 28 (2 levels), 16, 17, 18 (3), 14, 15, 16 (4)");
    CFD_REQUIRE(zchunk >= 0, "zchunk must be >= 0");
    tuning().tb_steps = steps;
    tuning().tb_rows = rows;
    tuning().tb_zchunk = zchunk;
    return CFD_OK;
}

int cfd_get_jacobi3d_levels(void) { return jacobi3d_tb_levels(); }
int cfd_get_rbgs3d_levels(void) { return rbgs3d_half_per_pass(); }

int cfd_set_jacobi3d_config(int variant, int waves, int zchunk) {
    CFD_REQUIRE(variant >= 0 && variant <= 2, "variant must be 0..2");
    CFD_REQUIRE(waves == 0 || waves == 1 || waves == 2 || waves == 4 || waves == 8 || waves == 16,
                "waves must be 0,1,2,4,8,16");
    CFD_REQUIRE(zchunk >= 0, "zchunk must be >= 0");
    tuning().j3_variant = variant;
    tuning().j3_waves = waves;
    tuning().j3_zchunk = zchunk;
    return CFD_OK;
}

int cfd_jacobi3d_sweep_f32(const float *in, float *out, const float *div, const uint8_t *mask,
                           int nz, int ny, int nx, int z_begin, int z_end, double h, float dt,
                           float *resid, void *stream) {
    CFD_REQUIRE(in && out && div, "jacobi3d_sweep: null pointer");
    CFD_REQUIRE(nz >= 1 && ny >= 1 && nx >= 1, "jacobi3d_sweep: bad shape");
    return jacobi3d_sweep(in, out, div, mask, nz, ny, nx, z_begin, z_end, (float)(h * h), dt, false,
                          resid, as_stream(stream));
}

int cfd_jacobi3d_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                     const uint8_t *mask, int nz, int ny, int nx, double h, float dt, int iters,
                     int resid_every, float *resid_out, void *stream) {
    CFD_REQUIRE(div && phi && phi_tmp, "jacobi3d: null array pointer");
    CFD_REQUIRE(nz >= 1 && ny >= 1 && nx >= 1 && iters >= 0, "jacobi3d: bad arguments");
    CFD_REQUIRE(resid_every <= 0 || resid_out, "jacobi3d: resid_every > 0 needs resid_out");
    if (iters == 0) return CFD_OK;
    hipStream_t s = as_stream(stream);
    const size_t plane = (size_t)ny * nx;
    int rc;
    const bool vec_ok0 = nx % 4 == 0 && aligned16(phi) && aligned16(phi_tmp) && aligned16(div);
    if (!mask && resid_every <= 0 && jacobi3d_first_ok(rhs_ws, vec_ok0, nz, ny, iters))
        return jacobi3d_blocked_solve(div, phi, phi_tmp, rhs_ws, nz, ny, nx, (float)(h * h), dt, iters,
                                      false, s);
    // Dirichlet faces the sweep never writes (planes 0, nz-1; rows 0, ny-1)
    if ((rc = launch_fix_faces3d(phi, phi_tmp, mask, ny, nx, 0, nz, 0, nz - 1, s))) return rc;
    const int nres = resid_every > 0 ? iters / resid_every : 0;
    if (nres > 0) CFD_CHECK_HIP(hipMemsetAsync(resid_out, 0, sizeof(float) * nres, s));
    const float h2 = (float)(h * h);
    // RHS prologue: with a workspace the sweeps read rhs instead of dividing
    const bool pre = rhs_ws != nullptr;
    const float *src = div;
    if (pre) {
        if ((rc = launch_rhs_f32(div, rhs_ws, plane * nz, h2, dt, s))) return rc;
        src = rhs_ws;
    }
    float *a = phi, *b = phi_tmp;
    const int tk = timing_begin(s);
    const bool vec_ok = nx % 4 == 0 && aligned16(phi) && aligned16(phi_tmp) && aligned16(src);
    if (jacobi3d_tb_enabled() && !mask && resid_every <= 0 && vec_ok && nz >= 3 && ny >= 3 &&
        iters >= 2) {
        // temporally blocked: passes of K sweeps, the remainder last
        const int K = jacobi3d_tb_levels();
        int done = 0;
        while (done < iters) {
            const int k = iters - done < K ? iters - done : K;
            rc = jacobi3d_blocked_pass(k, a, b, src, nz, ny, nx, 1, nz - 1, 1, 1, h2, dt, pre, s);
            if (rc) return rc;
            if (done == 0 && (rc = launch_fix_faces3d(phi_tmp, phi, nullptr, ny, nx, 0, nz, 0, nz - 1, s)))
                return rc;
            done += k;
            float *t = a;
            a = b;
            b = t;
        }
        timing_end(tk, s, iters);
        if (a != phi)
            CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(float) * plane * nz, hipMemcpyDeviceToDevice, s));
        return CFD_OK;
    }
    for (int it = 0; it < iters; ++it) {
        float *r = (resid_every > 0 && (it + 1) % resid_every == 0)
                       ? resid_out + ((it + 1) / resid_every - 1)
                       : nullptr;
        if ((rc = jacobi3d_sweep(a, b, src, mask, nz, ny, nx, 1, nz - 1, h2, dt, pre, r, s))) return rc;
        if (it == 0 && iters > 1 &&
            (rc = launch_fix_faces3d(phi_tmp, phi, nullptr, ny, nx, 0, nz, 0, nz - 1, s)))
            return rc;
        float *t = a;
        a = b;
        b = t;
    }
    timing_end(tk, s, iters);
    if (a != phi)
        CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(float) * plane * nz, hipMemcpyDeviceToDevice, s));
    return CFD_OK;
}

int cfd_jacobi3d_zero_f32(const float *div, float *phi, float *phi_tmp, float *rhs_ws, int nz,
                          int ny, int nx, double h, float dt, int iters, void *stream) {
    CFD_REQUIRE(div && phi && phi_tmp, "jacobi3d_zero: null array pointer");
    CFD_REQUIRE(nz >= 1 && ny >= 1 && nx >= 1 && iters >= 0, "jacobi3d_zero: bad arguments");
    hipStream_t s = as_stream(stream);
    const bool vec_ok = nx % 4 == 0 && aligned16(phi) && aligned16(phi_tmp) && aligned16(div);
    if (jacobi3d_first_ok(rhs_ws, vec_ok, nz, ny, iters))
        return jacobi3d_blocked_solve(div, phi, phi_tmp, rhs_ws, nz, ny, nx, (float)(h * h), dt, iters,
                                      true, s);
    // other layouts: the zero fill, then the general solve
    CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(float) * (size_t)nz * ny * nx, s));
    return cfd_jacobi3d_f32(div, phi, phi_tmp, rhs_ws, nullptr, nz, ny, nx, h, dt, iters, 0, nullptr,
                            stream);
}

int cfd_rbgs3d_f32(float *phi, const float *div, const uint8_t *mask, int nz, int ny, int nx,
                   double dx, double dy, double dz, float dt, int iterations, double tolerance,
                   float *phi_tmp, void *ws, int *iters_done, void *stream) {
    CFD_REQUIRE(phi && div && ws, "rbgs3d: null pointer");
    CFD_REQUIRE(nz >= 1 && ny >= 1 && nx >= 1 && iterations >= 0, "rbgs3d: bad arguments");
    hipStream_t s = as_stream(stream);
    const RbgsConsts k = rbgs3d_consts(dx, dy, dz, dt, tolerance);
    RbgsWs *w = reinterpret_cast<RbgsWs *>(ws);
    int rc = launch_rbgs_init(w, iterations, k.tol, iters_done, s);
    if (rc) return rc;
    if (nz < 3 || ny < 3 || nx < 3 || iterations == 0) return CFD_OK;
    const size_t n = (size_t)nz * ny * nx;
    const int tk = timing_begin(s);
    if (rbgs3d_fused_ok(phi, phi_tmp, div, mask, nx)) {
        // fused: out-of-place passes of pp iterations (both colours each),
        // ping-pong; the result's buffer and a stop inside a pair pass are
        // resolved on the device after the loop
        if ((rc = launch_fix_faces3d(phi, phi_tmp, nullptr, ny, nx, 0, nz, 0, nz - 1, s))) return rc;
        // passes of P half-sweeps (colour levels), the last one shorter
        const int P = rbgs3d_half_per_pass(), H = 2 * iterations;
        float *a = phi, *b = phi_tmp;
        for (int h = 0; h < H; h += P) {
            const int m = H - h >= P ? P : H - h;
            if ((rc = rbgs3d_half_pass(a, b, div, nz, ny, nx, 1, nz - 1, 1, 1, 0, k, h, m, w, s, 0)))
                return rc;
            float *t = a; a = b; b = t;
        }
        const int hpp = P;
        timing_end(tk, s, iterations);
        if ((rc = launch_rbgs_count(w, iters_done, s))) return rc;
        // a stop inside a pass: re-run its half-sweeps up to the stop, one
        // launch per possible count (2c - P j is even when P is); none when
        // no stop is possible (tolerance <= 0)
        for (int need = 1; need < hpp && k.tol > 0.f; ++need)
            if (!(hpp % 2 == 0 && need % 2 == 1) &&
                (rc = rbgs3d_tbr_pass(phi, phi_tmp, div, nz, ny, nx, 1, nz - 1, 1, 1, 0, k, 0, need, w, hpp,
                                      H, 0, s)))
                return rc;
        return launch_rbgs_copy(w, phi, phi_tmp, n, hpp, s);
    }
    for (int it = 0; it < iterations; ++it) {
        if ((rc = rbgs3d_colour_pass(0, phi, div, mask, ny, nx, 1, nz - 1, 0, k, w, it, s))) return rc;
        if ((rc = rbgs3d_colour_pass(1, phi, div, mask, ny, nx, 1, nz - 1, 0, k, w, it, s))) return rc;
    }
    timing_end(tk, s, iterations);
    return launch_rbgs_finish(w, phi, nullptr, n, iters_done, s);
}

int cfd_rbgs3d_pass_f32(const float *in, float *out, const float *div, int nz, int ny, int nx,
                        int z_begin, int z_end, int fixed_lo, int fixed_hi, int z_global_offset,
                        double dx, double dy, double dz, float dt, double tolerance, int iteration,
                        void *ws, void *stream) {
    CFD_REQUIRE(in && out && div && ws, "rbgs3d_pass: null pointer");
    CFD_REQUIRE(in != out, "rbgs3d_pass: out of place only");
    CFD_REQUIRE(nz >= 1 && ny >= 3 && nx >= 1 && iteration >= 0, "rbgs3d_pass: bad arguments");
    CFD_REQUIRE(nx % 4 == 0 && aligned16(in) && aligned16(out) && aligned16(div),
                "rbgs3d_pass: needs nx %% 4 == 0 and 16-byte aligned arrays");
    // a non-fixed neighbour plane is itself updated from the plane beyond it
    CFD_REQUIRE(z_begin >= (fixed_lo ? 1 : 2) && z_end <= nz - (fixed_hi ? 1 : 2) && z_begin <= z_end,
                "rbgs3d_pass: planes [%d,%d) need 1 (fixed) or 2 readable planes on each side (nz %d)",
                z_begin, z_end, nz);
    const RbgsConsts k = rbgs3d_consts(dx, dy, dz, dt, tolerance);
    return rbgs3d_fused_pass(in, out, div, nz, ny, nx, z_begin, z_end, fixed_lo, fixed_hi,
                             z_global_offset, k, iteration, 1, reinterpret_cast<RbgsWs *>(ws),
                             as_stream(stream));
}

int cfd_rbgs_init(void *ws, int iterations, double tolerance, int *iters_done, void *stream) {
    CFD_REQUIRE(ws && iterations >= 0, "rbgs_init: bad arguments");
    return launch_rbgs_init(reinterpret_cast<RbgsWs *>(ws), iterations, (float)tolerance, iters_done,
                            as_stream(stream));
}

int cfd_rbgs_finish(void *ws, float *phi, const float *phi_tmp, size_t n, int *iters_done,
                    void *stream) {
    CFD_REQUIRE(ws && phi, "rbgs_finish: null pointer");
    return launch_rbgs_finish(reinterpret_cast<RbgsWs *>(ws), phi, phi_tmp, n, iters_done,
                              as_stream(stream));
}

}  // extern "C"
