// fields2d.hip -- predictor (advection-diffusion), divergence, projection,
// step epilogue and diagnostic reductions of the v5 cylinder solver's
// time_step(), v5.py:375-441, for gfx950.
//
// Arithmetic follows the reference as it executes in NumPy-scalar form: every
// Python-float constant is rounded to float32 where it meets float32 data
// (NEP 50), operations run in float32 in the source order, nothing is fused
// (-ffp-contract=off).  |V| = (u**2 + v**2) ** 0.5 goes through the device
// copy of glibc's powf (libm_powf.hpp), as NumPy's float32 scalar `**` does
// in the reference, so the predictor is bit-exact too.
//
// These kernels are one-pass per cell and HBM-bound; the fused predictor
// reads u, v once (5-point neighbourhoods from L1/L2) and writes u*, v*, tau.
#include <atomic>
#include <map>
#include <mutex>

#include "common.hpp"
#include "internal.hpp"
#include "libm_powf.hpp"
#include "pred_rows.hpp"

namespace cfd {

using PredConst = PredK<float>;
static PredConst make_pred_const(double dx, double dy) { return make_pred_k<float>(dx, dy); }

// compute_supg_stabilization_fast body, v5.py:155-161: vel_mag =
// (u**2 + v**2) ** 0.5 on float32 scalars, i.e. libm powf three times
// (powf_sq / powf_sqrt: glibc powf at y = 2 / 0.5 bit for bit, with a cheap
// exact path away from rounding midpoints -- libm_powf.hpp)
__device__ inline float supg_tau(float u, float v, float nu, float dt, const PredConst &k,
                                 const libm::PowfTables &T = libm::kPowfTables) {
    const float vm = libm::powf_sqrt(libm::powf_sq(u, T) + libm::powf_sq(v, T), T);
    if (vm > k.eps) {
        const float pe = (vm * k.h) / (nu + k.eps);
        const float half = pe / 2.0f;
        const float lim = half < 1.0f ? half : 1.0f;  // Python min(1.0, Pe/2.0)
        return (k.h / (2.0f * vm)) * lim;
    }
    return dt / 2.0f;
}
__device__ inline bool interior(int i, int j, int ny, int nx) {
    return i >= 1 && i < ny - 1 && j >= 1 && j < nx - 1;
}

#define CFD_2D_INDEX                                     \
    const int j = blockIdx.x * blockDim.x + threadIdx.x; \
    const int i = blockIdx.y;                            \
    if (j >= nx) return;                                 \
    const size_t c = (size_t)i * nx + j;

__global__ void k_supg_tau(const float *__restrict__ u, const float *__restrict__ v,
                           const float *__restrict__ nu_eff, float nu_s, float *__restrict__ tau,
                           int ny, int nx, float dt, PredConst k) {
    CFD_2D_INDEX
    float t = 0.0f;  // np.zeros_like boundary ring
    if (interior(i, j, ny, nx)) t = supg_tau(u[c], v[c], nu_eff ? nu_eff[c] : nu_s, dt, k);
    tau[c] = t;
}

__global__ void k_conv_supg(const float *__restrict__ u, const float *__restrict__ v,
                            const float *__restrict__ f, const float *__restrict__ tau,
                            float *__restrict__ conv, int ny, int nx, PredConst k) {
    CFD_2D_INDEX
    float r = 0.0f;
    if (interior(i, j, ny, nx))
        r = conv_supg(u[c], v[c], f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], tau[c], k);
    conv[c] = r;
}

__global__ void k_conv_upwind(const float *__restrict__ u, const float *__restrict__ v,
                              const float *__restrict__ f, float *__restrict__ conv, int ny, int nx,
                              PredConst k) {
    CFD_2D_INDEX
    float r = 0.0f;
    if (interior(i, j, ny, nx))
        r = conv_upwind(u[c], v[c], f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], k);
    conv[c] = r;
}

__global__ void k_laplacian(const float *__restrict__ f, const float *__restrict__ nu_eff, float nu_s,
                            float *__restrict__ lap, int ny, int nx, PredConst k) {
    CFD_2D_INDEX
    float r = 0.0f;
    if (interior(i, j, ny, nx))
        r = laplacian(nu_eff ? nu_eff[c] : nu_s, f[c], f[c + 1], f[c - 1], f[c + nx], f[c - nx], k);
    lap[c] = r;
}

// Fused predictor, v5.py:388-403: u* = u + dt*(-conv_u + lap_u), likewise v.
template <bool SUPG>
__global__ __launch_bounds__(256) void k_predictor(const float *__restrict__ u,
                                                   const float *__restrict__ v,
                                                   const float *__restrict__ nu_eff, float nu_s,
                                                   float *__restrict__ us, float *__restrict__ vs,
                                                   float *__restrict__ tau_out, int ny, int nx,
                                                   float dt, PredConst k) {
    CFD_2D_INDEX
    const float uc = u[c], vc = v[c];
    float cu = 0.0f, cv = 0.0f, lu = 0.0f, lv = 0.0f, t = 0.0f;
    if (interior(i, j, ny, nx)) {
        const float nu = nu_eff ? nu_eff[c] : nu_s;
        const float uE = u[c + 1], uW = u[c - 1], uN = u[c + nx], uS = u[c - nx];
        const float vE = v[c + 1], vW = v[c - 1], vN = v[c + nx], vS = v[c - nx];
        if (SUPG) {
            t = supg_tau(uc, vc, nu, dt, k);
            cu = conv_supg(uc, vc, uc, uE, uW, uN, uS, t, k);
            cv = conv_supg(uc, vc, vc, vE, vW, vN, vS, t, k);
        } else {
            cu = conv_upwind(uc, vc, uc, uE, uW, uN, uS, k);
            cv = conv_upwind(uc, vc, vc, vE, vW, vN, vS, k);
        }
        lu = laplacian(nu, uc, uE, uW, uN, uS, k);
        lv = laplacian(nu, vc, vE, vW, vN, vS, k);
    }
    us[c] = uc + dt * (-cu + lu);
    vs[c] = vc + dt * (-cv + lv);
    if (tau_out) tau_out[c] = t;  // 0 without SUPG (v5.py:292: never assigned without SUPG)
}

// compute_divergence_fast, v5.py:178-187 (+ max|div| diagnostic, v5.py:410)
__global__ __launch_bounds__(256) void k_divergence(const float *__restrict__ u,
                                                    const float *__restrict__ v,
                                                    float *__restrict__ div, int ny, int nx,
                                                    float cx, float cy, float *absmax) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    float m = 0.0f;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        float d = 0.0f;
        if (interior(i, j, ny, nx)) d = (u[c + 1] - u[c - 1]) * cx + (v[c + nx] - v[c - nx]) * cy;
        div[c] = d;
        const float a = fabsf(d);
        if (a > m) m = a;
    }
    if (absmax) wave_reduce_max_store(m, absmax);
}

// compute_gradient_fast, v5.py:189-200
__global__ void k_gradient(const float *__restrict__ phi, float *__restrict__ gx,
                           float *__restrict__ gy, int ny, int nx, float cx, float cy) {
    CFD_2D_INDEX
    float a = 0.0f, b = 0.0f;
    if (interior(i, j, ny, nx)) {
        a = (phi[c + 1] - phi[c - 1]) * cx;
        b = (phi[c + nx] - phi[c - nx]) * cy;
    }
    gx[c] = a;
    gy[c] = b;
}

// v5.py:413-417: gradient of phi, then u = u* - dt*dpdx, v = v* - dt*dpdy;
// gradmax <- max sqrt(dpdx^2 + dpdy^2) (v5.py:414-415 diagnostic).
__global__ __launch_bounds__(256) void k_project(const float *__restrict__ phi,
                                                 const float *__restrict__ us,
                                                 const float *__restrict__ vs,
                                                 float *__restrict__ u, float *__restrict__ v,
                                                 int ny, int nx, float cx, float cy, float dt,
                                                 float *gradmax) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    float m = 0.0f;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        float a = 0.0f, b = 0.0f;
        if (interior(i, j, ny, nx)) {
            a = (phi[c + 1] - phi[c - 1]) * cx;
            b = (phi[c + nx] - phi[c - nx]) * cy;
        }
        u[c] = us[c] - dt * a;
        v[c] = vs[c] - dt * b;
        if (gradmax) {
            const float g = sqrtf(a * a + b * b);
            if (g > m) m = g;
        }
    }
    if (gradmax) wave_reduce_max_store(m, gradmax);
}

// ------------------------------------------------------------ epilogue
// clean_divergence_fast phi sweep (v5.py:250-253) in the serial lexicographic
// order: a single workgroup walks the anti-diagonals; every cell of a
// diagonal depends only on earlier diagonals (W, S: new) and later ones
// (E, N: old), so updating one diagonal at a time reproduces the serial loop
// exactly.  Thread t owns row b0+t of a band of blockDim rows and updates
// column j = s - t + 1 at step s, so the NEW values never go through global
// memory: W is the thread's own last output (a register), S the output of
// thread t-1 one step earlier (LDS, double-buffered by step parity, one
// barrier per step).  The OLD values -- E, div, and N -- are fetched PD steps
// ahead (N within a wave is lane t+1's E of the same step, by DPP).  Row b0-1
// (the previous band, finished) and the boundary rows are fetched like E.
__global__ __launch_bounds__(1024) void k_lex_gs_sweep(float *__restrict__ phi,
                                                       const float *__restrict__ div, int ny,
                                                       int nx, float cx, float cy, float cd) {
    constexpr int PD = 4;  // prefetch distance (steps)
    __shared__ float outb[2][1024];
    const int t = threadIdx.x, nt = blockDim.x, lane = t & 63;
    const int imax = ny - 2, jmax = nx - 2;
    for (int b0 = 1; b0 <= imax; b0 += nt) {
        __threadfence();  // the previous band's rows are final and visible
        __syncthreads();
        const int nrows = min(nt, imax - b0 + 1);
        const int i = b0 + t;
        const bool rowok = t < nrows;
        const size_t rowc = (size_t)(rowok ? i : 0) * nx;
        // N from memory for the last row of the band / grid and for lane 63
        // (its lower neighbour row is in another wave); S for thread 0
        const bool nmem = lane == 63 || t == nrows - 1;
        float qE[PD], qD[PD], qN[PD], qS[PD];
        auto fetch = [&](int st, float &e, float &d, float &n, float &sv) {
            const int j = st - t + 1;
            const bool act = rowok && j >= 1 && j <= jmax;
            e = (rowok && j >= 0 && j <= jmax) ? phi[rowc + j + 1] : 0.f;
            d = act ? div[rowc + j] : 0.f;
            n = (act && nmem) ? phi[rowc + j + nx] : 0.f;
            sv = (act && t == 0) ? phi[rowc + j - nx] : 0.f;
        };
#pragma unroll
        for (int p = 0; p < PD; ++p) fetch(p, qE[p], qD[p], qN[p], qS[p]);
        float w = rowok ? phi[rowc] : 0.f;  // phi(i, 0): W of column 1
        const int nsteps = nrows - 1 + jmax;
        for (int st = 0; st < nsteps; ++st) {
            const int j = st - t + 1;
            const bool act = rowok && j >= 1 && j <= jmax;
            const float E = qE[0], D = qD[0], Nm = qN[0], S0 = qS[0];
            const float nup = dpp_from_upper(E);  // lane t+1's E: old phi(i+1, j)
#pragma unroll
            for (int p = 0; p + 1 < PD; ++p) {
                qE[p] = qE[p + 1];
                qD[p] = qD[p + 1];
                qN[p] = qN[p + 1];
                qS[p] = qS[p + 1];
            }
            fetch(st + PD, qE[PD - 1], qD[PD - 1], qN[PD - 1], qS[PD - 1]);
            if (act) {
                const float S = t == 0 ? S0 : outb[(st + 1) & 1][t - 1];  // thread t-1 at step st-1
                const float N = nmem ? Nm : nup;
                const float a = cx * (E + w);
                const float b = cy * (N + S);
                const float v = ((a + b) - D) * cd;
                phi[rowc + j] = v;
                w = v;
                outb[st & 1][t] = v;
            }
            __syncthreads();
        }
    }
}

// The sweep on a SKEWED copy of phi and div (r05, the default): the r02-r04
// staged kernels kept phi row-major, so the diagonal a wave touches per step
// (lane l: row r0 + l, column d - l) is 64 cache lines, and a CU's vector
// memory path moves about one line per clock -- measured 90-100 us per
// 600-column sweep, several times the ~47-cycle dependent chain per step
// (scripts/chain_probe.hip).  clean_divergence owns its phi and div (the
// workspace), so it stores them diagonal-major instead:
//   rows in blocks of 64 (block m: rows 1 + 64 m + l, l < 64); within a
//   block, diagonal d = j + l in groups of four:
//     (m, d, l) -> ((m DG + d / 4) 64 + l) 4 + d % 4,   DG = ceil((nx + 63) / 4)
// so a wave's four consecutive steps of one field -- lane l's slots d .. d + 3
// -- are one coalesced 1-KB dwordx4.  The grid-wide kernels pay the scatter
// instead (k_divergence_skew writes div there, k_sub_gradient_skew reads phi
// there), spread over every CU.
// Per wave (one 64-row block, one lane per row, up to 4 waves per band), at
// step d lane l updates column j = d - l:
//  * E (old phi of its row at j + 1) is slot d + 1 of its own row;
//  * N (old phi of row r + 1 at j) is lane l + 1's E of the same step (DPP);
//    lane 63's is the next block's lane 0 at slot d - 63;
//  * S (new phi of row r - 1 at j) is lane l - 1's previous result (DPP);
//    lane 0's is the wave above's last lane, published per 16 steps into an
//    LDS row with a counter, or for a band's first wave the block above's
//    lane 63 at slot d + 63 (final: the band before);
//  * the operands stream kSkewRing groups of four steps ahead in registers
//    (the two rows from other blocks by lanes 63 and 0 alone); results leave
//    four steps at a time (0 at the zero side columns and the padding).
// Same arithmetic and order as the serial loop: bit-identical.
constexpr size_t kLexLdsMax = 160 * 1024;  // LDS a sweep workgroup may take
constexpr int kSkewWaves = 4;  // waves per band: at one wave per SIMD the chain, not the memory path, sets the pace
constexpr int kSkewRing = 8;   // groups of 4 steps in flight per wave (and per loop iteration)
constexpr int kSkewMcBlocks = 128;        // k_lex_gs_skew_mc: blocks (workgroups) at most
constexpr size_t kSkewMcLds = 64 * 1024;  // k_lex_gs_skew_mc: LDS asked for (unused; two per CU at most)
__host__ __device__ inline int lex_skew_blocks(int ny) { return (ny - 2 + 63) >> 6; }
__host__ __device__ inline int lex_skew_groups(int nx) { return (nx + 63 + 3) >> 2; }
size_t lex_skew_floats(int ny, int nx) { return (size_t)lex_skew_blocks(ny) * (size_t)lex_skew_groups(nx) * 256; }
// the per-block progress words of k_lex_gs_skew_mc, after div and the two phi
size_t lex_skew_prog_offset(int ny, int nx) { return (3 * sizeof(float) * lex_skew_floats(ny, nx) + 255) & ~(size_t)255; }
// floats per wave row of k_lex_gs_skew's LDS: column c at c + 64 for
// c = -63 .. nx + 76, 16 B aligned
constexpr int lex_skew_rsl(int nx) { return (nx + 160 + 3) & ~3; }
size_t lex_skew_lds_bytes(int nw, int nx) { return (size_t)nw * lex_skew_rsl(nx) * sizeof(float); }
__device__ inline size_t skew_at(int i, int j, int dg) {  // interior row i >= 1, column j >= 0
    const int m = (i - 1) >> 6, l = (i - 1) & 63, d = j + l;
    return (((size_t)m * dg + (d >> 2)) * 64 + l) * 4 + (d & 3);
}

// compute_divergence_fast (v5.py:178-187) into the skewed layout: interior
// rows, every column (0 at the side columns, as k_divergence).  With zphi the
// grid has one more row, ny - 1, and zphi gets zeros on row ny - 1 when that
// row is a lane of the last block: the first sweep leaves the rows past ny - 2
// unwritten, and the next sweep reads that one as the last row's N.
__global__ __launch_bounds__(256) void k_divergence_skew(const float *__restrict__ u, const float *__restrict__ v,
                                                         float *__restrict__ div_s, float *__restrict__ zphi, int ny,
                                                         int nx, float cx, float cy) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y + 1;
    if (j >= nx) return;
    const int dg = lex_skew_groups(nx);
    if (i == ny - 1) {  // zphi only
        if (((ny - 2) & 63) != 0) zphi[skew_at(i, j, dg)] = 0.0f;
        return;
    }
    const size_t c = (size_t)i * nx + j;
    float d = 0.0f;
    if (j >= 1 && j <= nx - 2) d = (u[c + 1] - u[c - 1]) * cx + (v[c + nx] - v[c - nx]) * cy;
    div_s[skew_at(i, j, dg)] = d;
}

// u -= dphi/dx, v -= dphi/dy (v5.py:255-256) with phi in the skewed layout
// (rows 0 and ny - 1 are the zero boundary).
__device__ inline float skew_phi(const float *phi_s, int i, int j, int ny, int dg) {
    return i >= 1 && i <= ny - 2 ? phi_s[skew_at(i, j, dg)] : 0.0f;
}
__global__ void k_sub_gradient_skew(const float *__restrict__ phi_s, float *__restrict__ u, float *__restrict__ v,
                                    int ny, int nx, float cx, float cy) {
    CFD_2D_INDEX
    if (!interior(i, j, ny, nx)) return;
    const int dg = lex_skew_groups(nx);
    const float a = (skew_phi(phi_s, i, j + 1, ny, dg) - skew_phi(phi_s, i, j - 1, ny, dg)) * cx;
    const float b = (skew_phi(phi_s, i + 1, j, ny, dg) - skew_phi(phi_s, i - 1, j, ny, dg)) * cy;
    u[c] = u[c] - a;
    v[c] = v[c] - b;
}

// clean_divergence's second iteration without materialising the first one's
// u, v (iterations == 2, the reference's call, v5.py:430): div of
// u1 = u - dphi1/dx, v1 = v - dphi1/dy, each neighbour's u1 / v1 re-formed with
// k_sub_gradient_skew's operations (the boundary ring keeps u, v), then
// k_divergence's -- the same bits as the three launches.
__global__ __launch_bounds__(256) void k_divergence2_skew(const float *__restrict__ u, const float *__restrict__ v,
                                                          const float *__restrict__ phi1, float *__restrict__ div_s,
                                                          int ny, int nx, float cx, float cy) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y + 1;
    if (j >= nx) return;
    const int dg = lex_skew_groups(nx);
    float d = 0.0f;
    if (j >= 1 && j <= nx - 2) {
        auto u1 = [&](int jj) {
            const float u0 = u[(size_t)i * nx + jj];
            if (jj < 1 || jj > nx - 2) return u0;
            const float a = (skew_phi(phi1, i, jj + 1, ny, dg) - skew_phi(phi1, i, jj - 1, ny, dg)) * cx;
            return u0 - a;
        };
        auto v1 = [&](int ii) {
            const float v0 = v[(size_t)ii * nx + j];
            if (ii < 1 || ii > ny - 2) return v0;
            const float b = (skew_phi(phi1, ii + 1, j, ny, dg) - skew_phi(phi1, ii - 1, j, ny, dg)) * cy;
            return v0 - b;
        };
        d = (u1(j + 1) - u1(j - 1)) * cx + (v1(i + 1) - v1(i - 1)) * cy;
    }
    div_s[skew_at(i, j, dg)] = d;
}

// both iterations' u -= dphi/dx, v -= dphi/dy in one pass: (u - a1) - a2, the
// two in-place subtractions' bits
__global__ void k_sub_gradient2_skew(const float *__restrict__ phi1, const float *__restrict__ phi2,
                                     float *__restrict__ u, float *__restrict__ v, int ny, int nx, float cx, float cy) {
    CFD_2D_INDEX
    if (!interior(i, j, ny, nx)) return;
    const int dg = lex_skew_groups(nx);
    const float a1 = (skew_phi(phi1, i, j + 1, ny, dg) - skew_phi(phi1, i, j - 1, ny, dg)) * cx;
    const float b1 = (skew_phi(phi1, i + 1, j, ny, dg) - skew_phi(phi1, i - 1, j, ny, dg)) * cy;
    const float a2 = (skew_phi(phi2, i, j + 1, ny, dg) - skew_phi(phi2, i, j - 1, ny, dg)) * cx;
    const float b2 = (skew_phi(phi2, i + 1, j, ny, dg) - skew_phi(phi2, i - 1, j, ny, dg)) * cy;
    u[c] = (u[c] - a1) - a2;
    v[c] = (v[c] - b1) - b2;
}

struct SkewArgs {
    float *phi_base;  // the skewed phi buffers (phi_bytes in all)
    const float *div_s;
    unsigned long long *prog;  // MC: per block {epoch, groups stored and complete}
    int *fail;                 // MC: the device's persistent-failure counter
    unsigned long long poll_ticks;
    int phi_bytes, old_off, new_off;  // old_off kOob: all zeros (the first sweep)
    int ny, nx;
    unsigned epoch;
    float cx, cy, cd;
};

// One wave's sweep of block m.  !MC: up to 4 waves per band share a workgroup
// (one CU), lane 0's row above from the wave above through an LDS row, a
// band's first wave (FIRST) from memory.  MC (r05): one wave per workgroup,
// every block on its own CU, each wave FIRST: lane 0's row above is block
// m - 1's lane 63 in the new buffer, read with sc1 loads once block m - 1 has
// published (sc1, per 16 steps) that those groups are stored and complete;
// the progress word is polled two chunks ahead, so the poll's wait is the
// ring's own.
template <bool MC>
__device__ inline void lex_skew_wave(const SkewArgs &sa, int m, int wv, int nw, int lane, float *lex_rows,
                                     int *flags) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    constexpr int R = kSkewRing;
    constexpr int XA = MC ? 16 : 0;  // sc1 on the cross-block loads and the stores
    const int old_off = sa.old_off, new_off = sa.new_off;
    const float cx = sa.cx, cy = sa.cy, cd = sa.cd;
    const int RSL = lex_skew_rsl(sa.nx);
    const int imax = sa.ny - 2, jmax = sa.nx - 2;
    const int nb = lex_skew_blocks(sa.ny), DG = lex_skew_groups(sa.nx);
    const int bytes = nb * DG * 1024;
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(sa.phi_base, 0, sa.phi_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(sa.div_s), 0, bytes, 0x00020000);
    // steps d = 0 .. 4 DG - 1, 16 per chunk: every slot of the block is stored
    // (lane 63's last interior column is at d = nx + 61, its zero side column
    // at nx + 62, and the padding up to 4 DG - 1 is written too)
    const int nq = (DG + 3) >> 2;
    const int nc = (nq + R / 4 - 1) / (R / 4);  // loop iterations of 4 R steps
    const bool rowok = 1 + 64 * m + lane <= imax;
    // byte offsets of group 0 (group G at + 1024 G): own slots (div; old
    // phi; new phi); lane 63: the next block's lane 0, group G - 16, old;
    // lane 0 of a band's first wave: the block above's lane 63, group
    // G + 15, new.  (kOob + an offset stays past the buffer.)
    const int oD = (m * DG * 64 + lane) * 16;
    const int oS = old_off + oD;
    const int oX = lane == 63 ? (m + 1 < nb ? old_off + ((m + 1) * DG - 16) * 1024 : (int)kOob)
                   : lane == 0 && (MC || wv == 0) && m > 0 ? new_off + (((m - 1) * DG + 15) * 64 + 63) * 16
                                                    : (int)kOob;
    const int oW = rowok ? new_off + oD : (int)kOob;
    float *mine = MC ? nullptr : lex_rows + (size_t)wv * RSL + 64;
    const float *above = MC ? nullptr : lex_rows + (size_t)(wv > 0 ? wv - 1 : 0) * RSL + 64;
    // MC: block m - 1's progress (groups stored and complete), the two polls
    // in flight (issued two and one chunks back) and what is known so far
    unsigned long long poll_a = 0, poll_b = 0;
    int known = 0;
    // the in-flight polls must stay vector registers: a value the compiler
    // sees as uniform is moved to scalar registers right after its load,
    // which waits for it (and, memory operations completing in order, for
    // the whole prefetch ring) -- an opaque lane-dependent zero in the
    // address keeps it per lane until it is used, two chunks later
    int vz = 0;
    __asm__ volatile("" : "+v"(vz));
    unsigned long long *const prog_up = MC && m > 0 ? sa.prog + (m - 1) + vz : nullptr;
    auto progress_of = [&](unsigned long long v) {
        return (unsigned)(v >> 32) == sa.epoch ? (int)(unsigned)(v & 0x7fffffffull) : 0;
    };
    // a software pipeline of R groups: iteration c computes groups R c ..
    // R c + R - 1 and loads groups R (c + 1) + g into the slots it frees;
    // it starts at c = -1, whose steps only load (no lane is at a column
    // >= 1 there: nothing is stored or kept), so the loop has one shape
    // and the compiler's wait counts are the steady-state ones
    f4v P[R], D[R], X[R];
    float w, vprev;  // w: phi(i, j - 1)
    // !FIRST: the row above for the next chunk, read one chunk ahead, and the
    // wave above's count read just before it
    float S0n[16];
    int s0_flag = 0;
    auto s0_read = [&](int q) {
        __asm__ volatile("" ::: "memory");  // after the count read, in issue order
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const float4 a4 = *reinterpret_cast<const float4 *>(above + 16 * q + 4 * p);
            S0n[4 * p] = a4.x;
            S0n[4 * p + 1] = a4.y;
            S0n[4 * p + 2] = a4.z;
            S0n[4 * p + 3] = a4.w;
        }
    };
    // One 16-step chunk (ring slots 4 H .. 4 H + 3).  The step is issue-
    // bound (a wave64 VALU op takes 4 cycles: ~13 per step were ~55 cycles
    // against the ~47-cycle dependent chain), so the chunk is specialised:
    // FULL chunks -- every lane at a column 1 .. nx - 2 in all 16 steps,
    // most of a sweep -- skip the per-step column test and the selects;
    // FIRST (a band's first wave) takes lane 0's row above from X, the
    // others from the LDS row, without a per-step select.
    auto chunk = [&](auto Hc, auto FULLc, auto FIRSTc, int qc) {
        constexpr int H = decltype(Hc)::value;
        constexpr bool FULL = decltype(FULLc)::value, FIRST = decltype(FIRSTc)::value;
        float S0[16];
        if constexpr (!FIRST) {
            if (qc >= 0) {
                // wave w - 1's last lane must have published chunks 0 .. qc + 4
                // (its column 16 qc + 15 comes at its step 16 qc + 78).  The
                // count and the row were read one chunk ago (s0_prefetch);
                // only when that count fell short are they read again here
                const int need = qc + 5 < nq ? qc + 5 : nq;
                if (!(s0_flag >= need)) {
                    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&flags[wv - 1], __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_WORKGROUP)) < need)
                        __builtin_amdgcn_s_sleep(1);
                    s0_read(qc);
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) S0[k] = S0n[k];
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k) S0[k] = 0.f;
            }
            // the next chunk's count and row, in flight during this chunk: the
            // wait for them no longer stalls a chunk (two LDS round trips a
            // chunk made the waves that read them ~25 % slower per step).
            // LDS operations of a wave run in issue order, and the writer
            // stores the row before the count, so a row read issued after a
            // count read that saw the writer's count holds the row
            if (qc + 1 >= 0 && qc + 1 < nq) {
                s0_flag = __hip_atomic_load(&flags[wv - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                s0_read(qc + 1);
            }
        }
        if constexpr (MC) {
            if (m > 0) {
                // this chunk's refills read block m - 1's groups up to
                // 4 qc + 3 + R + 16: they must be stored and complete
                const unsigned long long v = poll_a;
                poll_a = poll_b;
                poll_b = __hip_atomic_load(prog_up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int pv = progress_of(v);
                known = pv > known ? pv : known;
                const int need = 4 * qc + R + 20;
                if (known < need) {  // wait (draining) until two chunks past the need
                    const unsigned long long t0 = wall_clock64();
                    while (true) {
                        const int p2 = progress_of(
                            __hip_atomic_load(sa.prog + (m - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                        known = p2 > known ? p2 : known;
                        if (known >= need + 8 || known == 0x7fffffff) break;
                        if (wall_clock64() - t0 > sa.poll_ticks) {  // fail loudly: counted, results garbage
                            if (lane == 0 && sa.fail) atomicAdd(sa.fail, 1);
                            known = 0x7fffffff;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
            }
        }
        // this chunk's group 0 at + sof; the refills R groups later
        const int sof = __builtin_amdgcn_readfirstlane(qc * 4 * 1024);
        float out[16];
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
            const int g = 4 * H + gg;  // ring slot
            const f4v p0 = P[g], p1 = P[(g + 1) % R], x0 = X[g], x1 = X[(g + 1) % R], d4 = D[g];
            f4v o4;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float e = k < 3 ? p0[k + 1] : p1[0];   // slot d + 1
                const float xn = k < 3 ? x0[k + 1] : x1[0];  // lane 63: slot d - 63
                float s0;
                if constexpr (FIRST)
                    s0 = k == 0 ? x0[3] : x1[k - 1];  // lane 0: slot d + 63
                else
                    s0 = S0[4 * gg + k];
                const float n = __int_as_float(__builtin_amdgcn_update_dpp(
                    __float_as_int(xn), __float_as_int(e), 0x130, 0xf, 0xf, false));  // wave_shl:1
                const float S = __int_as_float(__builtin_amdgcn_update_dpp(
                    __float_as_int(s0), __float_as_int(vprev), 0x138, 0xf, 0xf, false));  // wave_shr:1
                const float a = cx * (e + w);
                const float bb = cy * (n + S);
                const float v = ((a + bb) - d4[k]) * cd;
                if constexpr (FULL) {
                    w = v;
                    o4[k] = v;
                } else {
                    const int j = 16 * qc + 4 * gg + k - lane;  // step d = 16 qc + 4 gg + k
                    const bool act = (uint32_t)(j - 1) < (uint32_t)jmax;
                    w = act ? v : w;
                    o4[k] = act ? v : 0.f;  // the side columns and the padding stay 0
                }
                vprev = v;
                out[4 * gg + k] = v;
            }
            // (groups past the block's DG belong to the next block: the
            // loop's last iteration runs up to 8 groups past the end)
            const bool gok = FULL || (qc >= 0 && 4 * qc + gg < DG);
            __builtin_amdgcn_raw_buffer_store_b128(o4, rp, gok ? oW + 1024 * gg : (int)kOob, sof, XA);
            // group G + R's operands into the slot just freed (after its
            // last use: a load issued before it would need a second
            // register and a copy that waits for the load).  Slot g is
            // also read by group G - 1 (done), slot g + 1 by this group
            // (refilled next).
            P[g] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rp, oS + 1024 * gg,
                                                                                  sof + R * 1024, 0));
            D[g] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rd, oD + 1024 * gg,
                                                                                  sof + R * 1024, 0));
            // (all lanes load X though only lane 63 -- and lane 0 of a
            // band's first wave -- reads it: exec-masking the load to
            // those lanes measured 8-11 % slower, r05)
            X[g] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rp, oX + 1024 * gg,
                                                                                  sof + R * 1024, XA));
            // keep the prefetch where it is: the scheduler would sink it
            // next to its use, R groups later, exposing the latency
            __builtin_amdgcn_sched_barrier(0);
        }
        if (wv + 1 < nw && qc >= 0 && lane == 63) {
            // publish the last lane's 16 results (columns 16 qc - 63 + k)
#pragma unroll
            for (int k = 0; k < 16; ++k) mine[16 * qc - 63 + k] = out[k];
            // the row before the count (LDS completes in order; this keeps
            // the compiler from sinking the row writes past the flag)
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __hip_atomic_store(&flags[wv], qc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (MC) {
            // groups stored and complete: the operands of group 4 qc + 3, just
            // consumed (the compiler's wait came before their first use), were
            // loaded after the store of group 4 qc + 3 - R, and memory
            // operations complete in order
            const int cnt = 4 * qc + 4 - R;
            __asm__ volatile("" ::: "memory");
            if (cnt > 0 && lane == 0)
                __hip_atomic_store(sa.prog + m, ((unsigned long long)sa.epoch << 32) | (unsigned)cnt, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    using T1 = std::true_type;
    using F0 = std::false_type;
    static_assert(R == 8, "two 16-step chunks per iteration");
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    // iterations whose two chunks are both FULL: chunk 2 c >= 4 and
    // 16 (2 c + 1) + 15 <= jmax; the loop is split into head, middle and
    // tail loops around them (a per-chunk branch made the register
    // allocator copy the ring at every merge, waiting for its loads)
    const int cf0 = 2, cf1 = (jmax - 31) >= 0 ? (jmax - 31) >> 5 : -1;  // [cf0, cf1]
    const int cm0 = cf1 >= cf0 ? cf0 : nc, cm1 = cf1 >= cf0 ? (cf1 + 1 < nc ? cf1 + 1 : nc) : nc;
    auto run = [&](auto FIRSTc) {
#pragma unroll
        for (int g = 0; g < R; ++g) P[g] = D[g] = X[g] = f4v{0.f, 0.f, 0.f, 0.f};
        w = 0.f;  // column 0 (boundary)
        vprev = 0.f;
        for (int c = -1; c < cm0; ++c) {
            chunk(H0{}, F0{}, FIRSTc, 2 * c);
            chunk(H1{}, F0{}, FIRSTc, 2 * c + 1);
        }
        for (int c = cm0; c < cm1; ++c) {
            chunk(H0{}, T1{}, FIRSTc, 2 * c);
            chunk(H1{}, T1{}, FIRSTc, 2 * c + 1);
        }
        for (int c = cm1; c < nc; ++c) {
            chunk(H0{}, F0{}, FIRSTc, 2 * c);
            chunk(H1{}, F0{}, FIRSTc, 2 * c + 1);
        }
    };
    if constexpr (MC) {
        run(T1{});
        // every group stored and complete (a release: waits for the stores)
        if (lane == 0)
            __hip_atomic_store(sa.prog + m, ((unsigned long long)sa.epoch << 32) | 0x7fffffffull, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
    } else {
        if (wv == 0)
            run(T1{});
        else
            run(F0{});
    }
}

__global__ __launch_bounds__(256) void k_lex_gs_skew(SkewArgs sa) {
    extern __shared__ float lex_rows[];  // [waves][lex_skew_rsl]: wave w's last-lane results, column c at c + 64
    __shared__ int flags[kSkewWaves];    // 16-step chunks wave w's last lane has published
    const int nw = blockDim.x >> 6, lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nb = lex_skew_blocks(sa.ny);
    for (int b0 = 0; b0 < nb; b0 += nw) {
        __threadfence();  // the band before is final and visible (a band's first wave reads its last row)
        __syncthreads();
        if ((int)threadIdx.x < nw) __hip_atomic_store(&flags[threadIdx.x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        const int m = b0 + wv;
        if (m >= nb) continue;  // wave-uniform
        lex_skew_wave<false>(sa, m, wv, nw, lane, lex_rows, flags);
    }
}

// one block per workgroup (the dynamic LDS the launch asks for keeps at most
// two such workgroups on a CU)
__global__ __launch_bounds__(64) void k_lex_gs_skew_mc(SkewArgs sa) {
    lex_skew_wave<true>(sa, (int)blockIdx.x, 0, 1, (int)threadIdx.x, nullptr, nullptr);
}

// u[1:-1,1:-1] -= grad_x[1:-1,1:-1] (no dt: v5.py:255-256)
__global__ void k_sub_gradient(const float *__restrict__ phi, float *__restrict__ u,
                               float *__restrict__ v, int ny, int nx, float cx, float cy) {
    CFD_2D_INDEX
    if (!interior(i, j, ny, nx)) return;
    const float a = (phi[c + 1] - phi[c - 1]) * cx;
    const float b = (phi[c + nx] - phi[c - nx]) * cy;
    u[c] = u[c] - a;
    v[c] = v[c] - b;
}

// apply_boundary_conditions, v5.py:349-360.  Net effect of the eight
// assignments in order: rows 0 and ny-1 end at 0; other rows get the inlet
// u = f32(V_inf*(1 + pert_scale*sin(2*pi*y/y_max + 0.02*step))), v = 0 at
// x = 0 and a zero-gradient outlet copy from x = nx-2.
__global__ void k_bc(float *__restrict__ u, float *__restrict__ v, const double *__restrict__ y,
                     int ny, int nx, double y_max, double v_inf, int step) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nx) {  // top / bottom rows
        u[t] = 0.0f;
        v[t] = 0.0f;
        u[(size_t)(ny - 1) * nx + t] = 0.0f;
        v[(size_t)(ny - 1) * nx + t] = 0.0f;
    }
    const int i = t;
    if (i >= 1 && i < ny - 1) {
        const double s = (double)step;
        double scale = s / 1000.0;
        scale = (1.0 < scale ? 1.0 : scale) * 0.01;
        const double two_pi = 2.0 * 3.141592653589793;
        const double pert = scale * sin(two_pi * y[i] / y_max + 0.02 * s);
        const size_t r = (size_t)i * nx;
        u[r] = (float)(v_inf * (1.0 + pert));
        v[r] = 0.0f;
        u[r + nx - 1] = u[r + nx - 2];
        v[r + nx - 1] = v[r + nx - 2];
    }
}

// Lid-driven cavity walls (BASELINE config 1; the reference has no
// incompressible cavity, so the walls follow the assignment pattern of
// v5.py:349-360): no-slip u = v = 0 on the left, right and bottom walls, the
// lid u = u_lid, v = 0 on the top row y = y_max (row ny-1), the lid written
// last so it owns the two top corners.
__global__ void k_lid_bc(float *__restrict__ u, float *__restrict__ v, int ny, int nx, float u_lid) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ny - 1) {  // side walls, rows 0 .. ny-2
        const size_t r = (size_t)t * nx;
        u[r] = 0.0f;
        v[r] = 0.0f;
        u[r + nx - 1] = 0.0f;
        v[r + nx - 1] = 0.0f;
    }
    if (t < nx) {
        u[t] = 0.0f;  // bottom wall
        v[t] = 0.0f;
        u[(size_t)(ny - 1) * nx + t] = u_lid;  // lid
        v[(size_t)(ny - 1) * nx + t] = 0.0f;
    }
}

// apply_ibm_fast, v5.py:228-237 (float64 mask => float64 arithmetic)
__global__ void k_ibm(float *__restrict__ u, float *__restrict__ v, const double *__restrict__ m,
                      int n, double fs) {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
        const double mv = m[c];
        if (mv > 0.0) {
            const double f = 1.0 - mv * fs;
            u[c] = (float)((double)u[c] * f);
            v[c] = (float)((double)v[c] * f);
        }
    }
}

__global__ void k_clip(float *__restrict__ a, size_t n, float lo, float hi) {
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n;
         c += (size_t)gridDim.x * blockDim.x) {
        const float x = a[c];
        a[c] = x < lo ? lo : (x > hi ? hi : x);  // NaN passes through like np.clip
    }
}

// ------------------------------------------------------------ reductions
__global__ void k_absmax(const float *__restrict__ a, const float *__restrict__ b, size_t n,
                         float *out) {
    float m = 0.0f;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n;
         c += (size_t)gridDim.x * blockDim.x) {
        float x = fabsf(a[c]);
        if (x > m) m = x;
        if (b) {
            x = fabsf(b[c]);
            if (x > m) m = x;
        }
    }
    wave_reduce_max_store(m, out);
}

// mean of 0.5*(u^2 + v^2) (v5.py:362-363, :431-432); each cell's energy in
// float32 like NumPy, the sum in float64.
__global__ void k_energy_sum(const float *__restrict__ u, const float *__restrict__ v, size_t n,
                             double *out) {
    double s = 0.0;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n;
         c += (size_t)gridDim.x * blockDim.x) {
        const float e = 0.5f * (u[c] * u[c] + v[c] * v[c]);
        s += (double)e;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, kWave);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

__global__ void k_scale_double(double *p, double f) { *p = *p * f; }

// compute_vorticity + nanmax(|w|), v5.py:365-373, :427-428: masked cells are
// NaN (skipped), the boundary ring is 0.
__global__ void k_vort_absmax(const float *__restrict__ u, const float *__restrict__ v,
                              const uint8_t *__restrict__ mask, int ny, int nx, float dx2,
                              float dy2, float *out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    float m = 0.0f;
    if (j < nx) {
        const size_t c = (size_t)i * nx + j;
        if (interior(i, j, ny, nx) && !(mask && mask[c])) {
            const float w = (v[c + 1] - v[c - 1]) / dx2 - (u[c + nx] - u[c - nx]) / dy2;
            const float a = fabsf(w);
            if (a > m) m = a;
        }
    }
    wave_reduce_max_store(m, out);
}

// compute_vorticity, v5.py:365-373: interior central differences, boundary
// ring 0, masked cells NaN.
__global__ void k_vorticity(const float *__restrict__ u, const float *__restrict__ v,
                            const uint8_t *__restrict__ mask, float *__restrict__ w, int ny,
                            int nx, float dx2, float dy2) {
    CFD_2D_INDEX
    float r = 0.0f;
    if (interior(i, j, ny, nx)) r = (v[c + 1] - v[c - 1]) / dx2 - (u[c + nx] - u[c - nx]) / dy2;
    if (mask && mask[c]) r = __builtin_nanf("");
    w[c] = r;
}

__global__ void k_nonfinite(const float *__restrict__ a, const float *__restrict__ b, size_t n,
                            int *out) {
    int cnt = 0;
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n;
         c += (size_t)gridDim.x * blockDim.x) {
        cnt += !isfinite(a[c]);
        if (b) cnt += !isfinite(b[c]);
    }
    if (cnt) atomicAdd(out, cnt);
}

// NumPy float32 scalar power (glibc powf, libm_powf.hpp) elementwise: the
// parity hook for the device powf the SUPG tau uses -- at y = 2 and 0.5 the
// exact-path forms it calls (powf_sq / powf_sqrt), else the restatement.
__global__ void k_numpy_powf(const float *__restrict__ x, float y, float *__restrict__ out, size_t n) {
    for (size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x; c < n;
         c += (size_t)gridDim.x * blockDim.x)
        out[c] = y == 2.0f ? libm::powf_sq(x[c]) : (y == 0.5f ? libm::powf_sqrt(x[c]) : libm::powf(x[c], y));
}

static dim3 grid2d(int ny, int nx) { return dim3(ceil_div(nx, 256), ny); }

static thread_local int g_last_pred[3] = {-1, 0, 0};
void set_last_predictor(int path, int tau, int vec) {
    g_last_pred[0] = path;
    g_last_pred[1] = tau;
    g_last_pred[2] = vec;
}
int pred_rows_resident(const void *f) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, f);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 256, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, 256, 0) != hipSuccess || per < 1) per = 1;
    return cache[key] = per * cus;
}
static int grid1d(size_t n) {
    long b = (long)((n + 255) / 256);
    if (b > 2048) b = 2048;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace cfd

using namespace cfd;

#define CFD_SHAPE2D(ny, nx) CFD_REQUIRE((ny) >= 1 && (nx) >= 1, "bad 2-D shape (%d, %d)", ny, nx)

extern "C" {

int cfd_supg_tau2d_f32(const float *u, const float *v, const float *nu_eff, float nu_eff_scalar,
                       float *tau, int ny, int nx, double dx, double dy, float dt, void *stream) {
    CFD_REQUIRE(u && v && tau, "supg_tau2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_supg_tau, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, nu_eff,
                       nu_eff_scalar, tau, ny, nx, dt, make_pred_const(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_convection_supg2d_f32(const float *u, const float *v, const float *phi, const float *tau,
                              float *conv, int ny, int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && phi && tau && conv, "convection_supg2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_conv_supg, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, phi, tau,
                       conv, ny, nx, make_pred_const(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_convection_upwind2d_f32(const float *u, const float *v, const float *phi, float *conv,
                                int ny, int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && phi && conv, "convection_upwind2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_conv_upwind, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, phi,
                       conv, ny, nx, make_pred_const(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_laplacian2d_f32(const float *phi, const float *nu_eff, float nu_eff_scalar, float *lap,
                        int ny, int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(phi && lap, "laplacian2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_laplacian, grid2d(ny, nx), dim3(256), 0, as_stream(stream), phi, nu_eff,
                       nu_eff_scalar, lap, ny, nx, make_pred_const(dx, dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_predictor2d_f32(const float *u, const float *v, const float *nu_eff, float nu_eff_scalar,
                        float *u_star, float *v_star, float *tau, int ny, int nx, double dx,
                        double dy, float dt, int use_supg, void *stream) {
    CFD_REQUIRE(u && v && u_star && v_star, "predictor2d: null pointer");
    CFD_REQUIRE(u_star != u && v_star != v && u_star != v && v_star != u,
                "predictor2d: outputs must not alias inputs");
    CFD_SHAPE2D(ny, nx);
    const PredConst k = make_pred_const(dx, dy);
    hipStream_t s = as_stream(stream);
    // cells per lane of the row march: the preferred count (tuning; default
    // 2), halved until nx and every array's alignment allow it (1 always does)
    int vec = tuning().pred_vec ? tuning().pred_vec : 2;
    auto fits = [&](int w) {
        const uintptr_t m = (uintptr_t)(4 * w - 1);
        auto al = [&](const void *p_) { return !p_ || ((uintptr_t)p_ & m) == 0; };
        return nx % w == 0 && al(u) && al(v) && al(u_star) && al(v_star) && al(tau) && al(nu_eff);
    };
    while (vec > 1 && !fits(vec)) vec /= 2;
    const bool rows_ok = (size_t)ny * nx * sizeof(float) < ((size_t)1 << 31);
    const int tau_mode = use_supg ? tuning().pred_tau : kTauExact;
    const int tk = timing_begin(s, kTimingPredictor);
    if (tuning().pred_variant != 1 && rows_ok) {
        PredRowArgs<float> a;
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
        a.k = k;
        CFD_CHECK_HIP(pred_rows_launch<float>(a, use_supg != 0, tau_mode, vec, tuning().pred_rows, s));
        set_last_predictor(1, tau_mode, vec);
    } else if (use_supg) {
        hipLaunchKernelGGL(k_predictor<true>, grid2d(ny, nx), dim3(256), 0, s, u, v, nu_eff, nu_eff_scalar, u_star,
                           v_star, tau, ny, nx, dt, k);
        set_last_predictor(0, kTauExact, 1);
    } else {
        hipLaunchKernelGGL(k_predictor<false>, grid2d(ny, nx), dim3(256), 0, s, u, v, nu_eff, nu_eff_scalar, u_star,
                           v_star, tau, ny, nx, dt, k);
        set_last_predictor(0, kTauExact, 1);
    }
    timing_end(tk, s, 1);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

// 0: auto (row march when the shape allows it), 1: one thread per cell
// (k_predictor), 2: row march; rows per chunk (0: auto); cells per lane
// (0: auto, 1, 2, 4)
int cfd_set_predictor2d_tau_mode(int mode) {
    CFD_REQUIRE(mode == kTauExact || mode == kTauFast, "predictor2d tau mode: 0 (exact) or 1 (fast)");
    tuning().pred_tau = mode;
    return CFD_OK;
}

int cfd_get_predictor2d_tau_mode(void) { return tuning().pred_tau; }

int cfd_get_last_predictor2d_path(int *tau_mode, int *cells_per_lane) {
    if (tau_mode) *tau_mode = g_last_pred[1];
    if (cells_per_lane) *cells_per_lane = g_last_pred[2];
    return g_last_pred[0];
}

int cfd_set_predictor2d_config(int variant, int rows, int cells_per_lane) {
    CFD_REQUIRE(variant >= 0 && variant <= 2 && rows >= 0, "predictor2d config: variant 0..2, rows >= 0");
    CFD_REQUIRE(cells_per_lane == 0 || cells_per_lane == 1 || cells_per_lane == 2 || cells_per_lane == 4,
                "predictor2d config: cells per lane 0 (auto), 1, 2 or 4");
    tuning().pred_variant = variant;
    tuning().pred_rows = rows;
    tuning().pred_vec = cells_per_lane;
    return CFD_OK;
}

int cfd_divergence2d_f32(const float *u, const float *v, float *div, int ny, int nx, double dx,
                         double dy, float *absmax, void *stream) {
    CFD_REQUIRE(u && v && div, "divergence2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_divergence, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, div, ny,
                       nx, (float)(0.5 / dx), (float)(0.5 / dy), absmax);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_gradient2d_f32(const float *phi, float *grad_x, float *grad_y, int ny, int nx, double dx,
                       double dy, void *stream) {
    CFD_REQUIRE(phi && grad_x && grad_y, "gradient2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_gradient, grid2d(ny, nx), dim3(256), 0, as_stream(stream), phi, grad_x,
                       grad_y, ny, nx, (float)(0.5 / dx), (float)(0.5 / dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_project2d_f32(const float *phi, const float *u_star, const float *v_star, float *u,
                      float *v, int ny, int nx, double dx, double dy, float dt, float *gradmax,
                      void *stream) {
    CFD_REQUIRE(phi && u_star && v_star && u && v, "project2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_project, grid2d(ny, nx), dim3(256), 0, as_stream(stream), phi, u_star,
                       v_star, u, v, ny, nx, (float)(0.5 / dx), (float)(0.5 / dy), dt, gradmax);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

size_t cfd_clean_divergence_workspace_bytes(int ny, int nx) {
    // scratch fields: phi and div row-major float64 (cfd_clean_divergence2d_f64)
    // or div and two phi in the skewed float32 layout of k_lex_gs_skew,
    // whichever is larger
    const size_t n = (size_t)(ny > 0 ? ny : 0) * (size_t)(nx > 0 ? nx : 0);
    const size_t skew = ny > 2 && nx > 2 ? lex_skew_prog_offset(ny, nx) + 8 * (size_t)lex_skew_blocks(ny) : 0;
    return 2 * sizeof(double) * n > skew ? 2 * sizeof(double) * n : skew;
}

int cfd_clean_divergence2d_f32(float *u, float *v, int ny, int nx, double dx, double dy,
                               int iterations, void *ws, void *stream) {
    CFD_REQUIRE(u && v && ws, "clean_divergence2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipStream_t s = as_stream(stream);
    const size_t n = (size_t)ny * nx;
    float *phi = reinterpret_cast<float *>(ws);
    float *div = phi + n;
    const double dx2_inv = 1.0 / (dx * dx), dy2_inv = 1.0 / (dy * dy);
    const double denom_inv = 1.0 / (2.0 * (dx2_inv + dy2_inv));
    const float cx = (float)(0.5 / dx), cy = (float)(0.5 / dy);
    if (ny > 2 && nx > 2 && 2 * lex_skew_floats(ny, nx) * 4 < ((size_t)1 << 31)) {
        // div and two phi buffers in the skewed layout (k_lex_gs_skew): the
        // first sweep starts from phi = 0 (np.zeros_like, v5.py:242) by
        // reading nothing; at iterations == 2 the second sweep writes the
        // second buffer, so both gradients are subtracted in one pass
        const size_t F = lex_skew_floats(ny, nx);
        float *div_s = reinterpret_cast<float *>(ws);
        float *phi1 = div_s + F, *phi2 = phi1 + F;
        const int pbytes = (int)(2 * F * sizeof(float));
        const size_t ldsmax = kLexLdsMax - 1024;
        static const int wmax = [] {
            const char *e = getenv("CFD_LEX_SKEW_WAVES");  // A/B knob: waves per band (1 .. 4)
            const int v = e ? atoi(e) : kSkewWaves;
            return v >= 1 && v <= kSkewWaves ? v : kSkewWaves;
        }();
        int nw = lex_skew_blocks(ny) < wmax ? lex_skew_blocks(ny) : wmax;
        while (nw > 1 && lex_skew_lds_bytes(nw, nx) > ldsmax) --nw;
        // one wave per band neither publishes nor reads a row through LDS (no
        // wave below it, and a band's first wave takes the row above from
        // memory): no dynamic LDS, whatever nx (short, very wide grids)
        const size_t lds = nw > 1 ? lex_skew_lds_bytes(nw, nx) : 0;
        static bool attr_s = false;
        if (!attr_s) {
            CFD_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(k_lex_gs_skew),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsmax));
            attr_s = true;
        }
        // past one band, one block per workgroup (k_lex_gs_skew_mc) up to
        // kSkewMcBlocks blocks: the bands ran one after another on one CU.
        // Within one band the single workgroup stays: the multi-CU wave is
        // ~10 % slower per step (sc1 stores, the polls) and lags its
        // neighbour by ~160 steps (r05: 600 x 180 87 -> 89 us per call with
        // it, 1026^2 504 -> 403 us)
        const int nbk = lex_skew_blocks(ny);
        static const int mc_on = [] {
            const char *e = getenv("CFD_LEX_SKEW_MC");  // A/B knob: 0 = the banded single-workgroup sweep
            return e ? atoi(e) : 1;
        }();
        const bool mc = mc_on && nbk > kSkewWaves && nbk <= kSkewMcBlocks;
        if (mc) {
            static bool attr_mc = false;
            if (!attr_mc) {
                CFD_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(k_lex_gs_skew_mc),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSkewMcLds));
                attr_mc = true;
            }
        }
        SkewArgs sa;
        sa.phi_base = phi1;
        sa.div_s = div_s;
        sa.prog = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(ws) + lex_skew_prog_offset(ny, nx));
        sa.fail = mc ? persist_fail_word(s) : nullptr;
        sa.poll_ticks = persist_poll_ticks();
        sa.phi_bytes = pbytes;
        sa.ny = ny;
        sa.nx = nx;
        sa.cx = (float)dx2_inv;
        sa.cy = (float)dy2_inv;
        sa.cd = (float)denom_inv;
        auto sweep = [&](int old_off, int new_off) {
            sa.old_off = old_off;
            sa.new_off = new_off;
            if (mc) {
                static std::atomic<unsigned> epoch{0};
                unsigned e = epoch.fetch_add(1) + 1;
                if (e == 0) e = epoch.fetch_add(1) + 1;
                sa.epoch = e;
                hipLaunchKernelGGL(k_lex_gs_skew_mc, dim3(nbk), dim3(64), kSkewMcLds, s, sa);
            } else {
                hipLaunchKernelGGL(k_lex_gs_skew, dim3(1), dim3(64 * nw), lds, s, sa);
            }
        };
        const dim3 gr(ceil_div(nx, 256), ny - 2);
        if (iterations >= 1) {
            hipLaunchKernelGGL(k_divergence_skew, dim3(gr.x, ny - 1), dim3(256), 0, s, u, v, div_s, phi1, ny, nx, cx,
                               cy);
            sweep((int)kOob, 0);
        }
        if (iterations == 2) {
            hipLaunchKernelGGL(k_divergence2_skew, gr, dim3(256), 0, s, u, v, phi1, div_s, ny, nx, cx, cy);
            sweep(0, (int)(F * sizeof(float)));
            hipLaunchKernelGGL(k_sub_gradient2_skew, grid2d(ny, nx), dim3(256), 0, s, phi1, phi2, u, v, ny, nx, cx,
                               cy);
        } else if (iterations >= 1) {
            hipLaunchKernelGGL(k_sub_gradient_skew, grid2d(ny, nx), dim3(256), 0, s, phi1, u, v, ny, nx, cx, cy);
            for (int it = 1; it < iterations; ++it) {  // in place on phi1
                hipLaunchKernelGGL(k_divergence_skew, gr, dim3(256), 0, s, u, v, div_s, (float *)nullptr, ny, nx, cx,
                                   cy);
                sweep(0, 0);
                hipLaunchKernelGGL(k_sub_gradient_skew, grid2d(ny, nx), dim3(256), 0, s, phi1, u, v, ny, nx, cx, cy);
            }
        }
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    CFD_CHECK_HIP(hipMemsetAsync(phi, 0, n * sizeof(float), s));  // np.zeros_like (v5.py:242)
    for (int it = 0; it < iterations; ++it) {
        hipLaunchKernelGGL(k_divergence, grid2d(ny, nx), dim3(256), 0, s, u, v, div, ny, nx, cx, cy,
                           (float *)nullptr);
        if (ny > 2 && nx > 2)  // past the skewed layout's 2^31-byte offsets: the plain wavefront
            hipLaunchKernelGGL(k_lex_gs_sweep, dim3(1), dim3(ny - 2 >= 1024 ? 1024 : 64 * ceil_div(ny - 2, 64)), 0, s,
                               phi, div, ny, nx, (float)dx2_inv, (float)dy2_inv, (float)denom_inv);
        hipLaunchKernelGGL(k_sub_gradient, grid2d(ny, nx), dim3(256), 0, s, phi, u, v, ny, nx, cx,
                           cy);
        CFD_LAUNCH_CHECK();
    }
    return CFD_OK;
}

int cfd_apply_bc2d_f32(float *u, float *v, const double *y, int ny, int nx, double y_max,
                       double v_inf, int step, void *stream) {
    CFD_REQUIRE(u && v && y, "apply_bc2d: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_bc2d: grid must be at least 2x2");
    const int n = ny > nx ? ny : nx;
    hipLaunchKernelGGL(k_bc, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), u, v, y, ny,
                       nx, y_max, v_inf, step);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_apply_lid_bc2d_f32(float *u, float *v, int ny, int nx, float u_lid, void *stream) {
    CFD_REQUIRE(u && v, "apply_lid_bc2d: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_lid_bc2d: grid must be at least 2x2");
    const int n = ny > nx ? ny : nx;
    hipLaunchKernelGGL(k_lid_bc, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), u, v, ny, nx, u_lid);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_apply_ibm2d_f32(float *u, float *v, const double *ibm_mask, int n, double force_strength,
                        void *stream) {
    CFD_REQUIRE(u && v && ibm_mask && n >= 0, "apply_ibm2d: bad arguments");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_ibm, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), u, v, ibm_mask, n,
                       force_strength);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_clip_f32(float *a, size_t n, float lo, float hi, void *stream) {
    CFD_REQUIRE(a, "clip: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_clip, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), a, n, lo, hi);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_absmax_f32(const float *a, size_t n, float *out, void *stream) {
    CFD_REQUIRE(a && out, "absmax: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_absmax, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), a,
                       (const float *)nullptr, n, out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_absmax2_f32(const float *a, const float *b, size_t n, float *out, void *stream) {
    CFD_REQUIRE(a && b && out, "absmax2: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_absmax, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), a, b, n, out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_energy_mean2d_f32(const float *u, const float *v, size_t n, double *out, void *stream) {
    CFD_REQUIRE(u && v && out && n > 0, "energy_mean2d: bad arguments");
    hipStream_t s = as_stream(stream);
    if (n <= kEnergyOneBlock) {
        if (unsigned *ws = energy_scratch(s))
            hipLaunchKernelGGL((k_energy_mean_mb<float, false>), dim3(kEnergyBlocks), dim3(256), 0, s,
                               const_cast<float *>(u), const_cast<float *>(v), n, out, float(0), float(0), ws);
        else
            hipLaunchKernelGGL((k_energy_mean_1blk<float, false>), dim3(1), dim3(1024), 0, s, const_cast<float *>(u),
                               const_cast<float *>(v), n, out, float(0), float(0));
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    CFD_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(double), s));
    hipLaunchKernelGGL(k_energy_sum, dim3(grid1d(n)), dim3(256), 0, s, u, v, n, out);
    hipLaunchKernelGGL(k_scale_double, dim3(1), dim3(1), 0, s, out, 1.0 / (double)n);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_energy_mean_clip2d_f32(float *u, float *v, size_t n, double *out, float lo, float hi, void *stream) {
    CFD_REQUIRE(u && v && out && n > 0, "energy_mean_clip2d_f32: bad arguments");
    hipStream_t s = as_stream(stream);
    if (n <= kEnergyOneBlock) {
        if (unsigned *ws = energy_scratch(s))
            hipLaunchKernelGGL((k_energy_mean_mb<float, true>), dim3(kEnergyBlocks), dim3(256), 0, s, u, v, n, out,
                               lo, hi, ws);
        else
            hipLaunchKernelGGL((k_energy_mean_1blk<float, true>), dim3(1), dim3(1024), 0, s, u, v, n, out, lo, hi);
        CFD_LAUNCH_CHECK();
        return CFD_OK;
    }
    int rc = cfd_energy_mean2d_f32(u, v, n, out, stream);
    if (!rc) rc = cfd_clip_f32(u, n, lo, hi, stream);
    if (!rc) rc = cfd_clip_f32(v, n, lo, hi, stream);
    return rc;
}

int cfd_apply_bc_ibm2d_f32(float *u, float *v, const double *y, int ny, int nx, double y_max, double v_inf, int step,
                           const double *ibm_mask, double force_strength, void *stream) {
    CFD_REQUIRE(u && v && y, "apply_bc_ibm2d_f32: null pointer");
    CFD_REQUIRE(ny >= 2 && nx >= 2, "apply_bc_ibm2d_f32: grid must be at least 2x2");
    int blocks = ceil_div(ny > nx ? ny : nx, 256);
    if (ibm_mask) {
        const int g = grid1d((size_t)ny * nx);
        if (g > blocks) blocks = g;
    }
    hipLaunchKernelGGL(k_bc_ibm<float>, dim3(blocks), dim3(256), 0, as_stream(stream), u, v, y, ibm_mask, ny, nx,
                       y_max, v_inf, step, force_strength);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_vorticity_absmax2d_f32(const float *u, const float *v, const uint8_t *mask, int ny, int nx,
                               double dx, double dy, float *out, void *stream) {
    CFD_REQUIRE(u && v && out, "vorticity_absmax2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_vort_absmax, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, mask,
                       ny, nx, (float)(2.0 * dx), (float)(2.0 * dy), out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_vorticity2d_f32(const float *u, const float *v, const uint8_t *mask, float *w, int ny,
                        int nx, double dx, double dy, void *stream) {
    CFD_REQUIRE(u && v && w, "vorticity2d: null pointer");
    CFD_SHAPE2D(ny, nx);
    hipLaunchKernelGGL(k_vorticity, grid2d(ny, nx), dim3(256), 0, as_stream(stream), u, v, mask, w,
                       ny, nx, (float)(2.0 * dx), (float)(2.0 * dy));
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_numpy_powf_f32(const float *x, float y, float *out, size_t n, void *stream) {
    CFD_REQUIRE(x && out, "numpy_powf: null pointer");
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_numpy_powf, dim3(grid1d(n)), dim3(256), 0, as_stream(stream), x, y, out, n);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int cfd_nonfinite_count_f32(const float *a, const float *b, size_t n, int *out, void *stream) {
    CFD_REQUIRE(a && out, "nonfinite_count: null pointer");
    hipStream_t s = as_stream(stream);
    CFD_CHECK_HIP(hipMemsetAsync(out, 0, sizeof(int), s));
    if (n == 0) return CFD_OK;
    hipLaunchKernelGGL(k_nonfinite, dim3(grid1d(n)), dim3(256), 0, s, a, b, n, out);
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // extern "C"

#ifdef CFD_PRED_COUNT
// measurement aid (a -DCFD_PRED_COUNT build only): cells the row march queued
extern "C" unsigned long long cfd_debug_pred_count(int reset) {
    unsigned long long h = 0;
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(&h, HIP_SYMBOL(cfd::g_pred_count), sizeof(h));
    if (reset) {
        const unsigned long long z = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(cfd::g_pred_count), &z, sizeof(z));
    }
    return h;
}
#endif
