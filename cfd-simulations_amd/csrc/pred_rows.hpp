// pred_rows.hpp -- the fused advection-diffusion predictor (v5.py:388-403:
// compute_supg_stabilization_fast :149-162, compute_convection_supg_fast
// :127-147, compute_convection_fast :112-125, compute_laplacian_fast
// :164-176) as a row march over float or double fields, and the per-cell
// stencil pieces it shares with the one-thread-per-cell kernels.
//
// Row march.  One wave owns a segment of 64 * VEC columns (64 lanes x VEC
// adjacent cells) and marches down a chunk of rows.  Rows i-1, i, i+1 of u and
// v sit in registers (row i+2 is in flight: each row is loaded once, one
// coalesced 64 * VEC * sizeof(T) load per field, two steps ahead), rotated at
// the end of a step.  y-neighbours are the other rows, x-neighbours the lane's
// own cells plus DPP wave shifts for its first and last cell; the two columns
// just outside the segment arrive as one load per row and field (lane 0:
// column xs - 1, lane 63: column xs + 64 VEC) and enter the shifts as their
// `old` operand.  The four waves of a workgroup take four adjacent segments;
// workgroups are dealt chunk by chunk, XCD-swizzled, so the two halo rows a
// chunk shares with its neighbours are read from the same L2.  u*, v* and tau
// leave as streaming stores.  HBM: u, v read once (+2 halo rows per chunk),
// u*, v*, tau written once: 20 B per float cell, 40 B per double cell (16 / 32
// without tau).
//
// tau modes (cfd_set_predictor2d_tau_mode):
// * kTauExact (default): |V| = (u**2 + v**2)**0.5 as the reference's NumPy
//   scalar `**` computes it, i.e. glibc's powf / pow, so the predictor and the
//   whole time_step are bit-exact against the reference fixtures.
//   - float: proven fast paths (libm_powf.hpp: powf_sq_fast / powf_sqrt_fast,
//     equal to glibc's powf unless near a rounding midpoint) and div_fast for
//     the two divisions; an operation whose check fails (~1.25 % of cells on
//     O(1) data) is re-done exactly in the march by the lane that needs it
//     (the squares, then the roots, through a wave-uniform loop that runs one
//     glibc powf per pass for every lane with a job left, tables in LDS; a
//     failed division takes the IEEE divide).  Each output is written once.
//   - double: glibc's pow for every square and root (libm_pow.hpp, tables in
//     LDS), IEEE divisions.
// * kTauFast: the compiled reference's arithmetic (@njit(fastmath=True):
//   x**2 -> x*x, **0.5 -> sqrt): |V| = sqrt(u*u + v*v) correctly rounded, the
//   two divisions of tau on v_rcp_f32 + one Newton step (float) / IEEE
//   (double), no proofs, no fallbacks.  Within north_star's 1e-6 relative
//   L-infinity of the exact mode (tests/test_gpu_predictor.py measures it).
// Everything else is k_predictor's arithmetic operation for operation, so the
// exact mode is bit-identical to the per-cell kernels.
#pragma once
#include "common.hpp"
#include "libm_pow.hpp"
#include "libm_powf.hpp"

namespace cfd {

enum PredTau { kTauExact = 0, kTauFast = 1 };

// stencil constants (Python floats rounded to T where they meet T data, NEP 50)
template <typename T>
struct PredK {
    T c1x, c1y;  // SUPG first derivative: 0.5 * (0.5/dx)   (v5.py:131,137)
    T c2x, c2y;  // SUPG second derivative: (0.5/dx)^2       (v5.py:141)
    T ux, uy;    // upwind: 1/dx                              (v5.py:116)
    T lx, ly;    // laplacian: 1/(dx*dx)                      (v5.py:168)
    T h;         // min(dx, dy)                               (v5.py:156)
    T eps;       // 1e-10                                     (v5.py:157,160)
};
template <typename T>
inline PredK<T> make_pred_k(double dx, double dy) {
    PredK<T> k;
    const double sdx = 0.5 / dx, sdy = 0.5 / dy;
    k.c1x = (T)(0.5 * sdx);
    k.c1y = (T)(0.5 * sdy);
    k.c2x = (T)(sdx * sdx);
    k.c2y = (T)(sdy * sdy);
    k.ux = (T)(1.0 / dx);
    k.uy = (T)(1.0 / dy);
    k.lx = (T)(1.0 / (dx * dx));
    k.ly = (T)(1.0 / (dy * dy));
    k.h = (T)(dx < dy ? dx : dy);
    k.eps = (T)1e-10;
    return k;
}

// tau from |V| already formed (v5.py:156-161), IEEE divisions; branch-free
// (both sides formed, one selected) so a march can interleave its cells
template <typename T>
__device__ inline T supg_tau_vm(T vm, T nu, T dt, const PredK<T> &k) {
    const T pe = (vm * k.h) / (nu + k.eps);
    const T half = pe / T(2);
    const T lim = half < T(1) ? half : T(1);  // Python min(1.0, Pe/2.0)
    T t = (k.h / (T(2) * vm)) * lim;
    asm volatile("" : "+v"(t));  // keeps the divisions out of a branch on vm > eps
    return vm > k.eps ? t : dt / T(2);
}

// compute_convection_supg_fast body, v5.py:135-146
template <typename T>
__device__ inline T conv_supg(T uc, T vc, T C, T E, T W, T N, T S, T t, const PredK<T> &k) {
    const T ddx = (E - W) * k.c1x;
    const T ddy = (N - S) * k.c1y;
    const T cs = uc * ddx + vc * ddy;
    if (t > T(0)) {
        const T d2x = ((E - T(2) * C) + W) * k.c2x;
        const T d2y = ((N - T(2) * C) + S) * k.c2y;
        return cs - t * (uc * d2x + vc * d2y);
    }
    return cs;
}
// the same without the branch on t > 0 (both forms, one selected; the asm
// keeps the compiler from sinking the second-derivative part into a branch)
template <typename T>
__device__ inline T conv_supg_sel(T uc, T vc, T C, T E, T W, T N, T S, T t, const PredK<T> &k) {
    const T ddx = (E - W) * k.c1x;
    const T ddy = (N - S) * k.c1y;
    const T cs = uc * ddx + vc * ddy;
    const T d2x = ((E - T(2) * C) + W) * k.c2x;
    const T d2y = ((N - T(2) * C) + S) * k.c2y;
    T cd = cs - t * (uc * d2x + vc * d2y);
    asm volatile("" : "+v"(cd));
    return t > T(0) ? cd : cs;
}
// compute_convection_fast body (first-order upwind), v5.py:120-124
template <typename T>
__device__ inline T conv_upwind(T uc, T vc, T C, T E, T W, T N, T S, const PredK<T> &k) {
    const T ddx = uc > T(0) ? (C - W) * k.ux : (E - C) * k.ux;
    const T ddy = vc > T(0) ? (C - S) * k.uy : (N - C) * k.uy;
    return uc * ddx + vc * ddy;
}
// compute_laplacian_fast body, v5.py:172-175
template <typename T>
__device__ inline T laplacian(T nu, T C, T E, T W, T N, T S, const PredK<T> &k) {
    const T l1 = ((E - T(2) * C) + W) * k.lx;
    const T l2 = ((N - T(2) * C) + S) * k.ly;
    return nu * (l1 + l2);
}

// a / b, correctly rounded, from rb ~ 1/b (v_rcp_f32) and one Newton step:
// q1 = q0 + (a - q0 b) rb.  With the exact residual r = a - q1 b (one fma),
// a/b = q1 + r/b, so |r| < |b| ulp(q1) / 2 proves q1 = RN(a/b) (the ulp taken
// below q1's last bit, as in powf_sq_fast: the lower binade's for a power of
// two).  The test is |r| < RN(ub * kDivT) with ub = |b| 2^e exact (2^e: q1's
// power of two below its last bit, so ulp = 2^(e - 23)):
// kDivT = RN((1/2 - 2^-20) 2^-23) and the product's rounding add at most
// (1 + 2^-24)^2 < 1 + 2^-21 to (1/2 - 2^-20), so the bound stays below
// |b| ulp / 2.  The guards keep every quantity normal: |b|, |q1| >= 2^-100 and
// ub (~ |a|) in [2^-100, 2^100] (the bound then >= 2^-124; the residual's
// granularity ulp(q1) ulp(b) ~ ub 2^-46 is representable: r is exact whenever
// q1 is within an ulp of a/b, and a q1 farther off leaves |r| above the bound).
// False otherwise (near a midpoint, tiny or huge operands, inf, NaN): the
// caller takes the IEEE division.
constexpr float kDivT = (float)((0.5 - 0x1p-20) * 0x1p-23);
__device__ inline float div_nr(float a, float b, float rb) {
    const float q0 = a * rb;
    return __builtin_fmaf(__builtin_fmaf(-q0, b, a), rb, q0);
}
__device__ inline bool div_fast(float a, float b, float rb, float &q) {
    const float q1 = div_nr(a, b, rb);
    const float r = __builtin_fmaf(-q1, b, a);
    const float ab = __builtin_fabsf(b);
    const float ub = ab * __uint_as_float(((__float_as_uint(q1) & 0x7fffffffu) - 1u) & 0x7f800000u);
    q = q1;
    // the guards select the bound (-1: refuse) and one compare decides: the
    // guard masks stay scalar masks feeding a single select (combining the
    // five compares as bools let the vectoriser pack them through VGPRs)
    const bool g = (ab >= 0x1p-100f) & (__builtin_fabsf(q1) >= 0x1p-100f) & (ub >= 0x1p-100f) & (ub <= 0x1p100f);
    const float thr = g ? ub * kDivT : -1.0f;
    return __builtin_fabsf(r) < thr;
}
// supg_tau_vm on the fast division: tau, and whether it is proven exact
// (rnu = an approximate 1 / (nu + eps))
__device__ inline float supg_tau_fast(float vm, float nu, float rnu, float dt, const PredK<float> &k, bool &ok) {
    float pe, q;
    const bool o1 = div_fast(vm * k.h, nu + k.eps, rnu, pe);
    const float half = pe / 2.0f;
    const float lim = half < 1.0f ? half : 1.0f;
    const float d = 2.0f * vm;
    const bool o2 = div_fast(k.h, d, __builtin_amdgcn_rcpf(d), q);
    float t = q * lim;
    asm volatile("" : "+v"(t));  // formed unconditionally (no branch on vm > eps)
    const bool big = vm > k.eps;
    ok = !big | (o1 & o2);
    return big ? t : dt / 2.0f;
}

// ---- per-type arithmetic of the row march ----------------------------------
template <typename T>
struct PredMath;

template <>
struct PredMath<float> {
    using Tables = libm::PowfTables;  // glibc powf's tables (LDS copy in the exact mode)
    static constexpr bool kFastPow = true;
    __device__ static void load_tables(Tables &dst) {
        const unsigned long long *src = reinterpret_cast<const unsigned long long *>(&libm::kPowfTables);
        unsigned long long *d = reinterpret_cast<unsigned long long *>(&dst);
        for (int q = threadIdx.x; q < (int)(sizeof(Tables) / 8); q += blockDim.x) d[q] = src[q];
    }
    __device__ static bool sq_fast(float x, float &p) { return libm::powf_sq_fast(x, p); }
    __device__ static bool sqrt_fast(float s, float &r) { return libm::powf_sqrt_fast(s, r); }
    __device__ static float pow_(float x, float y, const Tables &t) { return libm::powf(x, y, t); }
    __device__ static float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
    // exact tau from the exact |V|: the proven fast divisions, the IEEE ones
    // for a lane whose proof failed (rnu ~ 1 / (nu + eps))
    __device__ static float tau_exact(float vm, float nu, float rnu, float dt, const PredK<float> &k) {
        bool od;
        float t = supg_tau_fast(vm, nu, rnu, dt, k, od);
        if (__builtin_amdgcn_ballot_w64(!od)) {
            if (!od) t = supg_tau_vm(vm, nu, dt, k);
        }
        return t;
    }
    // sqrt(s) correctly rounded: the raw v_sqrt_f32 (within an ulp) moved to
    // the nearest float by its residual s - r0^2 (|residual| < r0 ulp(r0)
    // <=> |sqrt(s) - r0| < ulp / 2); 0 -> 0, inf / NaN pass through
    __device__ static float sqrt_rn(float s) {
        const float r0 = __builtin_amdgcn_sqrtf(s);
        const float e0 = __builtin_fmaf(-r0, r0, s);
        const float h = r0 * (__uint_as_float((__float_as_uint(r0) - 1u) & 0x7f800000u) * 0x1p-23f);
        const uint32_t b0 = __float_as_uint(r0);
        return __uint_as_float(e0 > h ? b0 + 1u : (e0 < -h ? b0 - 1u : b0));
    }
    // tolerance-mode tau (v5.py:156-161): half = (vm h / (nu + eps)) / 2 as one
    // quotient by b2 = 2 (nu + eps) (scaling by 2 is exact), h / (2 vm) as
    // (h / 2) / vm, each on v_rcp_f32 + one Newton step
    __device__ static float tau_tol(float vm, float b2, float rb2, float dt, const PredK<float> &k) {
        const float half = div_nr(vm * k.h, b2, rb2);
        const float lim = half < 1.0f ? half : 1.0f;
        const float t = div_nr(k.h * 0.5f, vm, __builtin_amdgcn_rcpf(vm)) * lim;
        return vm > k.eps ? t : dt / 2.0f;
    }
};

template <>
struct PredMath<double> {
    struct Tables {  // glibc pow's log and exp tables (LDS copy in the exact mode)
        double log[128][3];
        unsigned long long exp[256];
    };
    static constexpr bool kFastPow = false;  // every square and root through pow
    __device__ static void load_tables(Tables &dst) {
        const double *lsrc = &libm::kPowTab[0][0];
        double *ld = &dst.log[0][0];
        for (int q = threadIdx.x; q < 128 * 3; q += blockDim.x) ld[q] = lsrc[q];
        for (int q = threadIdx.x; q < 256; q += blockDim.x) dst.exp[q] = libm::kExpTab[q];
    }
    __device__ static bool sq_fast(double, double &) { return false; }
    __device__ static bool sqrt_fast(double, double &) { return false; }
    __device__ static double pow_(double x, double y, const Tables &t) { return libm::pow(x, y, t.log, t.exp); }
    __device__ static double rcp(double x) { return 1.0 / x; }
    __device__ static double tau_exact(double vm, double nu, double, double dt, const PredK<double> &k) {
        return supg_tau_vm(vm, nu, dt, k);
    }
    __device__ static double sqrt_rn(double s) { return __builtin_sqrt(s); }  // IEEE (correctly rounded)
    __device__ static double tau_tol(double vm, double b2, double, double dt, const PredK<double> &k) {
        const double half = (vm * k.h) / b2;
        const double lim = half < 1.0 ? half : 1.0;
        const double t = ((k.h * 0.5) / vm) * lim;
        return vm > k.eps ? t : dt / 2.0;
    }
};

// ---- row-march kernel --------------------------------------------------------
template <typename T>
struct PredRowArgs {
    const T *u, *v, *nu;  // nu: the nu_eff array, or null (nu_s)
    T *us, *vs, *tau;     // tau: null = not written
    T nu_s, dt;
    int ny, nx, rows, nseg, groups;
    PredK<T> k;
};

// a lane's VEC cells of one row
template <typename T, int VEC>
struct Cells {
    T x[VEC];
};
// load / store of a lane's cells through a buffer resource (kOob: reads 0,
// stores dropped); streaming store policy
template <typename T, int VEC>
__device__ inline Cells<T, VEC> pldv(__amdgpu_buffer_rsrc_t r, uint32_t ofs) {
    constexpr int B = VEC * (int)sizeof(T);
    static_assert(B == 4 || B == 8 || B == 16, "4, 8 or 16 bytes per lane");
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    if constexpr (B == 16) {
        return __builtin_bit_cast(Cells<T, VEC>, (u4)__builtin_amdgcn_raw_buffer_load_b128(r, (int)ofs, 0, 0));
    } else if constexpr (B == 8) {
        return __builtin_bit_cast(Cells<T, VEC>, (u2)__builtin_amdgcn_raw_buffer_load_b64(r, (int)ofs, 0, 0));
    } else {
        return __builtin_bit_cast(Cells<T, VEC>, (unsigned)__builtin_amdgcn_raw_buffer_load_b32(r, (int)ofs, 0, 0));
    }
}
template <typename T, int VEC>
__device__ inline void pstv(const Cells<T, VEC> &c, __amdgpu_buffer_rsrc_t r, uint32_t ofs) {
    constexpr int B = VEC * (int)sizeof(T);
    constexpr int kNt = 2;  // streaming (nt)
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    if constexpr (B == 16) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, c), r, (int)ofs, 0, kNt);
    } else if constexpr (B == 8) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, c), r, (int)ofs, 0, kNt);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, c), r, (int)ofs, 0, kNt);
    }
}
template <typename T>
__device__ inline T pld1(__amdgpu_buffer_rsrc_t r, uint32_t ofs) {
    return pldv<T, 1>(r, ofs).x[0];
}

template <typename T, int TAU, bool SUPG, bool NUA, int VEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 8))) void k_predictor_rows(PredRowArgs<T> a) {
    using M = PredMath<T>;
    constexpr bool kExactTau = SUPG && TAU == kTauExact;
    constexpr int SW = 64 * VEC;  // segment width (columns)
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // the exact mode's glibc tables in LDS: a table load from global memory
    // would wait (vmcnt) for every row load and store in flight (copied before
    // any wave of the workgroup can leave)
    __shared__ typename M::Tables ptab;
    if constexpr (kExactTau) {
        M::load_tables(ptab);
        __syncthreads();
    }
    const int b = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
    const int chunk = b / a.groups;
    const int seg = (b - chunk * a.groups) * 4 + wv;
    if (seg >= a.nseg) return;
    const int ny = a.ny, nx = a.nx;
    const int r0 = chunk * a.rows;
    const int r1 = min(r0 + a.rows, ny);
    const int xs = seg * SW;
    const int x0 = xs + lane * VEC;
    const bool lane_in = x0 < nx;  // nx % VEC == 0: a lane's cells are all in or all out
    const int bytes = (int)((size_t)ny * nx * sizeof(T));
    const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(a.u), 0, bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(a.v), 0, bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rn =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(NUA ? a.nu : a.u), 0, NUA ? bytes : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rus = __builtin_amdgcn_make_buffer_rsrc(a.us, 0, bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rvs = __builtin_amdgcn_make_buffer_rsrc(a.vs, 0, bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(a.tau ? a.tau : a.us, 0, a.tau ? bytes : 0, 0x00020000);
    // byte offset of this lane's cells in row i (kOob outside the grid: reads 0, stores dropped)
    auto rofs = [&](int i) -> uint32_t {
        return ((i >= 0) & (i < ny) & lane_in) ? (uint32_t)(((size_t)i * nx + x0) * sizeof(T)) : kOob;
    };
    // the segment's x-halo cells of row i: lane 0 column xs - 1, lane 63 column xs + SW
    const int hx = lane == 0 ? xs - 1 : (lane == kWave - 1 ? xs + SW : -1);
    const bool h_in = hx >= 0 && hx < nx;
    auto hofs = [&](int i) -> uint32_t {
        return ((i >= 0) & (i < ny) & h_in) ? (uint32_t)(((size_t)i * nx + hx) * sizeof(T)) : kOob;
    };
    const T dt = a.dt;
    // scalar nu: 1 / (nu + eps) (exact mode's proven divisions), and the
    // tolerance mode's 2 (nu + eps) with its reciprocal
    const T nue_s = a.nu_s + a.k.eps;
    const T rnu_s = M::rcp(nue_s);
    const T b2_s = T(2) * nue_s;
    const T rb2_s = M::rcp(b2_s);

    // rows i-1 (m), i (c), i+1 (p) and i+2 (n, in flight) of u and v; the
    // segment's x-halo cells and the nu_eff row of rows i, i+1, i+2
    Cells<T, VEC> Um = pldv<T, VEC>(ru, rofs(r0 - 1)), Vm = pldv<T, VEC>(rv, rofs(r0 - 1));
    Cells<T, VEC> Uc = pldv<T, VEC>(ru, rofs(r0)), Vc = pldv<T, VEC>(rv, rofs(r0));
    T HUc = pld1<T>(ru, hofs(r0)), HVc = pld1<T>(rv, hofs(r0));
    Cells<T, VEC> Up = pldv<T, VEC>(ru, rofs(r0 + 1)), Vp = pldv<T, VEC>(rv, rofs(r0 + 1));
    T HUp = pld1<T>(ru, hofs(r0 + 1)), HVp = pld1<T>(rv, hofs(r0 + 1));
    Cells<T, VEC> NUc = {}, NUp = {};
    if (NUA) {
        NUc = pldv<T, VEC>(rn, rofs(r0));
        NUp = pldv<T, VEC>(rn, rofs(r0 + 1));
    }
    for (int i = r0; i < r1; ++i) {
        // two rows ahead: row i+2 (and its halo cells / nu row)
        const Cells<T, VEC> Un = pldv<T, VEC>(ru, rofs(i + 2)), Vn = pldv<T, VEC>(rv, rofs(i + 2));
        const T HUn = pld1<T>(ru, hofs(i + 2)), HVn = pld1<T>(rv, hofs(i + 2));
        Cells<T, VEC> NUn = {};
        if (NUA) NUn = pldv<T, VEC>(rn, rofs(i + 2));
        Cells<T, VEC> uo = Uc, vo = Vc, to = {};
        if (i >= 1 && i <= ny - 2) {  // wave-uniform: boundary rows keep u* = u + dt*(-0 + 0)
            const T *uc = Uc.x, *vc = Vc.x;
            T uE[VEC], uW[VEC], vE[VEC], vW[VEC];
#pragma unroll
            for (int c = 0; c < VEC; ++c) {
                uE[c] = c < VEC - 1 ? uc[c + 1] : dpp_from_upper_old(HUc, uc[0]);
                uW[c] = c > 0 ? uc[c - 1] : dpp_from_lower_old(HUc, uc[VEC - 1]);
                vE[c] = c < VEC - 1 ? vc[c + 1] : dpp_from_upper_old(HVc, vc[0]);
                vW[c] = c > 0 ? vc[c - 1] : dpp_from_lower_old(HVc, vc[VEC - 1]);
            }
            T tq[VEC];
            if constexpr (kExactTau) {
                // the squares u**2, v**2 of the lane's cells, then their roots
                T sq[2 * VEC];
                if constexpr (M::kFastPow) {
                    // fast paths; a failing powf is re-done by the lane that
                    // needs it, one job per pass of a wave-uniform loop (one
                    // powf body per exponent in the code; a pass runs when
                    // any lane has a job left)
                    uint32_t f = 0;
#pragma unroll
                    for (int c = 0; c < VEC; ++c) {
                        f |= (M::sq_fast(uc[c], sq[2 * c]) ? 0u : 1u) << (2 * c);
                        f |= (M::sq_fast(vc[c], sq[2 * c + 1]) ? 0u : 1u) << (2 * c + 1);
                    }
                    while (__builtin_amdgcn_ballot_w64(f != 0)) {
                        if (f) {
                            const int j = __builtin_ctz(f);
                            T x = uc[0];
#pragma unroll
                            for (int q = 1; q < 2 * VEC; ++q) x = j == q ? ((q & 1) ? vc[q >> 1] : uc[q >> 1]) : x;
                            const T r = M::pow_(x, T(2), ptab);
#pragma unroll
                            for (int q = 0; q < 2 * VEC; ++q) sq[q] = j == q ? r : sq[q];
                            f &= f - 1;
                        }
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 2 * VEC; ++q) sq[q] = M::pow_((q & 1) ? vc[q >> 1] : uc[q >> 1], T(2), ptab);
                }
                T vmq[VEC], ss[VEC];
#pragma unroll
                for (int c = 0; c < VEC; ++c) ss[c] = sq[2 * c] + sq[2 * c + 1];
                if constexpr (M::kFastPow) {
                    uint32_t g = 0;
#pragma unroll
                    for (int c = 0; c < VEC; ++c) g |= (M::sqrt_fast(ss[c], vmq[c]) ? 0u : 1u) << c;
                    while (__builtin_amdgcn_ballot_w64(g != 0)) {
                        if (g) {
                            const int j = __builtin_ctz(g);
                            T x = ss[0];
#pragma unroll
                            for (int q = 1; q < VEC; ++q) x = j == q ? ss[q] : x;
                            const T r = M::pow_(x, T(0.5), ptab);
#pragma unroll
                            for (int q = 0; q < VEC; ++q) vmq[q] = j == q ? r : vmq[q];
                            g &= g - 1;
                        }
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < VEC; ++c) vmq[c] = M::pow_(ss[c], T(0.5), ptab);
                }
#pragma unroll
                for (int c = 0; c < VEC; ++c) {
                    const T nu = NUA ? NUc.x[c] : a.nu_s;
                    tq[c] = M::tau_exact(vmq[c], nu, NUA ? M::rcp(nu + a.k.eps) : rnu_s, dt, a.k);
                }
            } else if constexpr (SUPG) {
#pragma unroll
                for (int c = 0; c < VEC; ++c) {
                    const T vm = M::sqrt_rn(uc[c] * uc[c] + vc[c] * vc[c]);
                    T b2 = b2_s, rb2 = rb2_s;
                    if (NUA) {
                        b2 = T(2) * (NUc.x[c] + a.k.eps);
                        rb2 = M::rcp(b2);
                    }
                    tq[c] = M::tau_tol(vm, b2, rb2, dt, a.k);
                }
            }
            if constexpr (SUPG && VEC == 2 && sizeof(T) == 4) {
                // the lane's two cells as packed pairs (v_pk_add / v_pk_mul
                // on the Cells' register pairs): each element is the scalar
                // code's operation, in its order (conv_supg_sel, laplacian,
                // the u* / v* update below), so the bits are the same; the
                // selects stay per element
                typedef float f2 __attribute__((ext_vector_type(2)));
                const f2 U = {uc[0], uc[1]}, V = {vc[0], vc[1]};
                const f2 UE = {uE[0], uE[1]}, UW = {uW[0], uW[1]}, VE = {vE[0], vE[1]}, VW = {vW[0], vW[1]};
                const f2 UN = {Up.x[0], Up.x[1]}, US = {Um.x[0], Um.x[1]};
                const f2 VN = {Vp.x[0], Vp.x[1]}, VS = {Vm.x[0], Vm.x[1]};
                const f2 two = {2.0f, 2.0f};
                // the second differences, shared by SUPG and the Laplacian
                const f2 ux2 = (UE - two * U) + UW, uy2 = (UN - two * U) + US;
                const f2 vx2 = (VE - two * V) + VW, vy2 = (VN - two * V) + VS;
                const f2 t = {tq[0], tq[1]};
                const f2 csu = U * ((UE - UW) * a.k.c1x) + V * ((UN - US) * a.k.c1y);
                const f2 csv = U * ((VE - VW) * a.k.c1x) + V * ((VN - VS) * a.k.c1y);
                f2 cdu = csu - t * (U * (ux2 * a.k.c2x) + V * (uy2 * a.k.c2y));
                f2 cdv = csv - t * (U * (vx2 * a.k.c2x) + V * (vy2 * a.k.c2y));
                asm volatile("" : "+v"(cdu), "+v"(cdv));  // formed unconditionally (conv_supg_sel)
                const f2 NU = NUA ? f2{NUc.x[0], NUc.x[1]} : f2{a.nu_s, a.nu_s};
                const f2 lu = NU * (ux2 * a.k.lx + uy2 * a.k.ly);
                const f2 lv = NU * (vx2 * a.k.lx + vy2 * a.k.ly);
                const bool in0 = x0 >= 1 && x0 <= nx - 2, in1 = x0 + 1 >= 1 && x0 + 1 <= nx - 2;
                // a face cell: conv = lap = tau = 0 (np.zeros_like rings)
                const f2 cu = {in0 && t.x > 0.0f ? cdu.x : (in0 ? csu.x : 0.0f),
                               in1 && t.y > 0.0f ? cdu.y : (in1 ? csu.y : 0.0f)};
                const f2 cv = {in0 && t.x > 0.0f ? cdv.x : (in0 ? csv.x : 0.0f),
                               in1 && t.y > 0.0f ? cdv.y : (in1 ? csv.y : 0.0f)};
                const f2 lu0 = {in0 ? lu.x : 0.0f, in1 ? lu.y : 0.0f}, lv0 = {in0 ? lv.x : 0.0f, in1 ? lv.y : 0.0f};
                const f2 dt2 = {dt, dt};
                const f2 uo2 = U + dt2 * (-cu + lu0), vo2 = V + dt2 * (-cv + lv0);
                uo.x[0] = uo2.x;
                uo.x[1] = uo2.y;
                vo.x[0] = vo2.x;
                vo.x[1] = vo2.y;
                to.x[0] = in0 ? t.x : 0.0f;
                to.x[1] = in1 ? t.y : 0.0f;
            } else {
#pragma unroll
            for (int c = 0; c < VEC; ++c) {
                const T nu = NUA ? NUc.x[c] : a.nu_s;
                T cu, cv, t = T(0);
                if constexpr (SUPG) {
                    t = tq[c];
                    cu = conv_supg_sel(uc[c], vc[c], uc[c], uE[c], uW[c], Up.x[c], Um.x[c], t, a.k);
                    cv = conv_supg_sel(uc[c], vc[c], vc[c], vE[c], vW[c], Vp.x[c], Vm.x[c], t, a.k);
                } else {
                    cu = conv_upwind(uc[c], vc[c], uc[c], uE[c], uW[c], Up.x[c], Um.x[c], a.k);
                    cv = conv_upwind(uc[c], vc[c], vc[c], vE[c], vW[c], Vp.x[c], Vm.x[c], a.k);
                }
                const T lu = laplacian(nu, uc[c], uE[c], uW[c], Up.x[c], Um.x[c], a.k);
                const T lv = laplacian(nu, vc[c], vE[c], vW[c], Vp.x[c], Vm.x[c], a.k);
                const bool in = x0 + c >= 1 && x0 + c <= nx - 2;
                // a face cell: conv = lap = tau = 0 (np.zeros_like rings)
                uo.x[c] = uc[c] + dt * (-(in ? cu : T(0)) + (in ? lu : T(0)));
                vo.x[c] = vc[c] + dt * (-(in ? cv : T(0)) + (in ? lv : T(0)));
                to.x[c] = in ? t : T(0);
            }
            }
        } else {
#pragma unroll
            for (int c = 0; c < VEC; ++c) {
                uo.x[c] = Uc.x[c] + dt * (-T(0) + T(0));
                vo.x[c] = Vc.x[c] + dt * (-T(0) + T(0));
            }
        }
        const uint32_t o = rofs(i);
        pstv<T, VEC>(uo, rus, o);
        pstv<T, VEC>(vo, rvs, o);
        if (a.tau) pstv<T, VEC>(to, rt, o);  // zeros without SUPG (v5.py:292)
        Um = Uc;
        Vm = Vc;
        Uc = Up;
        Vc = Vp;
        Up = Un;
        Vp = Vn;
        HUc = HUp;
        HVc = HVp;
        HUp = HUn;
        HVp = HVn;
        if (NUA) {
            NUc = NUp;
            NUp = NUn;
        }
    }
}

// The row-march kernel for (tau mode, SUPG, array nu, cells per lane)
template <typename T, int VEC>
inline const void *pred_rows_kernel_v(bool supg, int tau, bool nua) {
    if (!supg) return nua ? (const void *)k_predictor_rows<T, kTauExact, false, true, VEC>
                          : (const void *)k_predictor_rows<T, kTauExact, false, false, VEC>;
    if (tau == kTauFast) return nua ? (const void *)k_predictor_rows<T, kTauFast, true, true, VEC>
                                    : (const void *)k_predictor_rows<T, kTauFast, true, false, VEC>;
    return nua ? (const void *)k_predictor_rows<T, kTauExact, true, true, VEC>
               : (const void *)k_predictor_rows<T, kTauExact, true, false, VEC>;
}

// workgroups of kernel f resident on the current device at once, cached per
// (device, kernel): the occupancy query is host latency on every step of a
// small grid
int pred_rows_resident(const void *f);
// the calling thread's last predictor launch (cfd_get_last_predictor2d_path):
// path 1 = row march, 0 = one thread per cell
void set_last_predictor(int path, int tau, int vec);

// Row-march launch: cells per lane `vec` (16 bytes per lane at most), rows per
// chunk `rows` (0: one resident round, 2..16); a.nseg / a.groups / a.rows are
// filled here.  The caller has checked shape and alignment.
template <typename T>
hipError_t pred_rows_launch(PredRowArgs<T> a, bool supg, int tau, int vec, int rows, hipStream_t s) {
    const void *f;
    if (vec == 4) {
        if constexpr (sizeof(T) == 4) f = pred_rows_kernel_v<T, 4>(supg, tau, a.nu != nullptr);
        else return hipErrorInvalidValue;
    } else if (vec == 2) {
        f = pred_rows_kernel_v<T, 2>(supg, tau, a.nu != nullptr);
    } else {
        f = pred_rows_kernel_v<T, 1>(supg, tau, a.nu != nullptr);
    }
    a.nseg = ceil_div(a.nx, 64 * vec);
    a.groups = ceil_div(a.nseg, 4);
    // rows per chunk: every workgroup resident at once (one round at the
    // kernel's occupancy), chunks of 2..16 rows (2 halo rows each) (r04 sweep,
    // 8192^2 SUPG f32: 16-row chunks beat 32 / 64 by 2-7 %; r05, 600 x 180:
    // 2-row chunks -- 450 workgroups instead of 46 -- take ~8 us off the
    // latency-bound launch)
    a.rows = rows;
    if (a.rows <= 0) {
        const int resident = pred_rows_resident(f);
        const int chunks = resident / a.groups > 0 ? resident / a.groups : 1;
        a.rows = ceil_div(a.ny, chunks);
        if (a.rows > 16) a.rows = 16;
        if (a.rows < 2) a.rows = 2;
    }
    const int nblk = a.groups * ceil_div(a.ny, a.rows);
    void *args[] = {&a};
    return hipLaunchKernel(f, dim3(nblk), dim3(256), args, 0, s);
}

}  // namespace cfd
