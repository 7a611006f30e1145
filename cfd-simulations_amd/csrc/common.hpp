// common.hpp -- shared helpers for the cfdsim HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/cfdsim.h"

// Every kernel in this library is written so that the compiler has nothing to
// contract: the reference never fuses a multiply-add, and bit-exact parity with
// the Jacobi branch depends on it.  The Makefile also passes -ffp-contract=off.
#pragma clang fp contract(off)

namespace cfd {

constexpr int kWave = 64;  // CDNA wavefront
constexpr int kNumXcd = 8; // MI355X: 8 XCDs, blocks dealt round-robin

void set_error(const char *fmt, ...);
// bench timing hooks (capi.hip): event pair around a solve's sweep launches
// (channel: kTimingSolve -- the pressure solves, what cfd_timing_read sums --
// or kTimingPredictor, read by cfd_timing_read_channel)
constexpr int kTimingSolve = 0, kTimingPredictor = 1;
int timing_begin(hipStream_t s, int channel = kTimingSolve);
void timing_end(int k, hipStream_t s, long long sweeps);
void timing_cancel(int k);

#define CFD_CHECK_HIP(expr)                                                          \
    do {                                                                             \
        hipError_t _e = (expr);                                                      \
        if (_e != hipSuccess) {                                                      \
            ::cfd::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                             __FILE__, __LINE__);                                    \
            return CFD_E_HIP;                                                        \
        }                                                                            \
    } while (0)

#define CFD_REQUIRE(cond, ...)               \
    do {                                     \
        if (!(cond)) {                       \
            ::cfd::set_error(__VA_ARGS__);   \
            return CFD_E_INVALID;            \
        }                                    \
    } while (0)

#define CFD_LAUNCH_CHECK()                                                             \
    do {                                                                               \
        hipError_t _e = hipGetLastError();                                             \
        if (_e != hipSuccess) {                                                        \
            ::cfd::set_error("kernel launch failed: %s (%s:%d)", hipGetErrorString(_e), \
                             __FILE__, __LINE__);                                      \
            return CFD_E_HIP;                                                          \
        }                                                                              \
    } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Wave-wide max of a non-negative float, then one atomic per wave.
// Non-negative IEEE floats order like their bit patterns as unsigned ints.
// NaN never wins: callers fold with `if (c > m) m = c`, like the reference
// (v5.py:220-222), before calling this.
__device__ inline float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    return v;
}
__device__ inline double wave_max(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
    return v;
}
// The same max over the wave by DPP (quad perms, row mirrors, row broadcasts
// 15 / 31, each a VALU modifier of a few cycles) instead of wave_max's six
// dependent ds_bpermute round trips through the LDS crossbar; every lane gets
// the result.  fmaxf ignores a NaN operand, as wave_max does.
template <int CTRL, int ROW_MASK>
__device__ inline float dpp_max_step(float v) {
    const int o = __float_as_int(v);
    return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(o, o, CTRL, ROW_MASK, 0xf, false)));
}
__device__ inline float wave_max_dpp(float v) {
    v = dpp_max_step<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_max_step<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_max_step<0x141, 0xf>(v);  // row_half_mirror
    v = dpp_max_step<0x140, 0xf>(v);  // row_mirror: every lane holds its row's max
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3: lane 63 has it all
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ inline void atomic_max_nonneg(float *dst, float v) {
    atomicMax(reinterpret_cast<unsigned int *>(dst), __float_as_uint(v));
}
__device__ inline void atomic_max_nonneg(double *dst, double v) {
    atomicMax(reinterpret_cast<unsigned long long *>(dst),
              static_cast<unsigned long long>(__double_as_longlong(v)));
}
// The target only grows during a kernel, so a (possibly stale, never larger)
// read that already covers m makes the atomic redundant: most waves skip it
// and millions of waves do not serialise on one address.
template <typename T>
__device__ inline void wave_reduce_max_store(T local, T *dst) {
    T m = wave_max(local);
    if ((threadIdx.x & (kWave - 1)) == 0 && m > T(0) && m > *reinterpret_cast<volatile T *>(dst))
        atomic_max_nonneg(dst, m);
}
// Workgroup-wide version: one atomic per workgroup.  Every thread of the
// workgroup must call it (it synchronises); `red` is __shared__ scratch of
// blockDim.x / 64 floats.
__device__ inline void block_reduce_max_store(float local, float *dst, float *red) {
    const float m = wave_max(local);
    const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
    if (lane == 0) red[wv] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float b = red[0];
        for (int k = 1; k < (int)(blockDim.x / kWave); ++k) b = fmaxf(b, red[k]);
        if (b > 0.0f && b > *reinterpret_cast<volatile float *>(dst)) atomic_max_nonneg(dst, b);
    }
}

// XCD-aware remap of a linear block id: blocks b and b+8 share an XCD (observed
// round-robin dealing, speed only -- never relied on for correctness).  Gives
// each XCD a contiguous run of logical tiles so neighbouring tiles (which share
// halo rows) hit the same L2.  Bijective; the tail beyond a multiple of 8 maps
// to itself.
__device__ inline int xcd_swizzle(int bid, int nblocks) {
    const int full = (nblocks / kNumXcd) * kNumXcd;
    if (bid >= full) return bid;
    const int per = full / kNumXcd;
    return (bid % kNumXcd) * per + bid / kNumXcd;
}

// x-neighbours across lanes by DPP wave shifts (a VALU modifier, a few cycles)
// instead of ds_bpermute (__shfl_up/down go through the LDS crossbar, ~100
// cycles each, and a K-level row march chains 2K of them): lane i receives
// lane i-1's value (from_lower, wave_shr:1) or lane i+1's (from_upper,
// wave_shl:1).  Lane 0 / 63 receive 0 (bound_ctrl: no old value has to be
// materialised first): callers overwrite them or never use them.
__device__ inline int dpp_i32_from_lower(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, true); }
__device__ inline int dpp_i32_from_upper(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, true); }
__device__ inline float dpp_from_lower(float v) { return __int_as_float(dpp_i32_from_lower(__float_as_int(v))); }
__device__ inline float dpp_from_upper(float v) { return __int_as_float(dpp_i32_from_upper(__float_as_int(v))); }
__device__ inline double dpp_from_lower(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)dpp_i32_from_lower((int)(unsigned)b);
    const unsigned hi = (unsigned)dpp_i32_from_lower((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ inline double dpp_from_upper(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)dpp_i32_from_upper((int)(unsigned)b);
    const unsigned hi = (unsigned)dpp_i32_from_upper((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the same shifts with an `old` operand: lane 0 (from_lower) / lane 63
// (from_upper) receive `old`, the value a neighbouring wave supplies
__device__ inline float dpp_from_lower_old(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ inline float dpp_from_upper_old(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), 0x130, 0xf, 0xf, false));
}
__device__ inline double dpp_from_lower_old(double old, double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), o = (unsigned long long)__double_as_longlong(old);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)b, 0x138, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(b >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ inline double dpp_from_upper_old(double old, double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v), o = (unsigned long long)__double_as_longlong(old);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)b, 0x130, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(b >> 32), 0x130, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// LDS-DMA of one 1 KiB row (64 lanes x 16 B) into lds_row[0..255]: the data
// lands in LDS without passing through VGPRs (buffer_load_dwordx4 ... lds,
// destination M0 + 16 * lane; a lane whose offset is outside the resource
// writes zeros).  Issued as inline asm on purpose: for a DMA the compiler can
// see, the waitcnt pass cannot tell the destination from other LDS data and
// drains every DMA (vmcnt(0)) before each LDS access.  Consumers wait with
// wait_vmcnt<> themselves; the compiler's own vmcnt counts only grow stricter
// with the extra in-flight operations.
typedef int v4i32 __attribute__((ext_vector_type(4)));
constexpr uint32_t kOob = 0x80000000u;  // a buffer offset past any resource: reads 0
// raw buffer resource over [base, base + bytes), stride 0
__device__ inline v4i32 buf_rsrc4(const void *base, uint32_t bytes) {
    const unsigned long long b = (unsigned long long)base;
    v4i32 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xffffu));
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
    r.w = 0x00020000;
    return r;
}
// (the same by LDS byte address)
__device__ inline void dma_row_at(v4i32 rs, uint32_t byte_ofs, uint32_t la) {
    int saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "s"(__builtin_amdgcn_readfirstlane(la)), "v"(byte_ofs), "s"(rs)
        : "memory");
}
__device__ inline void dma_row(v4i32 rs, uint32_t byte_ofs, void *lds_row) {
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)lds_row;
    int saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "s"(__builtin_amdgcn_readfirstlane(la)), "v"(byte_ofs), "s"(rs)
        : "memory");
}
// s_waitcnt vmcnt(N) (expcnt, lgkmcnt: no wait)
template <int N>
__device__ inline void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

// Mean of 0.5 (u^2 + v^2) over n cells (v5.py:362-363, :431-432) for grids
// up to kEnergyOneBlock cells: ONE 1024-thread workgroup, a fixed summation
// order (deterministic run to run) and no atomics -- the many-block version
// serialised ~1700 same-address double atomics (22 us at 600 x 180).  The
// per-cell energy is formed in T, summed in double, then scaled by 1/n.
constexpr size_t kEnergyOneBlock = (size_t)1 << 20;
// CLIP: the step's two np.clip calls (v5.py:437-438) fused in -- each cell's
// energy is formed from the value loaded (before the clip, as v5.py:431-435
// reads it), then the clipped value is stored (NaN passes like np.clip).
template <typename T>
__device__ inline T clip_val(T x, T lo, T hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <typename T, bool CLIP = false>
__global__ __launch_bounds__(1024) void k_energy_mean_1blk(T *__restrict__ u, T *__restrict__ v, size_t n,
                                                           double *out, T lo, T hi) {
    // 8 independent partial sums per thread (8 loads of each field in flight,
    // elements c, c + 1024, ..., c + 7 * 1024 of a round), folded in a fixed order
    constexpr int U = 8;
    __shared__ double part[16];
    double s[U];
#pragma unroll
    for (int q = 0; q < U; ++q) s[q] = 0.0;
    size_t c = threadIdx.x;
    for (; c + (U - 1) * 1024 < n; c += U * 1024) {
        T a[U], b[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            a[q] = u[c + q * 1024];
            b[q] = v[c + q * 1024];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) s[q] += (double)(T(0.5) * (a[q] * a[q] + b[q] * b[q]));
        if constexpr (CLIP) {
#pragma unroll
            for (int q = 0; q < U; ++q) {
                u[c + q * 1024] = clip_val(a[q], lo, hi);
                v[c + q * 1024] = clip_val(b[q], lo, hi);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < U; ++q)
        if (c + q * 1024 < n) {
            const T a = u[c + q * 1024], b = v[c + q * 1024];
            s[q] += (double)(T(0.5) * (a * a + b * b));
            if constexpr (CLIP) {
                u[c + q * 1024] = clip_val(a, lo, hi);
                v[c + q * 1024] = clip_val(b, lo, hi);
            }
        }
    double t = s[0];
#pragma unroll
    for (int q = 1; q < U; ++q) t += s[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, kWave);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) r += part[k];
        *out = r * (1.0 / (double)n);
    }
}

// The same mean over kEnergyBlocks workgroups (r05, the default): block b sums
// a fixed contiguous range of cells (the 1-block kernel's thread-strided fold
// at 256 threads), writes its partial, and the last block to take a ticket
// sums the partials in block order -- deterministic run to run, and one
// 108k-cell field no longer streams through a single CU (20.5 -> ~5 us at
// 600 x 180).  ws: a counter word (zero between calls; the last block
// resets it) and kEnergyBlocks doubles, per device and stream
// (energy_scratch).
constexpr int kEnergyBlocks = 64;
template <typename T, bool CLIP = false>
__global__ __launch_bounds__(256) void k_energy_mean_mb(T *__restrict__ u, T *__restrict__ v, size_t n, double *out,
                                                        T lo, T hi, unsigned *ws) {
    constexpr int U = 4;
    __shared__ double part[4];
    __shared__ int last;
    double *partial = reinterpret_cast<double *>(ws + 16);
    const size_t per = (n + kEnergyBlocks - 1) / kEnergyBlocks;
    const size_t b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    double s[U];
#pragma unroll
    for (int q = 0; q < U; ++q) s[q] = 0.0;
    size_t c = b0 + threadIdx.x;
    for (; c + (U - 1) * 256 < b1; c += U * 256) {
        T a[U], b[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            a[q] = u[c + q * 256];
            b[q] = v[c + q * 256];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) s[q] += (double)(T(0.5) * (a[q] * a[q] + b[q] * b[q]));
        if constexpr (CLIP) {
#pragma unroll
            for (int q = 0; q < U; ++q) {
                u[c + q * 256] = clip_val(a[q], lo, hi);
                v[c + q * 256] = clip_val(b[q], lo, hi);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < U; ++q)
        if (c + q * 256 < b1) {
            const T a = u[c + q * 256], b = v[c + q * 256];
            s[q] += (double)(T(0.5) * (a * a + b * b));
            if constexpr (CLIP) {
                u[c + q * 256] = clip_val(a, lo, hi);
                v[c + q * 256] = clip_val(b, lo, hi);
            }
        }
    double t = s[0];
#pragma unroll
    for (int q = 1; q < U; ++q) t += s[q];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off, kWave);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = ((part[0] + part[1]) + part[2]) + part[3];
        __threadfence();  // the partial before the ticket
        last = atomicAdd(ws, 1u) == (unsigned)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the partials, one load per thread (in flight together), then summed in
    // block order by one thread
    __shared__ double all[kEnergyBlocks];
    __threadfence();
    if ((int)threadIdx.x < (int)gridDim.x)
        all[threadIdx.x] = __hip_atomic_load(partial + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = 0.0;
        for (int k = 0; k < (int)gridDim.x; ++k) r += all[k];
        *out = r * (1.0 / (double)n);
        __hip_atomic_store(ws, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// apply_ibm_fast's factor on one cell (v5.py:228-237): float64 mask, float64
// product, rounded to the field's type
template <typename T>
__device__ inline T ibm_cell(T x, double mv, double fs) {
    return mv > 0.0 ? (T)((double)x * (1.0 - mv * fs)) : x;
}

// apply_boundary_conditions (v5.py:349-360, net effect as k_bc in
// fields2d.hip) followed by apply_ibm_fast (v5.py:228-237) in ONE launch.
// Every cell is written by one thread, which applies the BC assignment and
// then the IBM factor, the reference's order: threads t < nx own rows 0 and
// ny - 1; threads 1 <= t < ny - 1 own columns 0, nx - 2 and nx - 1 of row t
// (the outlet copy reads column nx - 2 before its IBM factor); the rest of
// the cells go to a grid-stride loop over the mask.  m == nullptr: no IBM.
template <typename T>
__global__ void k_bc_ibm(T *__restrict__ u, T *__restrict__ v, const double *__restrict__ y,
                         const double *__restrict__ m, int ny, int nx, double y_max, double v_inf, int step,
                         double fs) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    auto mk = [&](size_t c) { return m ? m[c] : 0.0; };
    if (t < nx) {
        const size_t c0 = t, c1 = (size_t)(ny - 1) * nx + t;
        u[c0] = ibm_cell(T(0), mk(c0), fs);
        v[c0] = ibm_cell(T(0), mk(c0), fs);
        u[c1] = ibm_cell(T(0), mk(c1), fs);
        v[c1] = ibm_cell(T(0), mk(c1), fs);
    }
    if (t >= 1 && t < ny - 1) {
        const double s = (double)step;
        double scale = s / 1000.0;
        scale = (1.0 < scale ? 1.0 : scale) * 0.01;
        const double two_pi = 2.0 * 3.141592653589793;
        const double pert = scale * sin(two_pi * y[t] / y_max + 0.02 * s);
        const size_t r = (size_t)t * nx;
        const T inlet = (T)(v_inf * (1.0 + pert));
        // the outlet copy's source: column nx - 2 after the inlet assignment
        const T uo = nx == 2 ? inlet : u[r + nx - 2], vo = nx == 2 ? T(0) : v[r + nx - 2];
        u[r] = ibm_cell(inlet, mk(r), fs);
        v[r] = ibm_cell(T(0), mk(r), fs);
        if (nx > 2) {
            u[r + nx - 2] = ibm_cell(uo, mk(r + nx - 2), fs);
            v[r + nx - 2] = ibm_cell(vo, mk(r + nx - 2), fs);
        }
        u[r + nx - 1] = ibm_cell(uo, mk(r + nx - 1), fs);
        v[r + nx - 1] = ibm_cell(vo, mk(r + nx - 1), fs);
    }
    if (!m) return;
    const size_t n = (size_t)ny * nx;
    for (size_t c = t; c < n; c += (size_t)gridDim.x * blockDim.x) {
        const double mv = m[c];
        if (mv > 0.0) {
            const int i = (int)(c / nx), j = (int)(c % nx);
            if (i >= 1 && i < ny - 1 && j >= 1 && j < nx - 2) {
                u[c] = ibm_cell(u[c], mv, fs);
                v[c] = ibm_cell(v[c], mv, fs);
            }
        }
    }
}

inline int ceil_div(long a, long b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace cfd
