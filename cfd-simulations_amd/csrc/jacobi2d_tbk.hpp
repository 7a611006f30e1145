// jacobi2d_tbk.hpp -- the temporally blocked 2-D Jacobi (K sweeps per HBM
// pass).  Instantiated in jacobi2d_tbk_f32.hip / _f64.hip, one translation
// unit per type: the unrolled row marches (lcm(3, K) steps) dominate the
// library's build time.
#pragma once
#include "stencil2d.hpp"

namespace cfd {

// ---------------------------------------------------------------------------
// Temporally blocked 2-D Jacobi: K sweeps per pass (K = 2..6, 8, 10, 12): one pass reads
// phi^k and the rhs once and writes phi^(k+K), 12 B (f32) / 24 B (f64) per
// cell for K cell-updates.  A wave owns 64 lanes x VEC cells, but its
// x-segments OVERLAP by HL = ceil(K / VEC) lanes on each side: it writes only
// the inner (64 - 2 HL) * VEC cells, so every lane runs the same code, and the
// intermediate levels it needs near the segment edge are computed in-wave
// (erosion: level l is exact HL*VEC - l cells deep into the halo lanes), never
// exchanged.  Rows march with register queues, the 2-D analogue of
// jacobi3d_tbk: at front row r, level l is computed for row r - l + 1 from
// the level-(l-1) queue (rows p-1, p, p+1) and lane shuffles.  Every level
// uses the single sweep's operation order and mask rule (masked cells -> 0,
// edges included; Dirichlet rows/columns copied), so the result is
// bit-identical to K single sweeps.
// f(integral_constant<int, I>) for I in the sequence, in order
template <int... I, class F>
__device__ inline void static_for(std::integer_sequence<int, I...>, F &&f) {
    (f(std::integral_constant<int, I>{}), ...);
}
constexpr int gcd_c(int a, int b) { return b ? gcd_c(b, a % b) : a; }
// steps per unrolled group of jacobi2d_tbk: lcm(3, K) (level-0 / level rows
// rotate through 3 slots, rhs rows through K)
template <int K>
constexpr int kTbkUnroll = 3 * K / gcd_c(3, K);

// the pass's output rows with the streaming (nt) store policy: 8192^2 f64,
// r03: 0.3354 -> 0.3305 ms per pass
template <typename T, int VEC>
__device__ inline void st_out(T *p, const T (&r)[VEC]) {
    if constexpr (VEC > 1) {
        typename VecOf<T, VEC>::type v;
#pragma unroll
        for (int k = 0; k < VEC; ++k) v[k] = r[k];
        __builtin_nontemporal_store(v, reinterpret_cast<typename VecOf<T, VEC>::type *>(p));
    } else {
        __builtin_nontemporal_store(r[0], p);
    }
}
template <typename T, int VEC, int K, bool PRE, bool MASK>
__global__ __launch_bounds__(256) void jacobi2d_tbk(const T *__restrict__ in, T *__restrict__ out,
                                                    const T *__restrict__ div,
                                                    const uint8_t *__restrict__ mask, int ny,
                                                    int nx, int nseg, int rows_per_chunk, T dx2,
                                                    T dtv) {
    constexpr int HL = (K + VEC - 1) / VEC;    // halo lanes per side
    constexpr int SOUT = (64 - 2 * HL) * VEC;  // cells written per wave
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x / 64;
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * wpb + threadIdx.x / 64;
    const int seg = (int)(wave % nseg);
    const int chunk = (int)(wave / nseg);
    const int y0 = 1 + chunk * rows_per_chunk;
    if (y0 >= ny - 1) return;  // wave-uniform
    const int y1 = min(y0 + rows_per_chunk, ny - 1);
    const int x0 = seg * SOUT - HL * VEC + lane * VEC;  // this lane's first cell
    const bool valid = x0 >= 0 && x0 < nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
    auto inrow = [&](int y) { return valid && y >= 0 && y <= ny - 1; };
    // Register queues without moves: level l of row q lives in slot
    // (q - rs) mod 3 of Q[l], the rhs / mask of row q in slot (q - rs) mod K
    // of R / M, and the march is unrolled by U = lcm(3, K) steps so that every
    // slot is a compile-time constant (the shifting queues' moves were a fifth
    // of the VALU instructions at K = 8).  Chunks run whole groups of U steps
    // (the launcher sizes them so; steps past a chunk store nothing).
    constexpr int U = kTbkUnroll<K>;
    T Q[K][3][VEC];  // Q[l][s][k]: level l of a row in slot s
    T R[K][VEC];     // rhs of a row in slot s
    uint8_t M[K][VEC];
#pragma unroll
    for (int l = 0; l < K; ++l)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            Q[l][0][k] = Q[l][1][k] = Q[l][2][k] = R[l][k] = T(0);
            M[l][k] = 0;
        }
    const int rs = y0 - K + 1;  // first front row
    const int rl = y1 + K - 2;  // last front row
    const int nsteps = U * ((rl - rs + U) / U);
    // level 0 of rows rs - 1, rs, rs + 1: slots 2, 0, 1 (rhs rows before rs
    // only feed the pipeline fill, whose rows no output needs, so they stay 0)
    if (inrow(rs - 1)) ld<T, VEC>(in + row(rs - 1), Q[0][2]);
    if (inrow(rs)) ld<T, VEC>(in + row(rs), Q[0][0]);
    if (inrow(rs + 1)) ld<T, VEC>(in + row(rs + 1), Q[0][1]);
    if (inrow(rs)) {
        ld<T, VEC>(div + row(rs), R[0]);
        if (MASK) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) M[0][k] = mask[row(rs) + k];
        }
    }
    auto step = [&](int r, auto rotc) {
        constexpr int RT = decltype(rotc)::value;  // (r - rs) mod U
        constexpr int S2 = (RT + 2) % 3;  // level-0 slot of row r + 2
        // prefetch: level 0 of row r + 2 (into the slot of row r - 1, read by
        // level 1 below first), rhs / mask of row r + 1 (next step's)
        T nq[VEC], nd[VEC];
        uint8_t nm[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) { nq[k] = nd[k] = T(0); nm[k] = 0; }
        if (inrow(r + 2)) ld<T, VEC>(in + row(r + 2), nq);
        if (inrow(r + 1)) {
            ld<T, VEC>(div + row(r + 1), nd);
            if (MASK) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) nm[k] = mask[row(r + 1) + k];
            }
        }
#pragma unroll
        for (int l = 1; l <= K; ++l) {
            const int p = r - l + 1;
            const bool fixed = p == 0 || p == ny - 1;
            // slots: level l-1 at rows p (C), p + 1 (N), p - 1 (S); the rhs of row p
            const int sc = ((RT - l + 1) % 3 + 3) % 3, sn = ((RT - l + 2) % 3 + 3) % 3,
                      ss = ((RT - l) % 3 + 3) % 3, sr = ((RT - l + 1) % K + K) % K;
            const T *C = l == 1 ? Q[0][sc] : Q[l - 1][sc];
            const T *Nn = l == 1 ? Q[0][sn] : Q[l - 1][sn];
            const T *Ss = l == 1 ? Q[0][ss] : Q[l - 1][ss];
            const T wl = dpp_from_lower(C[VEC - 1]);
            const T er = dpp_from_upper(C[0]);
            T v[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T E = (k + 1 < VEC) ? C[k + 1] : er;
                const T W = (k > 0) ? C[k - 1] : wl;
                const int x = x0 + k;
                T val = (fixed || x <= 0 || x >= nx - 1) ? C[k]
                                                         : jac5<T>(E, W, Nn[k], Ss[k], R[sr][k], dx2, dtv, PRE);
                if (MASK && M[sr][k]) val = T(0);
                v[k] = val;
            }
            if (l < K) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) Q[l][sc][k] = v[k];  // over row p - 3 of level l, dead
            } else if (writer && p >= y0 && p < y1) {
                st_out<T, VEC>(out + row(p), v);
            }
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            Q[0][S2][k] = nq[k];  // row r + 2 over row r - 1 (dead after level 1)
            R[(RT + 1) % K][k] = nd[k];
            M[(RT + 1) % K][k] = nm[k];
        }
    };
    for (int rb = rs; rb < rs + nsteps; rb += U)
        static_for(std::make_integer_sequence<int, U>{}, [&](auto i) { step(rb + decltype(i)::value, i); });
}
// jacobi2d_tbk without a mask, its rows staged through LDS D rows ahead.
// The register march prefetches a row one step ahead, and at 8192^2 f64
// (K = 8) a step is ~600 VALU cycles against an HBM latency several times
// that, so the waves sat in vmcnt waits (r02: 0.59 of the HBM roofline, VALU
// busy ~0.3 per wave).  Here each wave owns a ring of D level-0 rows and D
// rhs rows in LDS, filled by LDS-DMA (buffer_load ... lds, no VGPRs) D steps
// before use: step t waits until its pair of rows has landed (vmcnt of the
// 2 (D - 1) younger DMAs; loads retire in order, the interleaved stores do not
// matter), copies them into the register queues and refills the two slots
// with rows t + D.  Same queues, levels and operation order as jacobi2d_tbk:
// bit-identical.
template <typename T, int VEC, int K, bool PRE, int D>
__global__ __launch_bounds__(256) void jacobi2d_tbd(const T *__restrict__ in, T *__restrict__ out,
                                                    const T *__restrict__ div, int ny, int nx, int nseg,
                                                    int rows_per_chunk, T dx2, T dtv) {
    static_assert(VEC * sizeof(T) == 16, "16 B per lane: one DMA of 1 KiB per row");
    constexpr int HL = (K + VEC - 1) / VEC;
    constexpr int SOUT = (64 - 2 * HL) * VEC;
    constexpr int WPB = 4;
    __shared__ __attribute__((aligned(16))) T ring[WPB][2][D][64 * VEC];  // [wave][phi, rhs][slot]
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const long wave = (long)bid * WPB + wv;
    const int seg = (int)(wave % nseg);
    const int chunk = (int)(wave / nseg);
    const int y0 = 1 + chunk * rows_per_chunk;
    if (y0 >= ny - 1) return;  // wave-uniform
    const int y1 = min(y0 + rows_per_chunk, ny - 1);
    const int x0 = seg * SOUT - HL * VEC + lane * VEC;
    const bool valid = x0 >= 0 && x0 < nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    auto row = [&](int y) { return (size_t)y * nx + (valid ? x0 : 0); };
    auto inrow = [&](int y) { return valid && y >= 0 && y <= ny - 1; };
    constexpr int U = kTbkUnroll<K>;
    T Q[K][3][VEC];
    T R[K][VEC];
#pragma unroll
    for (int l = 0; l < K; ++l)
#pragma unroll
        for (int k = 0; k < VEC; ++k) Q[l][0][k] = Q[l][1][k] = Q[l][2][k] = R[l][k] = T(0);
    const int rs = y0 - K + 1;
    const int rl = y1 + K - 2;
    const int nsteps = U * ((rl - rs + U) / U);
    if (inrow(rs - 1)) ld<T, VEC>(in + row(rs - 1), Q[0][2]);
    if (inrow(rs)) ld<T, VEC>(in + row(rs), Q[0][0]);
    if (inrow(rs + 1)) ld<T, VEC>(in + row(rs + 1), Q[0][1]);
    if (inrow(rs)) ld<T, VEC>(div + row(rs), R[0]);
    // row q of `a` (q <= qmax, inside the grid; else nothing: reads 0) into a
    // ring slot; invalid lanes read 0 through an out-of-range offset
    const uint32_t lofs = valid ? (uint32_t)x0 * (uint32_t)sizeof(T) : kOob;
    auto fetch = [&](const T *a, int q, int qmax, T *slot) {
        const bool ok = q >= 0 && q <= ny - 1 && q <= qmax;
        dma_row(buf_rsrc4(a + (size_t)(ok ? q : 0) * nx, ok ? (uint32_t)(nx * sizeof(T)) : 0u), lofs, slot);
    };
    // rows the march reads: level 0 up to rl + 1, the rhs up to rl
    auto refill = [&](int t) {  // the pair step t consumes: level-0 row rs+t+2, rhs row rs+t+1
        fetch(in, rs + t + 2, rl + 1, ring[wv][0][(t + 2) % D]);
        fetch(div, rs + t + 1, rl, ring[wv][1][(t + 1) % D]);
    };
#pragma unroll
    for (int t = 0; t < D; ++t) refill(t);
    auto step = [&](int t, auto rotc) {
        constexpr int RT = decltype(rotc)::value;  // t mod U
        constexpr int S2 = (RT + 2) % 3;
        const int r = rs + t;
        wait_vmcnt<2 * (D - 1)>();  // step t's pair has landed
        asm volatile("" ::: "memory");
        T nq[VEC], nd[VEC];
        ld<T, VEC>(&ring[wv][0][(t + 2) % D][lane * VEC], nq);
        ld<T, VEC>(&ring[wv][1][(t + 1) % D][lane * VEC], nd);
#pragma unroll
        for (int l = 1; l <= K; ++l) {
            const int p = r - l + 1;
            const bool fixed = p == 0 || p == ny - 1;
            const int sc = ((RT - l + 1) % 3 + 3) % 3, sn = ((RT - l + 2) % 3 + 3) % 3,
                      ss = ((RT - l) % 3 + 3) % 3, sr = ((RT - l + 1) % K + K) % K;
            const T *C = Q[l - 1][sc];
            const T *Nn = Q[l - 1][sn];
            const T *Ss = Q[l - 1][ss];
            const T wl = dpp_from_lower(C[VEC - 1]);
            const T er = dpp_from_upper(C[0]);
            T v[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const T E = (k + 1 < VEC) ? C[k + 1] : er;
                const T W = (k > 0) ? C[k - 1] : wl;
                const int x = x0 + k;
                v[k] = (fixed || x <= 0 || x >= nx - 1) ? C[k] : jac5<T>(E, W, Nn[k], Ss[k], R[sr][k], dx2, dtv, PRE);
            }
            if (l < K) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) Q[l][sc][k] = v[k];
            } else if (writer && p >= y0 && p < y1) {
                st_out<T, VEC>(out + row(p), v);
            }
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            Q[0][S2][k] = nq[k];
            R[(RT + 1) % K][k] = nd[k];
        }
        // the slots' reads are done before the DMA refills them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        refill(t + D);
    };
    for (int tb = 0; tb < nsteps; tb += U)
        static_for(std::make_integer_sequence<int, U>{}, [&](auto i) { step(tb + decltype(i)::value, i); });
    wait_vmcnt<0>();  // no DMA may land in LDS after the workgroup is gone
}

template <typename T, int VEC, int K, bool PRE, bool MASK>
static void jacobi2d_tbk_launch(const T *in, T *out, const T *div, const uint8_t *mask, int ny,
                                int nx, T dx2, T dtv, hipStream_t s) {
    constexpr int HL = (K + VEC - 1) / VEC;
    constexpr int SOUT = (64 - 2 * HL) * VEC;
    constexpr int wpb = 4;
    const int nseg = ceil_div(nx, SOUT);
    const int rows = ny - 2;
    // the kernel: the LDS-ring march where it applies (jacobi2d_tbd), else the
    // register march
    constexpr bool DMA_OK = !MASK && VEC * sizeof(T) == 16 && (K == 4 || K == 6 || K == 8);
    const int dma = DMA_OK ? tuning().j2_dma : 0;
    static int slot_cache[3] = {0, 0, 0};  // resident waves per chip, by kernel (register, ring 4, ring 6)
    int &slots = slot_cache[dma == 6 ? 2 : dma == 4 ? 1 : 0];
    if (slots <= 0) {
        int nb = 0, dev = 0, ncu = 0;
        hipError_t e = hipErrorInvalidValue;
        if constexpr (DMA_OK) {
            if (dma == 6) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jacobi2d_tbd<T, VEC, K, PRE, 6>, wpb * 64, 0);
            if (dma == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jacobi2d_tbd<T, VEC, K, PRE, 4>, wpb * 64, 0);
        }
        if (dma == 0) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, jacobi2d_tbk<T, VEC, K, PRE, MASK>, wpb * 64, 0);
        if (e != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            nb <= 0 || ncu <= 0) {
            (void)hipGetLastError();
            nb = 2;
            ncu = 256;
        }
        slots = nb * wpb * ncu;
    }
    int nchunk = slots / nseg;
    if (nchunk < 1) nchunk = 1;
    int rpc = ceil_div(rows, nchunk);
    // at least 2 (K-1) rows: the 2K-2 re-marched rows are at most half the
    // march (large grids get long chunks from the round sizing anyway)
    const int rmin = 2 * (K - 1);
    if (rpc < rmin) rpc = rmin;
    // whole groups of U steps per chunk (rpc + 2K - 2 steps): no step wasted
    // but in the last chunk
    constexpr int U = kTbkUnroll<K>;
    rpc = U * ceil_div(rpc + 2 * K - 2, U) - (2 * K - 2);
    nchunk = ceil_div(rows, rpc);
    const int blocks = ceil_div((long)nseg * nchunk, wpb);
    if constexpr (DMA_OK) {
        if (dma == 6) {
            hipLaunchKernelGGL((jacobi2d_tbd<T, VEC, K, PRE, 6>), dim3(blocks), dim3(wpb * 64), 0, s, in, out,
                               div, ny, nx, nseg, rpc, dx2, dtv);
            return;
        }
        if (dma == 4) {
            hipLaunchKernelGGL((jacobi2d_tbd<T, VEC, K, PRE, 4>), dim3(blocks), dim3(wpb * 64), 0, s, in, out,
                               div, ny, nx, nseg, rpc, dx2, dtv);
            return;
        }
    }
    hipLaunchKernelGGL((jacobi2d_tbk<T, VEC, K, PRE, MASK>), dim3(blocks), dim3(wpb * 64), 0, s, in,
                       out, div, mask, ny, nx, nseg, rpc, dx2, dtv);
}

template <typename T, int VEC>
int jacobi2d_tbk_pass(int K, const T *in, T *out, const T *div, const uint8_t *mask, int ny,
                             int nx, T dx2, T dtv, bool pre, hipStream_t s) {
    if (ny - 2 <= 0) return CFD_OK;
#define CFD_J2K(KV, PR, M) jacobi2d_tbk_launch<T, VEC, KV, PR, M>(in, out, div, mask, ny, nx, dx2, dtv, s)
#define CFD_J2KK(KV)                                                              \
    do {                                                                          \
        if (mask) {                                                               \
            if (pre) CFD_J2K(KV, true, true); else CFD_J2K(KV, false, true);      \
        } else {                                                                  \
            if (pre) CFD_J2K(KV, true, false); else CFD_J2K(KV, false, false);    \
        }                                                                         \
    } while (0)
    switch (K) {
        case 2: CFD_J2KK(2); break;
        case 3: CFD_J2KK(3); break;
        case 4: CFD_J2KK(4); break;
        case 5: CFD_J2KK(5); break;
        case 6: CFD_J2KK(6); break;
        case 10: CFD_J2KK(10); break;
        case 12: CFD_J2KK(12); break;
        default: CFD_J2KK(8); break;
    }
#undef CFD_J2KK
#undef CFD_J2K
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

}  // namespace cfd
