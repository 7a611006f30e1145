// jacobi3d_tbr.hip -- K Jacobi sweeps per HBM pass with TALL tiles: several
// rows per wave and single-buffered LDS level tiles (two barriers per step).
//
// The round-1 design (one row per wave, double-buffered tiles, since
// removed) was limited to 16 waves = W + 2K - 1, so a tile of W output rows
// re-read 2K halo rows of its neighbours (W = 11 rows for K = 3: 17 rows of
// phi and 15 of rhs fetched per 11 output rows).  Here a row wave owns RPW rows (its
// register queues are RPW times as large; 8-12 waves per workgroup leave
// 168-256 VGPRs per wave), and the level tiles are single-buffered so that
// the taller tile still fits in LDS:
//
//    phase W: level 0 of plane z, and the level-l values computed in the
//             previous step (plane z-l), into the tiles T_0 .. T_(K-1);
//    barrier;
//    phase R: level l of plane z-l+1 for l = 1..K, reading T_(l-1) (y) and
//             the register queues (z); level K goes to HBM;
//    barrier.
//
// Shapes (K, row waves, rows per wave) -> output rows W = NWR*RPW + 2 - 2K:
// (3, 11, 2) W = 18; (4, 7, 3) W = 15; (3, 7, 3) W = 17.  Everything else --
// the halo wave, the z-march bounds, Dirichlet copies, erosion of garbage --
// is as in that design, and the result is bit-identical to K single
// sweeps (tests/test_gpu_parity.py).
#include <type_traits>

#include "internal.hpp"

namespace cfd {

namespace {

// Global (not flat) loads and stores: the halo wave's pointers reach it as
// generic pointers (TbrArgs by value), and a flat load counts in lgkmcnt as
// well as vmcnt, so the LDS barrier's lgkmcnt(0) waited for the halo wave's
// just-issued prefetch -- a full memory latency at the first barrier of every
// step (r03 per-wave trace, cfd_set_tbr_trace: the halo wave arrived last at
// it, ~2200 cycles into a 5500-cycle step).
// (The HIP float4 struct would still load through a generic `this`: native
// ext vectors in the global address space.)
typedef float gv4g __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) gv4g *gcv4p;
typedef __attribute__((address_space(1))) gv4g *gv4p;
__device__ inline float4 ldg4(const float *p) {
    const gv4g v = *(gcv4p)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ inline void stg4(float *p, float4 v) { *(gv4p)p = gv4g{v.x, v.y, v.z, v.w}; }
__device__ inline float4 lds4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ inline void sts4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// Plane rows through buffer resources: one resource per (array, plane) in
// SGPRs with num_records = the plane's bytes (0 for a plane outside the
// array); a lane outside the grid passes kOob and reads 0, with no branch.
typedef float gv4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
// LDS float pointers (32-bit addresses) for the lane-based addressing of the
// Jacobi row waves: a float4 at base + compile-time offset is one ds_read_b128
// / ds_write_b128 with the offset in the instruction's immediate field
typedef __attribute__((address_space(3))) float lfloat;
typedef __attribute__((address_space(3))) gv4f lgv4f;
__device__ inline uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)(const lds_void *)p; }
__device__ inline lfloat *lds_ptr(uint32_t a) { return (lfloat *)(uintptr_t)a; }
__device__ inline float4 lds4l(const lfloat *p) {
    const gv4f v = *(const lgv4f *)p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ inline void sts4l(lfloat *p, float4 v) { *(lgv4f *)p = gv4f{v.x, v.y, v.z, v.w}; }
__device__ inline __amdgpu_buffer_rsrc_t plane_rsrc(const float *base, int p, int nz, size_t plane) {
    const bool in = p >= 0 && p <= nz - 1;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(in ? base + (size_t)p * plane : base),
                                             (short)0, in ? (int)(plane * sizeof(float)) : 0, 0x00020000);
}
// Cache policy of the passes' HBM stores (buffer-store aux bits): nt, the
// streaming policy -- 1024^3, r03: K = 3 Jacobi 2.204 -> 2.174 ms per pass,
// K = 4 2.954 -> 2.894, the 4-level GS 2.752 -> 2.675.  (sc1 and sc0 sc1,
// which drop the line from L2: K = 4 3.07; nt on the LDS-DMA / buffer loads
// as well: 2.97 ms at K = 3 -- the neighbouring tiles' halo re-reads then
// miss L2.)
constexpr int kStoreNt = 2;
// lane-based LDS addressing and exact vmcnt waits in the Jacobi row waves
// (A/B knobs; see the DMA row wave)
#ifndef CFD_TBR_LB
#define CFD_TBR_LB 1
#endif
#ifndef CFD_TBR_XW
#define CFD_TBR_XW 1
#endif
#ifndef CFD_TBR_SD  // per-step scalar state by additions (Jacobi row waves; see the DMA row wave)
#define CFD_TBR_SD 1
#endif
#ifndef CFD_TBR_T0S  // level-0 tile = the DMA staging slot (Jacobi; see jacobi3d_tbr)
#define CFD_TBR_T0S 1
#endif
#ifndef CFD_TBR_EARLY
#define CFD_TBR_EARLY 1
#endif


__device__ inline float4 ldb4(__amdgpu_buffer_rsrc_t r, uint32_t byte_ofs) {
    const gv4f v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_ofs, 0, 0);
    return make_float4(v.x, v.y, v.z, v.w);
}
// (dma_row, wait_vmcnt: common.hpp)
__device__ inline v4i32 plane_rsrc4(const float *base, int p, int nz, size_t plane) {
    const bool in = p >= 0 && p <= nz - 1;
    const unsigned long long b = (unsigned long long)(in ? base + (size_t)p * plane : base);
    v4i32 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(b >> 32) & 0xffffu));  // stride 0
    r.z = __builtin_amdgcn_readfirstlane(in ? (int)(plane * sizeof(float)) : 0);
    r.w = 0x00020000;
    return r;
}
// LDS barrier that leaves LDS-DMA in flight (__syncthreads' fence would wait
// vmcnt(0)); the memory clobber keeps the compiler's LDS accesses in place
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
enum { kJacobi = 0, kRbgs = 1 };
// register-queue slot of a plane offset v: v mod 3 / v mod k, non-negative
constexpr int sl3(int v) { return ((v % 3) + 3) % 3; }
constexpr int slk(int v, int k) { return ((v % k) + k) % k; }

struct TbrArgs {
    const float *in;
    float *out;
    const float *div;  // div, or the precomputed rhs (PRE)
    int nz, ny, nx, nseg, ntile_y, zb, ze, zchunk, fixed_lo, fixed_hi;
    float h2, dt;                      // Jacobi
    float cx, cy, cz, cd, dt_inv, tol; // red-black GS
    int zoff;        // global z of local plane 0 (colour parity)
    int h0;          // GS: first half-sweep of this pass (iteration h0 / 2, colour h0 & 1)
    float *maxc;     // per-iteration max|change| (device), NULL: not accumulated
    int rollback;    // GS: 0, or the half-sweeps per pass P of the solve whose stop this undoes
    int nhalf;       // GS rollback: half-sweeps the solve scheduled (2 x iterations)
    const int *count;  // GS rollback: iterations done (device)
    int lag;         // GS: the stop test reads maxc[it-1-lag], maxc[it-2-lag] (see rbgs3d_tbr_pass)
    float *rhs_out;  // first pass (F & kFirstRhs): the rhs of the owned cells goes here
    int xbw;         // XCD block width in x-segments (0: each XCD takes whole tile rows), see tbr_launch
    unsigned long long *trace;  // diagnostics (cfd_set_tbr_trace): per-wave step timestamps, or NULL
};
// Diagnostics (builds with -DCFD_TBR_TRACE only: the marks cost the 4-level
// kernels registers, 9-33 VGPRs of spill): workgroup 0's waves record the
// shader clock at 5 points of kTraceSteps z-steps from kTraceStep0 on (step
// entry, before / after the first barrier, before / after the second) into
// trace[wave][step][5].  r03 finding, 1024^3, cycles per step: K = 3 Jacobi
// 5430-5500 = phase W ~2000 (the third wave of each SIMD and the halo wave
// arrive last at the first barrier) + phase R ~3300 (VALU-bound per SIMD);
// 4-level GS 6900-7300.
constexpr int kTraceStep0 = 200, kTraceSteps = 64;
__device__ inline void trace_mark(unsigned long long *tr, int wave, int step, int e) {
#ifdef CFD_TBR_TRACE
    const int k = step - kTraceStep0;
    if (tr && blockIdx.x == 0 && (threadIdx.x & 63) == 0 && k >= 0 && k < kTraceSteps)
        tr[((size_t)wave * kTraceSteps + k) * 5 + e] = __builtin_readcyclecounter();
#else
    (void)tr;
    (void)wave;
    (void)step;
    (void)e;
#endif
}
// First-pass flags (template F of jacobi3d_tbr, Jacobi on the LDS-DMA path):
// kFirstRhs: `div` is raw; the row waves form f32(h*h)*div/dt once per cell
// (the bits k_rhs_f32 and the in-register form give) and store it to rhs_out
// for the later passes, replacing the separate RHS prologue;
// kFirstZero: level 0 is phi = 0 (v5.py:337's zero fill): nothing is read
// from `in`, so the pass can write either buffer and no memset is needed.
enum { kFirstRhs = 1, kFirstZero = 2 };

// One level on the float4 of cells x .. x+3.  Jacobi: every interior cell.
// Red-black GS: the cells of colour `par` parity (v5.py:213-219 generalised:
// (((cx(E+W) + cy(N+S)) + cz(U+D)) - rhs) * cd with rhs = -div * dt_inv, the
// in-place kernel's operation order); `chg` folds max|change| of own cells.
template <int MODE, bool PRE, bool PK = false>
__device__ inline float4 level4(float4 c, float wl, float er, float4 N, float4 S, float4 U,
                                float4 D, float4 d, int x, int nx, bool upd, const TbrArgs &a,
                                int par, bool own, float &chg) {
    if (!upd) return c;
    if (MODE == kRbgs) {
        // x % 4 == 0, so the colour updates cells k = par & 1 and k + 2 of the
        // float4: those two only, as one float2 pair through packed math, in
        // the in-place kernel's operation order.  The row waves pass a par that
        // is a compile-time constant once their loops are unrolled (see
        // `march`), so the selects below fold away there.
        typedef float v2f __attribute__((ext_vector_type(2)));
        const bool hi = (par & 1) != 0;
        const v2f C = hi ? v2f{c.y, c.w} : v2f{c.x, c.z};
        const v2f E = hi ? v2f{c.z, er} : v2f{c.y, c.w};
        const v2f Wv = hi ? v2f{c.x, c.z} : v2f{wl, c.y};
        const v2f Nv = hi ? v2f{N.y, N.w} : v2f{N.x, N.z};
        const v2f Sv = hi ? v2f{S.y, S.w} : v2f{S.x, S.z};
        const v2f Uv = hi ? v2f{U.y, U.w} : v2f{U.x, U.z};
        const v2f Dv = hi ? v2f{D.y, D.w} : v2f{D.x, D.z};
        const v2f Rv = hi ? v2f{d.y, d.w} : v2f{d.x, d.z};
        const v2f rhs = -Rv * a.dt_inv;
        const v2f p = a.cx * (E + Wv);
        const v2f q = a.cy * (Nv + Sv);
        const v2f r = a.cz * (Uv + Dv);
        v2f o = (((p + q) + r) - rhs) * a.cd;
        const int x0 = x + (hi ? 1 : 0);  // the pair's cells x0, x0 + 2 (x0 + 2 >= 2)
        o.x = (x0 != 0 && x0 != nx - 1) ? o.x : C.x;
        o.y = (x0 + 2 != nx - 1) ? o.y : C.y;
        if (own) {  // fmaxf ignores a NaN change like the `ch > mx` test
            chg = fmaxf(chg, fabsf(o.x - C.x));
            chg = fmaxf(chg, fabsf(o.y - C.y));
        }
        return hi ? make_float4(c.x, o.x, c.z, o.y) : make_float4(o.x, c.y, o.y, c.w);
    }
    // PK: the packed form below; else this one, left to the compiler's
    // vectoriser (1024^3, r03: the K = 4 pass 3.67 ms this way against 2.81
    // packed -- 36 VGPRs of spill -- the K = 3 pass 2.17 against 2.24)
    if constexpr (!PK) {
        float o[4];
        const float cv[4] = {c.x, c.y, c.z, c.w};
        const float nv[4] = {N.x, N.y, N.z, N.w};
        const float sv[4] = {S.x, S.y, S.z, S.w};
        const float uv[4] = {U.x, U.y, U.z, U.w};
        const float dv[4] = {D.x, D.y, D.z, D.w};
        const float rv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float E = k < 3 ? cv[k + 1] : er;
            const float Wv = k > 0 ? cv[k - 1] : wl;
            float s = E + Wv;
            s = s + nv[k];
            s = s + sv[k];
            s = s + uv[k];
            s = s + dv[k];
            const float rhs = PRE ? rv[k] : (a.h2 * rv[k]) / a.dt;
            const int xk = x + k;
            o[k] = (xk != 0 && xk != nx - 1) ? (1.0f / 6.0f) * (s - rhs) : cv[k];
    }
    return make_float4(o[0], o[1], o[2], o[3]);
    }
    // cells (0, 1) and (2, 3) as packed pairs (v_pk_add / v_pk_mul: each
    // element the scalar operation, in the single sweep's order), written
    // out so that the pairs are the aligned register pairs of the float4s
    typedef float v2 __attribute__((ext_vector_type(2)));
    const v2 mid = {c.y, c.z};  // E of cells 0, 1 and W of cells 2, 3
    v2 s01 = mid + v2{wl, c.x};
    v2 s23 = v2{c.w, er} + mid;
    s01 = s01 + v2{N.x, N.y};
    s23 = s23 + v2{N.z, N.w};
    s01 = s01 + v2{S.x, S.y};
    s23 = s23 + v2{S.z, S.w};
    s01 = s01 + v2{U.x, U.y};
    s23 = s23 + v2{U.z, U.w};
    s01 = s01 + v2{D.x, D.y};
    s23 = s23 + v2{D.z, D.w};
    v2 r01 = {d.x, d.y}, r23 = {d.z, d.w};
    if constexpr (!PRE) {
        r01 = (a.h2 * r01) / a.dt;
        r23 = (a.h2 * r23) / a.dt;
    }
    v2 o01 = (1.0f / 6.0f) * (s01 - r01);
    v2 o23 = (1.0f / 6.0f) * (s23 - r23);
    // edge columns 0 and nx - 1 keep their values: with x % 4 == 0 and
    // nx % 4 == 0 (the launcher's requirement) only cell 0 can be column 0
    // and only cell 3 column nx - 1
    o01.x = x != 0 ? o01.x : c.x;
    o23.y = x + 3 != nx - 1 ? o23.y : c.w;
    return make_float4(o01.x, o01.y, o23.x, o23.y);
}

// Red-black GS pairs: in a float4 at x % 4 == 0 a colour owns the cells
// h, h + 2 (h = 0 or 1, the same for every level of a row in a z-step, see
// the DMA row wave); pick / other take the pair at h / 1 - h, join puts `a`
// at h and `b` at 1 - h.
typedef float v2f_t __attribute__((ext_vector_type(2)));
__device__ inline v2f_t pick2(float4 f, int h) { return h ? v2f_t{f.y, f.w} : v2f_t{f.x, f.z}; }
__device__ inline float4 join2(v2f_t a, v2f_t b, int h) {
    return h ? make_float4(b.x, a.x, b.y, a.y) : make_float4(a.x, b.x, a.y, b.y);
}
// A float4 of the GS row waves' level-0 and rhs queues, held as its two
// colour pairs (cells 0, 2 and 1, 3): a level takes its pair without the
// moves that picking one out of a float4 costs (2 per pick, ~10 per update)
struct P4 {
    v2f_t e, o;
};
__device__ inline v2f_t pick2(const P4 &f, int h) { return h ? f.o : f.e; }
__device__ inline P4 split4(float4 f) { return P4{v2f_t{f.x, f.z}, v2f_t{f.y, f.w}}; }

// Jacobi register-queue entry as two 64-bit values (CFD_TBR_Q64): a float4
// held this way is copied by two v_mov_b64 when its queue shifts, where the
// float4's four 32-bit components were copied one v_mov_b32 at a time
#ifndef CFD_TBR_Q64
#define CFD_TBR_Q64 1
#endif
struct Q4 {
    unsigned long long lo, hi;
};
__device__ inline Q4 q4_of(float4 f) {
    return Q4{__builtin_bit_cast(unsigned long long, v2f_t{f.x, f.y}),
              __builtin_bit_cast(unsigned long long, v2f_t{f.z, f.w})};
}
__device__ inline float4 f4_of(const Q4 &q) {
    const v2f_t a = __builtin_bit_cast(v2f_t, q.lo), b = __builtin_bit_cast(v2f_t, q.hi);
    return make_float4(a.x, a.y, b.x, b.y);
}
[[maybe_unused]] __device__ inline float4 f4_of(float4 f) { return f; }
__device__ inline const P4 &f4_of(const P4 &p) { return p; }
// from LDS: two ds_read2_b32 (words 0, 2 and 1, 3) straight into the pairs
__device__ inline P4 ldsp(const float *p) { return P4{v2f_t{p[0], p[2]}, v2f_t{p[1], p[3]}}; }
// GS tiles (SPLIT): the 256 cells of a tile row are stored by colour pair,
// cells 4 i + {0, 2} at 4 + 2 i and cells 4 i + {1, 3} at 132 + 2 i, so a
// lane reads its pair as one conflict-free ds_read_b64 (the float4 layout
// makes it a ds_read2_b32 of words 8 B apart at a 16-B lane stride: bank
// conflicts); the x-halo columns 0..3 / 260..263 keep the plain layout, and
// the cells next to them (xs at 4, xs + 255 at 259) land where they were.
__device__ inline void sts4s(float *row, int lane, float4 v) {
    *reinterpret_cast<v2f_t *>(row + 4 + 2 * lane) = v2f_t{v.x, v.z};
    *reinterpret_cast<v2f_t *>(row + 132 + 2 * lane) = v2f_t{v.y, v.w};
}
__device__ inline void sts4s(float *row, int lane, const P4 &v) {
    *reinterpret_cast<v2f_t *>(row + 4 + 2 * lane) = v.e;
    *reinterpret_cast<v2f_t *>(row + 132 + 2 * lane) = v.o;
}
// pair-tile row (PT): left chunk pair | 64 lanes x pair | right chunk pair
constexpr int kPairRow = 132;
__device__ inline v2f_t lds2s(const float *row, int lane, int h) {
    return *reinterpret_cast<const v2f_t *>(row + 4 + 128 * h + 2 * lane);
}
// One red-black level on a pair: C its cells' old values, O the other
// colour's pair of the same row (E / W, with the lanes' DPP neighbours), N,
// S, U, D the neighbour rows' / planes' pairs at the same positions, rhs the
// pair of -div * dt_inv (formed once per row as it enters the queue, the
// product level4 forms per update); level4's operation order and edge rule,
// so the same bits.
// The GS stencil constants as packed pairs held in VGPRs (GsPk): as scalar
// operands of the packed ops they were four SGPR pairs live across the whole
// march, which pushed the lane masks out to VGPR lanes (r05: 59 in-loop
// v_readlane / v_writelane); the row waves have VGPRs to spare (154 of 168).
struct GsPk {
    v2f_t cx, cy, cz, cd, ndt;  // ndt = -dt_inv: the rhs pair -div * dt_inv as div * ndt (same bits)
};
__device__ inline GsPk gs_pk(const TbrArgs &a) {
    GsPk k{v2f_t{a.cx, a.cx}, v2f_t{a.cy, a.cy}, v2f_t{a.cz, a.cz}, v2f_t{a.cd, a.cd},
           v2f_t{-a.dt_inv, -a.dt_inv}};
    asm volatile("" : "+v"(k.cx), "+v"(k.cy), "+v"(k.cz), "+v"(k.cd), "+v"(k.ndt));
    return k;
}
__device__ inline v2f_t level2(v2f_t C, v2f_t O, float wl, float er, v2f_t N, v2f_t S, v2f_t U, v2f_t D,
                               v2f_t rhs, int h, int x, int nx, bool upd, const GsPk &a, bool own,
                               float &chg) {
    if (!upd) return C;
    const v2f_t E = h ? v2f_t{O.y, er} : v2f_t{O.x, O.y};
    const v2f_t W = h ? v2f_t{O.x, O.y} : v2f_t{wl, O.x};
    const v2f_t p = a.cx * (E + W);
    const v2f_t q = a.cy * (N + S);
    const v2f_t r = a.cz * (U + D);
    v2f_t o = (((p + q) + r) - rhs) * a.cd;
    const int x0 = x + h;  // the pair's cells x0, x0 + 2
    // (x % 4 == 0, nx % 4 == 0: only x0 = 0 can be column 0 and only
    // x0 + 2 = x + 3 column nx - 1)
    if (h == 0) o.x = x0 != 0 ? o.x : C.x;
    if (h == 1) o.y = x0 + 2 != nx - 1 ? o.y : C.y;
    if (own) {
        chg = fmaxf(chg, fabsf(o.x - C.x));
        chg = fmaxf(chg, fabsf(o.y - C.y));
    }
    return o;
}

}  // namespace

// The halo wave of jacobi3d_tbr (see there): loads the two outermost level-0
// rows and the 4-float x-halo chunks of every row, and computes levels
// 1..K-1 of the chunks, in lock step (two barriers per step) with the row waves.
template <int K, int NWR, int RPW, bool PRE, int PD, int MODE, int F, bool SPLIT, bool PT, bool T0S = false>
__device__ __forceinline__ void tbr_halo_wave(const TbrArgs a, float *smem, int z0, int z1, int y0, int xs,
                                              int zl, float *slots = nullptr) {
    constexpr int NR = NWR * RPW + 2;
    constexpr int RS = 264, RS2 = kPairRow;
    // T0S: level 0 of plane z is slot (z - zs) mod 3 of `slots` (the row
    // waves' LDS-DMA staging ring), the level tiles 1..K-1 start at smem
    int t0 = 0;  // this step's slot offset (floats)
    auto T = [&](int l, int r) -> float * {
        if (T0S && l == 0) return slots + t0 + r * RS;
        int base = 0;
#pragma unroll
        for (int m = T0S ? 1 : 0; m < K; ++m)
            if (m < l) base += (NR - 2 * m) * (PT && m ? RS2 : RS);
        return smem + base + (r - l) * (PT && l ? RS2 : RS);
    };
    const int nz = a.nz, ny = a.ny, nx = a.nx;
    const int lane = threadIdx.x & 63;
    const int x = xs + 4 * lane;
    const bool xin = x < nx;
    const size_t plane = (size_t)ny * nx;
    const int zs = z0 - K + 1;  // zl: the row waves' last front plane (they may run past z1 + K - 2)
    auto P = [&](int p) { return a.in + (size_t)p * plane; };
    auto fixedp = [&](int p) { return (p == a.zb - 1 && a.fixed_lo) || (p == a.ze && a.fixed_hi); };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // ------------------------------------------------------------ halo wave
    const int ylo = y0 - K, yhi = y0 - K + NR - 1;
    const bool elo = xin && ylo >= 0 && ylo <= ny - 1;
    const bool ehi = xin && yhi >= 0 && yhi <= ny - 1;
    const size_t olo = (size_t)(elo ? ylo : 0) * nx + (xin ? x : 0);
    const size_t ohi = (size_t)(ehi ? yhi : 0) * nx + (xin ? x : 0);
    const int hr = lane >> 1, side = lane & 1;
    const int yr = y0 - K + hr;
    const bool hact = lane < 2 * NR;
    const bool hon = hact && yr >= 0 && yr <= ny - 1 && (side ? xs + 256 < nx : xs > 0);
    const bool hint = hon && yr >= 1 && yr <= ny - 2;
    const int hx = side ? xs + 256 : xs - 4;
    const size_t hofs = (size_t)(hon ? yr : 0) * nx + (hon ? hx : 0);
    const int col = side ? 260 : 0;
    constexpr bool ZERO = (F & kFirstZero) != 0;  // level 0 = 0: no phi loads
    auto ldh = [&](const float *base, int p) {
        return (hon && p >= 0 && p <= nz - 1) ? ldg4(base + (size_t)p * plane + hofs) : z4;
    };
    auto ldhp = [&](int p) { return ZERO ? z4 : ldh(a.in, p); };
    auto ldlo = [&](int p) { return (!ZERO && elo && p >= 0 && p <= nz - 1) ? ldg4(P(p) + olo) : z4; };
    auto ldhi = [&](int p) { return (!ZERO && ehi && p >= 0 && p <= nz - 1) ? ldg4(P(p) + ohi) : z4; };
    float4 lo = ldlo(zs), hi = ldhi(zs);
    float4 H[K][3];
    float4 Hr[K];
#pragma unroll
    for (int l = 0; l < K; ++l) H[l][0] = H[l][1] = H[l][2] = z4;
    H[0][0] = ldhp(zs - 1);
    H[0][1] = ldhp(zs);
    H[0][2] = ldhp(zs + 1);
#pragma unroll
    for (int i = 0; i < K; ++i) Hr[i] = ldh(a.div, zs - i);
    float4 Lq[PD], Uq[PD], Hq[PD], Rn[PD];
#pragma unroll
    for (int i = 0; i + 1 < PD; ++i) {
        Lq[i] = ldlo(zs + 1 + i);
        Uq[i] = ldhi(zs + 1 + i);
        Hq[i] = ldhp(zs + 2 + i);
        Rn[i] = ldh(a.div, zs + 1 + i);
    }
    const int hw = threadIdx.x >> 6;
    for (int z = zs; z <= zl; ++z) {
        if constexpr (T0S) t0 = ((z - zs) % 3) * (NR * RS);
        trace_mark(a.trace, hw, z - zs, 0);
        Lq[PD - 1] = ldlo(z + PD);
        Uq[PD - 1] = ldhi(z + PD);
        Hq[PD - 1] = ldhp(z + 1 + PD);
        Rn[PD - 1] = ldh(a.div, z + PD);
        // phase W
        if constexpr (SPLIT) {
            if (elo) sts4s(T(0, 0), lane, lo);
            if (ehi) sts4s(T(0, NR - 1), lane, hi);
        } else {
            if (elo) sts4(T(0, 0) + 4 + 4 * lane, lo);
            if (ehi) sts4(T(0, NR - 1) + 4 + 4 * lane, hi);
        }
        if (hon) {
            sts4(T(0, hr) + col, H[0][1]);
#pragma unroll
            for (int l = 1; l < K; ++l)
                if (hr >= l && hr < NR - l) {
                    if constexpr (PT) {  // the pair level l updated in plane z - l
                        const int hl = (a.zoff + (z - l) + yr + 1 + ((a.h0 + l - 1) & 1)) & 1;
                        *reinterpret_cast<v2f_t *>(T(l, hr) + (side ? 130 : 0)) = pick2(H[l][2], hl);
                    } else {
                        sts4(T(l, hr) + col, H[l][2]);
                    }
                }
        }
        trace_mark(a.trace, hw, z - zs, 1);
        __syncthreads();
        trace_mark(a.trace, hw, z - zs, 2);
        // phase R: levels 1..K-1 of the halo chunks
#pragma unroll
        for (int l = 1; l < K; ++l) {
            const int p = z - l + 1;
            if (hact && hr >= l && hr < NR - l) {
                const float4 c = H[l - 1][1];
                const int par = (a.zoff + p + yr + 1 + ((a.h0 + l - 1) & 1)) & 1;
                // the row wave's cell next to the chunk (xs, or xs + 255), level
                // l - 1; in a pair tile it is there when this level uses it (the
                // chunk updates its cell 3 / cell 0 next to it)
                const float inner = PT && l > 1 ? T(l - 1, hr)[side ? 129 : 2] : T(l - 1, hr)[side ? 259 : 4];
                float4 v = c;
                if (hon) {
                    float4 N, S;
                    if (PT && l > 1) {  // pairs at this level's positions
                        const v2f_t n2 = *reinterpret_cast<const v2f_t *>(T(l - 1, hr + 1) + (side ? 130 : 0));
                        const v2f_t s2 = *reinterpret_cast<const v2f_t *>(T(l - 1, hr - 1) + (side ? 130 : 0));
                        N = join2(n2, n2, par);
                        S = join2(s2, s2, par);
                    } else {
                        N = lds4(T(l - 1, hr + 1) + col);
                        S = lds4(T(l - 1, hr - 1) + col);
                    }
                    float dummy = 0.f;
                    v = level4<MODE, PRE>(c, side ? inner : 0.f, side ? 0.f : inner, N, S,
                                          H[l - 1][2], H[l - 1][0], Hr[l - 1], hx, nx,
                                          hint && !fixedp(p), a, par, false, dummy);
                }
                H[l][0] = H[l][1];
                H[l][1] = H[l][2];
                H[l][2] = v;
            }
        }
        trace_mark(a.trace, hw, z - zs, 3);
        __syncthreads();
        trace_mark(a.trace, hw, z - zs, 4);
        lo = Lq[0];
        hi = Uq[0];
        H[0][0] = H[0][1];
        H[0][1] = H[0][2];
        H[0][2] = Hq[0];
#pragma unroll
        for (int i = K - 1; i > 0; --i) Hr[i] = Hr[i - 1];
        Hr[0] = Rn[0];
#pragma unroll
        for (int i = 0; i + 1 < PD; ++i) {
            Lq[i] = Lq[i + 1];
            Uq[i] = Uq[i + 1];
            Hq[i] = Hq[i + 1];
            Rn[i] = Rn[i + 1];
        }
    }
}

// The halo wave as a called function (K <= 3: measured 1.5-2.5 % faster than
// inlined there); K = 4 inlines it (as a call it takes the TbrArgs by value in
// VGPRs and a call frame: 168-181 VGPRs, which spill).
template <int K, int NWR, int RPW, bool PRE, int PD, int MODE, int F, bool SPLIT, bool PT, bool T0S>
__device__ __noinline__ void tbr_halo_wave_call(const TbrArgs a, float *smem, int z0, int z1, int y0,
                                                int xs, int zl, float *slots) {
    tbr_halo_wave<K, NWR, RPW, PRE, PD, MODE, F, SPLIT, PT, T0S>(a, smem, z0, z1, y0, xs, zl, slots);
}

// (A double-buffered, one-barrier-per-step version of the (3, 11, 2) shape --
// 139 KB of LDS -- was measured at 1007 against 1131 Gcell/s for this one.)
// MODE kRbgs: K red-black half-sweeps per pass, level l = half-sweep h0+l-1
// (colour (h0+l-1) & 1, iteration (h0+l-1) / 2), so a pass may start or end
// inside an iteration; see rbgs3d_tbr_pass for the stop rule and the rollback.
// SHIFTQ: shifting register queues instead of the rotated ones (below) --
// for short z-chunks whose step count is no multiple of 6, where the rotated
// march would run up to 5 steps that store nothing (the slab boundary
// launches: 7 steps of which 12 would run)
template <int K, int NWR, int RPW, bool PRE, int PD, int MODE, int F = 0, bool SHIFTQ = false>
__global__ __launch_bounds__((NWR + 1) * 64) void jacobi3d_tbr(TbrArgs a) {
    constexpr int NR = NWR * RPW + 2;  // level-0 rows per tile
    constexpr int W = NR - 2 * K;      // output rows
    constexpr int RS = 264;            // LDS row: 4 halo | 256 | 4 halo floats
    static_assert(K >= 1 && K <= 4 && W >= 1, "bad shape");
    static_assert(2 * NR <= 64, "halo wave: one lane per (row, side)");
    // PT (red-black GS on the LDS-DMA path): the tiles of levels 1..K-1 hold
    // only the pair a level updated (kPairRow floats a row: the left chunk's
    // pair, 64 lanes' pairs, the right chunk's): a level's neighbours read
    // the pair at their own positions, which is the one the level below
    // updated (see the row wave); half the LDS of those tiles, so the rhs rows
    // come by LDS-DMA too at 4 levels
    constexpr bool PT = MODE == kRbgs && PD == 1 && K == 4;  // (at 3 levels: 16 VGPRs spill)
    constexpr int RS2 = kPairRow;
    // T0S (Jacobi, LDS-DMA path): the level-0 tile of plane z IS the DMA
    // staging slot that plane landed in -- a ring of 3 full tiles (planes z,
    // z + 1 landed, z + 2 in flight), the rows DMA'd straight to their tile
    // position and the halo wave adding the outer rows and x-halo chunks -- so
    // phase W no longer copies level 0 into a tile: a quarter of the K = 4
    // pass's LDS stores, the slow direction of the LDS (ds_write_b128 ~79
    // B/clk/CU against 256 for reads)
    constexpr bool T0S = MODE == kJacobi && PD == 1 && CFD_TBR_LB && CFD_TBR_T0S;
    constexpr int SLOT = NR * RS;
    constexpr int TOTAL = [] {
        int t = 0;
        for (int l = T0S ? 1 : 0; l < K; ++l) t += (NR - 2 * l) * (PT && l ? RS2 : RS);
        return t;
    }();
    __shared__ __attribute__((aligned(16))) float smem[TOTAL > 0 ? TOTAL : 4];
    __shared__ __attribute__((aligned(16))) float slots[T0S ? 3 * SLOT : 4];
    // DMA staging (row waves, when it fits in LDS with the level tiles): the
    // level-0 row of plane z + 2 and the rhs row of plane z + 1 are fetched by
    // LDS-DMA at the start of step z into the even/odd buffers and read at
    // step z + 1, so a fetch has a whole step in flight and holds no VGPRs.
    // Separate arrays per parity let the compiler see that step z's reads do
    // not alias step z's DMA (no vmcnt(0) before them).
    constexpr int SR_ = NR - 2;  // rows 1 .. NR-2 (the row waves' rows)
    // DMA: the phi rows by LDS-DMA; RDMA: the rhs rows too when both staging
    // pairs fit beside the level tiles, else the rhs row of plane z + 1 is a
    // register load issued a step ahead (4 VGPRs per row)
    constexpr int STG = T0S ? 3 * SLOT : 2 * SR_ * 256;  // the phi staging floats
    constexpr bool DMA = PD == 1 && (TOTAL + STG) * 4 <= 160 * 1024;
    constexpr bool RDMA = DMA && (TOTAL + STG + 2 * SR_ * 256) * 4 <= 160 * 1024;
    static_assert(!T0S || DMA, "T0S: the LDS-DMA path");
    // GS level-0 tile by colour pair (sts4s; at 3 levels every tile): +1.2 %
    // at K = 3
    constexpr bool SPLIT = MODE == kRbgs && DMA;
    // EARLY (DMA path): each step's staging rows are fetched two steps ahead,
    // in phase R right after the wave read its rows of the same buffer,
    // instead of one step ahead at the start of phase W
    constexpr bool EARLY = DMA && MODE == kRbgs && CFD_TBR_EARLY;
    constexpr int SST = DMA && !T0S ? SR_ * 256 : 4;
    constexpr int SSR = RDMA ? SR_ * 256 : 4;
    __shared__ __attribute__((aligned(16))) float st_p0[SST], st_p1[SST], st_r0[SSR], st_r1[SSR];
    // level l keeps rows [l, NR - l) (T0S: l >= 1 only; level 0 is a slot)
    auto T = [&](int l, int r) -> float * {
        int base = 0;
#pragma unroll
        for (int m = T0S ? 1 : 0; m < K; ++m)
            if (m < l) base += (NR - 2 * m) * (PT && m ? RS2 : RS);
        return smem + base + (r - l) * (PT && l ? RS2 : RS);
    };

    static_assert(!PT || DMA, "pair tiles: LDS-DMA path");
    static_assert(MODE == kJacobi || !PRE, "GS: raw div");
    static_assert(F == 0 || (MODE == kJacobi && !PRE && DMA), "first pass: Jacobi, raw div, DMA path");
    constexpr bool ZERO = (F & kFirstZero) != 0, RHSW = (F & kFirstRhs) != 0;
    constexpr bool PREL = PRE || RHSW;  // the row waves' queues hold the rhs
    // the rhs from raw div (RHSW), the same bits as k_rhs_f32
    auto torhs = [&](float4 d) {
        if constexpr (MODE == kRbgs) {  // -div * dt_inv (v5.py:209, rhs = -div / dt as * (1/dt))
            d.x = -d.x * a.dt_inv;
            d.y = -d.y * a.dt_inv;
            d.z = -d.z * a.dt_inv;
            d.w = -d.w * a.dt_inv;
        }
        if constexpr (RHSW) {
            d.x = (a.h2 * d.x) / a.dt;
            d.y = (a.h2 * d.y) / a.dt;
            d.z = (a.h2 * d.z) / a.dt;
            d.w = (a.h2 * d.w) / a.dt;
        }
        return d;
    };
    // GS iterations a pass touches: (h0 >> 1) + q, q < NIT (K = 3: one and a half)
    constexpr int NIT = MODE == kRbgs ? (K + 2) / 2 : 1;
    if (MODE == kRbgs) {
        if (a.rollback) {
            // The stop fell inside pass j* of a solve of P half-sweeps per pass
            // when the 2c half-sweeps of its c iterations end inside it: re-run
            // those of its half-sweeps that count (need = 2c - P j*) from the
            // pass's input buffer, which no later (skipped) pass overwrote, into
            // its output.  One launch per possible need; this one does K.
            const int P = a.rollback, H = 2 * *a.count;
            const int js = (H - 1) / P, need = H - P * js;
            if (need != K || need >= P || P * js + P > a.nhalf) return;
            a.h0 = P * js;
            if (js & 1) {  // pass j* read phi_tmp
                float *t_ = const_cast<float *>(a.in);
                a.in = a.out;
                a.out = t_;
            }
        } else {
            // skip when an iteration the previous pass completed met the
            // tolerance (v5.py:224-225); with a lag, the pass before that
            const int ic = a.h0 >> 1, d = 1 + a.lag;
            if ((ic >= d && a.maxc[ic - d] < a.tol) || (ic >= d + 1 && a.maxc[ic - d - 1] < a.tol))
                return;
        }
    }
    const int nz = a.nz, ny = a.ny, nx = a.nx;
    const int lane = threadIdx.x & 63;
    // wave index, uniform by construction: rows, row masks and colours derived
    // from it stay scalar
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int t = xcd_swizzle(blockIdx.x, gridDim.x);
    int seg = t % a.nseg;
    int ty = (t / a.nseg) % a.ntile_y;
    const int zc = t / (a.nseg * a.ntile_y);
    if (a.xbw) {  // XCD x takes a block of xbw segments x (per / xbw) tile rows
        const int per = gridDim.x / kNumXcd, x = t / per, k = t - x * per;
        const int nbx = a.nseg / a.xbw, bh = per / a.xbw;
        seg = (x % nbx) * a.xbw + k % a.xbw;
        ty = (x / nbx) * bh + k / a.xbw;
    }
    const int z0 = a.zb + zc * a.zchunk;
    if (z0 >= a.ze) return;  // workgroup-uniform
    const int z1 = min(z0 + a.zchunk, a.ze);
    const int y0 = 1 + ty * W;
    const int xs = seg * 256;
    const int x = xs + 4 * lane;
    const bool xin = x < nx;
    const size_t plane = (size_t)ny * nx;
    const int zs = z0 - K + 1;  // first front plane
    // last front plane; the LDS-DMA march runs whole groups of 6 steps (the
    // extra steps at the end compute planes past the chunk and store nothing)
    const int zl0 = z1 + K - 2;
    // register queues rotated by compile-time slots (see the DMA row wave) up
    // to 3 levels: -2.3 % per pass for the Jacobi at K = 3, -2.9 % for the
    // red-black GS (whose level queues hold pairs, so its two march copies fit
    // with them at 2 rows per wave); K = 4 spills with them (r03: 111 VGPRs
    // for the Jacobi, 34 for the GS -- although the shifting queues' moves are
    // about half of the K = 4 passes' VALU instructions)
    constexpr bool ROT = DMA && K <= 3 && (MODE == kJacobi || RPW <= 2) && !SHIFTQ;
    // (a K = 4 Jacobi with its rhs queue rotated with period 4 -- a march
    // unrolled by 4 -- spilled 22 VGPRs and took 4.96-5.04 ms per pass against
    // 2.71, r04: removed in r05)
    const int zl = ROT ? zs + 6 * ((zl0 - zs + 6) / 6) - 1 : zl0;
    auto P = [&](int p) { return a.in + (size_t)p * plane; };
    auto fixedp = [&](int p) { return (p == a.zb - 1 && a.fixed_lo) || (p == a.ze && a.fixed_hi); };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // GS: max|change| of own cells per level (a compile-time slot, one v_max
    // per update), folded into the pass's iterations after the march.  A
    // 4-level pass always starts at an even half-sweep (the solve's passes of
    // 4 from h0 = 0, slab passes from h0 = 2 it; rollbacks run 1 or 2
    // levels), so there levels 1, 2 and 3, 4 are one iteration each and share
    // a slot (2 VGPRs: no spill at 4 levels)
    constexpr int KS = MODE == kRbgs ? (K == 4 ? 2 : K) : 1;
    auto slot = [](int l) { return K == 4 ? (l - 1) >> 1 : l - 1; };
    float chgl[KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) chgl[i] = 0.f;
    auto fold = [&](int l, float lm) {
        if constexpr (MODE == kRbgs) chgl[slot(l)] = fmaxf(chgl[slot(l)], lm);
    };

    if constexpr (T0S && ZERO) {
        // level 0 = 0 (no DMA fills the slots): zero them once
        for (int k = threadIdx.x; k < 3 * SLOT / 4; k += blockDim.x) sts4(slots + 4 * k, z4);
        __syncthreads();
    }
    if (wv < NWR) {
        if constexpr (DMA) {
            // --------------------------------------------- row wave, DMA-staged
            int rr[RPW];
            uint32_t bo[RPW], so[RPW];  // load / store byte offsets in a plane, kOob outside
            bool irow[RPW], orow[RPW];
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                rr[j] = 1 + wv + j * NWR;
                const int y = y0 - K + rr[j];
                const bool rowin = y >= 0 && y <= ny - 1;
                irow[j] = y >= 1 && y <= ny - 2;
                orow[j] = rr[j] >= K && rr[j] < NR - K && y <= ny - 2 && xin;
                const uint32_t o = (uint32_t)(((size_t)(rowin ? y : 0) * nx + (xin ? x : 0)) * sizeof(float));
                bo[j] = xin && rowin ? o : kOob;
                so[j] = orow[j] ? o : kOob;
            }
            // V[j][i]: level 0 of plane z-1+i; Q[j][l][i]: level l of plane
            // (z-l)-1+i after level l is computed; Rq[j][i]: rhs of plane z-i
            // GS: Q holds only the pair a level updated (the other colour's
            // cells keep the previous level's values, which the level below
            // holds): half the registers of the level queues
            using QT = std::conditional_t<MODE == kRbgs, v2f_t, float4>;
            // Jacobi queue entries: Q4 (64-bit halves) or float4
            using JQ = std::conditional_t<CFD_TBR_Q64 != 0, Q4, float4>;
            // GS: V and Rq hold colour pairs (P4)
            using VT = std::conditional_t<MODE == kRbgs, P4, JQ>;
            using QQ = std::conditional_t<MODE == kRbgs, v2f_t, JQ>;
            auto toV = [](float4 f) -> VT {
                if constexpr (MODE == kRbgs)
                    return split4(f);
                else if constexpr (CFD_TBR_Q64 != 0)
                    return q4_of(f);
                else
                    return f;
            };
            VT V[RPW][3], Rq[RPW][K];
            QQ Q[RPW][K][3];
            float4 Rn[RPW];  // !RDMA: the rhs row of the next step's plane, in flight
            // Lane-based LDS addressing (Jacobi): every tile and staging access
            // of a row wave is one of a few per-wave base addresses (the lane's
            // float4 in the wave's first row; the level tiles past T_1 from a
            // second base, so offsets fit the 16-bit immediate) plus a
            // compile-time offset, folded into the DS instruction.  The bases
            // are made opaque once per step, so the compiler keeps 4 + 2 VGPRs
            // instead of hoisting one address per (level, row) out of the
            // z-loop -- which spilled 5 VGPRs at K = 4 whose scratch reloads
            // each waited vmcnt(0), i.e. for the DMAs of the next planes.
            constexpr bool LB = MODE == kJacobi && CFD_TBR_LB;
            // (T0S: tiles 1..K-1 all within the 16-bit offset of one base)
            constexpr int kTb2 = [] {  // first float of tile T_2 (0 when K < 3)
                int t = 0;
                for (int m = 0; m < 2 && m < K; ++m) t += (NR - 2 * m) * RS;
                return K >= 3 && !T0S ? t : 0;
            }();
            auto tbase = [](int l) {
                int t = 0;
                for (int m = T0S ? 1 : 0; m < l; ++m) t += (NR - 2 * m) * RS;
                return t;
            };
            [[maybe_unused]] const GsPk gk = MODE == kRbgs ? gs_pk(a) : GsPk{};
            const uint32_t lds_st_p0 = lds_addr(st_p0), lds_st_p1 = lds_addr(st_p1);
            const uint32_t lds_st_r0 = lds_addr(st_r0), lds_st_r1 = lds_addr(st_r1);
            (void)lds_st_p0;
            (void)lds_st_p1;
            (void)lds_st_r0;
            (void)lds_st_r1;
            const uint32_t lbA0 = lds_addr(smem) + 4u * (uint32_t)(wv * RS + 4 + 4 * lane);
            const uint32_t lbU0 = lds_addr(smem) + 4u * (uint32_t)(wv * RS);
            const uint32_t lbP00 = lds_addr(st_p0) + 4u * (uint32_t)(wv * 256 + 4 * lane);
            const uint32_t lbP10 = lds_addr(st_p1) + 4u * (uint32_t)(wv * 256 + 4 * lane);
            // T0S: the lane's float4 in row wv of slot 0, and row wv's first float
            const uint32_t lbS0 = lds_addr(slots) + 4u * (uint32_t)(wv * RS + 4 + 4 * lane);
            const uint32_t lbUS0 = lds_addr(slots) + 4u * (uint32_t)(wv * RS);
            // a row's DMA destination in slot q: row rr[j], column 4
            auto slot_row = [&](int q, int j) { return slots + q * SLOT + rr[j] * RS + 4; };
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
#pragma unroll
                for (int l = 0; l < K; ++l) Q[j][l][0] = Q[j][l][1] = Q[j][l][2] = QQ{};
                // planes zs - 1 and zs in slots 2 and 0 (slot (q - zs) mod 3), or 0
                // and 1 (shifted queues)
                V[j][ROT ? 2 : 0] = toV(ZERO ? z4 : ldb4(plane_rsrc(a.in, zs - 1, nz, plane), bo[j]));
                V[j][ROT ? 0 : 1] = toV(ZERO ? z4 : ldb4(plane_rsrc(a.in, zs, nz, plane), bo[j]));
                V[j][ROT ? 1 : 2] = toV(z4);
                // rhs rows of planes before zs only feed levels of planes below the
                // ones the outputs need (the pipeline fill), so they start at 0
#pragma unroll
                for (int i = 0; i < K; ++i) Rq[j][i] = toV(z4);
                // read at step zs (even): plane zs + 1 and rhs zs in the odd buffers
                // (T0S: planes zs and zs + 1 into slots 0 and 1)
                if constexpr (T0S) {
                    if (!ZERO) {
                        dma_row(plane_rsrc4(a.in, zs, nz, plane), bo[j], slot_row(0, j));
                        dma_row(plane_rsrc4(a.in, zs + 1, nz, plane), bo[j], slot_row(1, j));
                    }
                } else if (!ZERO) {
                    dma_row(plane_rsrc4(a.in, zs + 1, nz, plane), bo[j], st_p1 + (rr[j] - 1) * 256);
                }
                if constexpr (RDMA)
                    dma_row(plane_rsrc4(a.div, zs, nz, plane), bo[j], st_r1 + (rr[j] - 1) * 256);
                else
                    Rn[j] = ldb4(plane_rsrc(a.div, zs, nz, plane), bo[j]);
            }
            if constexpr (EARLY) {
                // and step zs + 1's (plane zs + 2, rhs zs + 1) in the even ones;
                // from then on step z fetches step z + 2's (see the step)
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    if (!ZERO) dma_row(plane_rsrc4(a.in, zs + 2, nz, plane), bo[j], st_p0 + (rr[j] - 1) * 256);
                    if constexpr (RDMA) dma_row(plane_rsrc4(a.div, zs + 1, nz, plane), bo[j], st_r0 + (rr[j] - 1) * 256);
                }
                wait_vmcnt<0>();
            }
            // XW (Jacobi): the prologue's loads land before the march, so the
            // waits the compiler places for them in the loop's first step are
            // no-ops (it does not count the LDS-DMAs, so a wait of its own for
            // an older load would wait for this step's DMAs as well)
            constexpr bool XW = MODE == kJacobi && !EARLY && CFD_TBR_XW;
            if constexpr (XW) wait_vmcnt<0>();
            // Register queues without moves: plane q of level 0 / level l lives
            // in slot (q - zs) mod 3 of V / Q[.][l], and (when the unroll
            // period 6 is a multiple of K) the rhs of plane q in slot
            // (q - zs) mod K of Rq; the march is unrolled by 6 so that every
            // slot index is a compile-time constant.  (K = 4 shifts Rq.)
            constexpr bool ROTR = ROT && 6 % K == 0;
            // memory operations per step and wave, for EARLY's vmcnt wait:
            // staging DMAs, !RDMA rhs loads, level-K stores (one per row, issued
            // for every row: see phase R), first-pass rhs stores
            constexpr int kND = ((ZERO ? 0 : 1) + (RDMA ? 1 : 0)) * RPW, kNR = RDMA ? 0 : RPW, kNSK = RPW,
                          kNSR = RHSW ? RPW : 0;
            static_assert(2 * kNSK + 2 * kNR + kNSR + kND < 64, "vmcnt range");
            // SD (Jacobi, XW): the per-step scalar state -- the plane bases of
            // the DMA source (in, plane z + 2), the rhs loads (div, z + 1), the
            // level-K stores (out, z - K + 1) and the first pass's rhs stores
            // (rhs_out, z), and the slot ring's byte offsets -- carried from
            // step to step by additions and rotations.  Recomputed per step
            // they were ~80 SALU per wave in phase W (64-bit products, a
            // division by 3), and the CU's one scalar unit serialised the 12
            // waves' phase W (r05 trace: the third wave of each SIMD reached
            // the first barrier ~1150 cycles after the first)
            // (the red-black GS's EARLY path too: its DMAs fetch planes z + 3 / rhs z + 2)
            constexpr bool SD = (XW || EARLY) && CFD_TBR_SD;
            constexpr int kAh = EARLY ? 3 : 2;  // plane of the step's phi DMA, relative to z
            const uint64_t pbytes = (uint64_t)plane * sizeof(float);
            uint64_t sd_in = (uint64_t)(uintptr_t)a.in + (uint64_t)(int64_t)(zs + kAh) * pbytes;
            uint64_t sd_div = (uint64_t)(uintptr_t)a.div + (uint64_t)(int64_t)(zs + kAh - 1) * pbytes;
            uint64_t sd_out = (uint64_t)(uintptr_t)a.out + (uint64_t)(int64_t)(zs - K + 1) * pbytes;
            uint64_t sd_rhs = (uint64_t)(uintptr_t)a.rhs_out + (uint64_t)(int64_t)zs * pbytes;
            int sd_oz = 0, sd_on = 4 * SLOT, sd_od = 8 * SLOT;  // slot byte offsets: planes z, z + 1, z + 2
            // the launch's fixed (Dirichlet) planes, or a plane no step reaches
            const int sd_flo = a.fixed_lo ? a.zb - 1 : -(1 << 30), sd_fhi = a.fixed_hi ? a.ze : -(1 << 30);
            // a raw buffer resource over one plane at byte address b (empty unless ok)
            auto rsrc4 = [&](uint64_t b, bool ok) {
                v4i32 r;
                r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
                r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xffffu));
                r.z = __builtin_amdgcn_readfirstlane(ok ? (int)pbytes : 0);
                r.w = 0x00020000;
                return r;
            };
            auto rsrc = [&](uint64_t b, bool ok) {
                return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)b, (short)0, ok ? (int)pbytes : 0,
                                                         0x00020000);
            };
            (void)rsrc4;
            (void)rsrc;
            auto step = [&](int z, auto parc, auto rotc, auto bpc) {
                constexpr int E = decltype(parc)::value;  // (z - zs) & 1
                constexpr int R = decltype(rotc)::value;  // (z - zs) mod 6 (ROT), else 0
                // queue slots: level 0 / level l-1 at planes p (C), p + 1 (U), p - 1 (D)
                // of level l's plane p = z - l + 1; the slot level l's new value takes
                auto vs = [](int d) { return ROT ? sl3(R + d) : d + 1; };        // V: plane z + d
                auto qs = [](int l, int d) { return ROT ? sl3(R - l - 1 + d) : d; }; // Q[l]: plane z - l - 1 + d
                // GS colour parity of row j at this step, for every level:
                // (zoff + p + y + 1 + h0 + l - 1) with p = z - l + 1 and z = zs + E
                // is BP ^ E ^ (j * NWR) mod 2 (BP: see march)
                constexpr int BPv = decltype(bpc)::value;
                trace_mark(a.trace, wv, z - zs, 0);
                float *const pw = E ? st_p1 : st_p0;
                float *const rw = E ? st_r1 : st_r0;
                const float *const pr = E ? st_p0 : st_p1;
                const float *const rdr = E ? st_r0 : st_r1;
                // LB: this step's opaque bases; tp(l, d): the lane's float4 of
                // level tile l in row rr[j] + d (d = j * NWR + delta); up(l, d):
                // that row's first float (uniform)
                // T0S: slot sz holds plane z (this step's level 0), sn plane
                // z + 1 (landed), sd receives plane z + 2
                const int sz = T0S && !SD ? (z - zs) % 3 : 0;
                const int sn = sz == 2 ? 0 : sz + 1, sd = sn == 2 ? 0 : sn + 1;
                // byte offsets of the slots of planes z, z + 1, z + 2
                const uint32_t oz = SD ? (uint32_t)sd_oz : 4u * (uint32_t)(sz * SLOT);
                const uint32_t on = SD ? (uint32_t)sd_on : 4u * (uint32_t)(sn * SLOT);
                const uint32_t od = SD ? (uint32_t)sd_od : 4u * (uint32_t)(sd * SLOT);
                uint32_t bA = lbA0, bU = lbU0, bP = E ? lbP00 : lbP10;
                uint32_t bS = lbS0 + oz, bSn = lbS0 + on;
                uint32_t bUS = lbUS0 + oz;
                if constexpr (LB && T0S)
                    asm volatile("" : "+v"(bA), "+v"(bU), "+v"(bS), "+v"(bSn), "+v"(bUS));
                else if constexpr (LB)
                    asm volatile("" : "+v"(bA), "+v"(bU), "+v"(bP));
                const uint32_t bB = bA + 4u * kTb2, bUB = bU + 4u * kTb2;
                auto tp = [&](int l, int d) -> lfloat * {
                    if (T0S && l == 0) return lds_ptr(bS) + (1 + d) * RS;
                    return l < 2 ? lds_ptr(bA) + (tbase(l) + (1 + d - l) * RS)
                                 : lds_ptr(bB) + (tbase(l) - kTb2 + (1 + d - l) * RS);
                };
                auto up = [&](int l, int d) -> const lfloat * {
                    if (T0S && l == 0) return lds_ptr(bUS) + (1 + d) * RS;
                    return l < 2 ? lds_ptr(bU) + (tbase(l) + (1 + d - l) * RS)
                                 : lds_ptr(bUB) + (tbase(l) - kTb2 + (1 + d - l) * RS);
                };
                (void)sd;
                (void)tp;
                (void)up;
                // !RDMA: this step's rhs row (loaded last step) and the next one's load
                float4 Rc[RPW];
                if constexpr (!RDMA && XW) {
#pragma unroll
                    for (int j = 0; j < RPW; ++j) Rc[j] = Rn[j];  // landed: see phase R
                }
                if constexpr (!EARLY) {
                    const v4i32 rp = SD ? rsrc4(sd_in, z + 2 >= 0 && z + 2 <= nz - 1) : plane_rsrc4(a.in, z + 2, nz, plane);
                    const v4i32 rd = SD ? rsrc4(sd_div, z + 1 >= 0 && z + 1 <= nz - 1) : plane_rsrc4(a.div, z + 1, nz, plane);
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        if (!ZERO)
                            dma_row(rp, bo[j],
                                    T0S ? (SD ? (float *)((char *)slots + od) + rr[j] * RS + 4 : slot_row(sd, j))
                                        : pw + (rr[j] - 1) * 256);
                        if constexpr (RDMA) dma_row(rd, bo[j], rw + (rr[j] - 1) * 256);
                    }
                } else {
                    (void)pw;
                    (void)rw;
                }
                if constexpr (!RDMA) {
                    (void)rw;
                    (void)rdr;
                    const __amdgpu_buffer_rsrc_t rdn =
                        SD ? rsrc(sd_div - (EARLY ? pbytes : 0), z + 1 >= 0 && z + 1 <= nz - 1)  // (sd_div: rhs z + kAh - 1)
                           : plane_rsrc(a.div, z + 1, nz, plane);
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        if constexpr (!XW) Rc[j] = Rn[j];
                        Rn[j] = ldb4(rdn, bo[j]);
                    }
                }
                // phase W: level 0 of plane z and level l of plane z - l
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    if (xin && !T0S) {  // (T0S: level 0 is in its slot already)
                        if constexpr (SPLIT)
                            sts4s(T(0, rr[j]), lane, f4_of(V[j][vs(0)]));
                        else if constexpr (LB)
                            sts4l(tp(0, j * NWR), f4_of(V[j][vs(0)]));
                        else
                            sts4(T(0, rr[j]) + 4 + 4 * lane, f4_of(V[j][vs(0)]));
                    }
#pragma unroll
                    for (int l = 1; l < K; ++l)
                        if (xin && rr[j] >= l && rr[j] < NR - l) {
                            if constexpr (MODE == kRbgs) {
                                // level l of plane z - l: its own pair (computed last
                                // step, at 1 - h) joined with level l - 1's (two steps
                                // ago, at h) -- or level 0's
                                const int h = (BPv ^ E ^ (j * NWR)) & 1;
                                const v2f_t lo = l == 1 ? pick2(V[j][vs(-1)], h)
                                                        : Q[j][l - 1][ROT ? sl3(R - l) : 1];
                                if constexpr (PT) {  // its own pair only
                                    (void)lo;
                                    *reinterpret_cast<v2f_t *>(T(l, rr[j]) + 2 + 2 * lane) =
                                        Q[j][l][ROT ? sl3(R - l) : 2];
                                } else {
                                    const float4 f = join2(lo, Q[j][l][ROT ? sl3(R - l) : 2], h);
                                    if constexpr (SPLIT)
                                        sts4s(T(l, rr[j]), lane, f);
                                    else
                                        sts4(T(l, rr[j]) + 4 + 4 * lane, f);
                                }
                            } else if constexpr (LB) {
                                sts4l(tp(l, j * NWR), f4_of(Q[j][l][ROT ? sl3(R - l) : 2]));
                            } else {
                                sts4(T(l, rr[j]) + 4 + 4 * lane, f4_of(Q[j][l][ROT ? sl3(R - l) : 2]));
                            }
                        }
                }
                // this step's DMAs have landed once at most the memory
                // operations issued after them remain in flight (vmcnt counts
                // in issue order): without EARLY, this step's 2 * RPW
                // fetches (the next step's rows); with EARLY (issued in step
                // z - 2's phase R), step z - 2's level-K stores, the !RDMA rhs
                // loads of steps z - 1 and z, step z - 1's rhs stores (first
                // pass) and DMAs, and step z - 1's level-K stores
                if constexpr (EARLY)
                    wait_vmcnt<2 * kNSK + 2 * kNR + kNSR + kND>();
                else if constexpr (XW)
                    // issued after step z - 1's DMAs: its rhs loads, rhs
                    // stores (first pass), 0..RPW level-K stores, and this
                    // step's DMAs and rhs loads -- so last step's level-K
                    // stores may still be in flight
                    wait_vmcnt<2 * kNR + kNSR + kND>();
                else
                    wait_vmcnt<((ZERO ? 0 : 1) + 1) * RPW>();
                trace_mark(a.trace, wv, z - zs, 1);
                lds_barrier();
                trace_mark(a.trace, wv, z - zs, 2);
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    if constexpr (MODE == kRbgs)
                        V[j][vs(1)] = ldsp(pr + (rr[j] - 1) * 256 + 4 * lane);
                    else if constexpr (LB && T0S)
                        V[j][vs(1)] = toV(ZERO ? z4 : lds4l(lds_ptr(bSn) + (1 + j * NWR) * RS));
                    else if constexpr (LB)
                        V[j][vs(1)] = toV(ZERO ? z4 : lds4l(lds_ptr(bP) + j * NWR * 256));
                    else
                        V[j][vs(1)] = toV(ZERO ? z4 : lds4(pr + (rr[j] - 1) * 256 + 4 * lane));
                    constexpr int RS0 = ROTR ? slk(R, K) : 0;  // slot of this step's rhs
                    if constexpr (!ROTR) {
#pragma unroll
                        for (int i = K - 1; i > 0; --i) Rq[j][i] = Rq[j][i - 1];
                    }
                    if constexpr (RDMA && MODE == kRbgs) {
                        // -div * dt_inv on the pairs (each element the scalar form)
                        P4 d = ldsp(rdr + (rr[j] - 1) * 256 + 4 * lane);
                        d.e = d.e * gk.ndt;  // (-x) * y == -(x * y): the same bits as -div * dt_inv
                        d.o = d.o * gk.ndt;
                        Rq[j][RS0] = d;
                    } else if constexpr (RDMA) {
                        Rq[j][RS0] = toV(torhs(lds4(rdr + (rr[j] - 1) * 256 + 4 * lane)));
                    } else {
                        Rq[j][RS0] = toV(torhs(Rc[j]));
                    }
                    if constexpr (RHSW) {
                        // the rhs of plane z for the later passes: owned planes and
                        // rows only (so[j] = kOob elsewhere), every x of the row
                        const bool own = z >= z0 && z < z1;
                        const __amdgpu_buffer_rsrc_t ro =
                            SD ? rsrc(sd_rhs, own)
                               : __builtin_amdgcn_make_buffer_rsrc(a.rhs_out + (size_t)(own ? z : 0) * plane, (short)0,
                                                                   own ? (int)(plane * sizeof(float)) : 0, 0x00020000);
                        const float4 rq = f4_of(Rq[j][RS0]);
                        const gv4f rv = {rq.x, rq.y, rq.z, rq.w};
                        __builtin_amdgcn_raw_buffer_store_b128(rv, ro, (int)so[j], 0, kStoreNt);
                    }
                }
                if constexpr (EARLY) {
                    // the staging rows just read are this wave's own: once the
                    // reads are done, fetch step z + 2's rows into them (plane
                    // z + 3, rhs z + 2), two steps ahead and off phase W
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const v4i32 rp = SD ? rsrc4(sd_in, z + 3 >= 0 && z + 3 <= nz - 1) : plane_rsrc4(a.in, z + 3, nz, plane);
                    const v4i32 rd = SD ? rsrc4(sd_div, z + 2 >= 0 && z + 2 <= nz - 1) : plane_rsrc4(a.div, z + 2, nz, plane);
                    // destinations as 32-bit LDS addresses (the staging rows'
                    // generic pointers, hoisted out of the march, were 64-bit
                    // SGPR pairs with a null-check select each: r05's in-loop
                    // SGPR spills to VGPR lanes)
                    const uint32_t lpr = E ? lds_st_p0 : lds_st_p1, lrr = E ? lds_st_r0 : lds_st_r1;
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        const uint32_t ro_ = 1024u * (uint32_t)(rr[j] - 1);
                        if (!ZERO) dma_row_at(rp, bo[j], lpr + ro_);
                        if constexpr (RDMA) dma_row_at(rd, bo[j], lrr + ro_);
                    }
                }
                // phase R: level l of plane p = z - l + 1, one (level, row)
                // at a time.  (Reading the next update's LDS operands before
                // this one computes -- they all come from tiles phase W wrote
                // -- ran at 3.40 against 2.24 ms per K = 3 pass: 17 VGPRs of
                // spill.)
                struct LdsIn {
                    QT N, S;       // rows r + 1, r - 1 of level l - 1 (GS: the pair)
                    float wl, er;  // the x-halo cells xs - 1, xs + 256
                };
                auto fetch = [&](int l, int j) {
                    const int r = rr[j];
                    LdsIn o;
                    const float *row = T(l - 1, r);
                    if constexpr (MODE == kRbgs) {
                        const int h = (BPv ^ E ^ (j * NWR)) & 1;
                        // cell xs - 1 (the left chunk's cell 3) and xs + 256 (the
                        // right chunk's cell 0), level l - 1; in a pair tile the
                        // left pair holds cells 1, 3 when h = 0 and the right one
                        // cells 0, 2 when h = 1, the cases that read them
                        const bool pt = PT && l > 1;
                        o.wl = pt ? row[1] : row[3];
                        o.er = pt ? row[130] : row[260];
                        if (pt) {
                            o.N = *reinterpret_cast<const v2f_t *>(T(l - 1, r + 1) + 2 + 2 * lane);
                            o.S = *reinterpret_cast<const v2f_t *>(T(l - 1, r - 1) + 2 + 2 * lane);
                        } else if (SPLIT) {
                            o.N = lds2s(T(l - 1, r + 1), lane, h);
                            o.S = lds2s(T(l - 1, r - 1), lane, h);
                        } else {
                            o.N = pick2(lds4(T(l - 1, r + 1) + 4 + 4 * lane), h);
                            o.S = pick2(lds4(T(l - 1, r - 1) + 4 + 4 * lane), h);
                        }
                    } else if constexpr (LB) {
                        (void)row;
                        o.wl = up(l - 1, j * NWR)[3];
                        o.er = up(l - 1, j * NWR)[260];
                        o.N = lds4l(tp(l - 1, j * NWR + 1));
                        o.S = lds4l(tp(l - 1, j * NWR - 1));
                    } else {
                        o.wl = row[3];
                        o.er = row[260];
                        o.N = lds4(T(l - 1, r + 1) + 4 + 4 * lane);
                        o.S = lds4(T(l - 1, r - 1) + 4 + 4 * lane);
                    }
                    return o;
                };
#pragma unroll
                for (int l = 1; l <= K; ++l) {
                    const int p = z - l + 1;
                    // (SD: two compares against the fixed planes found once per launch)
                    const bool fx = SD ? ((p == sd_flo) | (p == sd_fhi)) : fixedp(p);
                    if (!RDMA && XW && l == K) {
                        // the next step's rhs rows (loaded at this step's
                        // start) taken into registers here, as late as
                        // possible but before this step's level-K stores: the
                        // compiler's wait for them then counts only the first
                        // pass's rhs stores after them and nothing it cannot
                        // see (the LDS-DMAs); a wait counted from the next
                        // step would also wait for that step's DMAs
#pragma unroll
                        for (int j = 0; j < RPW; ++j) {
                            gv4f r4 = {Rn[j].x, Rn[j].y, Rn[j].z, Rn[j].w};
                            asm volatile("" : "+v"(r4));
                            Rn[j] = make_float4(r4.x, r4.y, r4.z, r4.w);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        const int r = rr[j];
                        if constexpr (MODE == kRbgs) {
                          if (r >= l && r < NR - l) {
                            // the colour's cells h, h + 2 of plane p: their old values
                            // (level l - 2's pair, or level 0), the other colour's pair
                            // of the same row (level l - 1) for E / W, level l - 1's
                            // pairs of planes p +- 1 and rows r +- 1 (same positions)
                            const int h = (BPv ^ E ^ (j * NWR)) & 1;
                            const v2f_t Cp = l == 1   ? pick2(V[j][vs(0)], h)
                                             : l == 2 ? pick2(V[j][vs(-1)], h)
                                                      : Q[j][l - 2][qs(l - 2, 0)];
                            const v2f_t Op = l == 1 ? pick2(V[j][vs(0)], 1 - h) : Q[j][l - 1][qs(l - 1, 1)];
                            const v2f_t Up = l == 1 ? pick2(V[j][vs(1)], h) : Q[j][l - 1][qs(l - 1, 2)];
                            const v2f_t Dp = l == 1 ? pick2(V[j][vs(-1)], h) : Q[j][l - 1][qs(l - 1, 0)];
                            const LdsIn in = fetch(l, j);
                            // lanes 0 / 63 take the x-halo cells as the DPP
                            // shifts' `old` operand: no lane-mask select (the
                            // two lane masks were SGPR pairs held across the
                            // march)
                            const float wl = dpp_from_lower_old(in.wl, Op.y), er = dpp_from_upper_old(in.er, Op.x);
                            // every lane computes (one beyond nx reads zeros and is
                            // never stored: its LDS writes and HBM store are masked)
                            const v2f_t v = level2(Cp, Op, wl, er, in.N, in.S, Up, Dp,
                                                   pick2(Rq[j][ROTR ? slk(R - l + 1, K) : l - 1], h), h, x, nx,
                                                   irow[j] && !fx, gk, orow[j] && p >= z0 && p < z1, chgl[slot(l)]);
                            if (l < K) {
                                if constexpr (ROT) {
                                    Q[j][l][sl3(R - l + 1)] = v;
                                } else {
                                    Q[j][l][0] = Q[j][l][1];
                                    Q[j][l][1] = Q[j][l][2];
                                    Q[j][l][2] = v;
                                }
                            } else {
                                // level K of plane p: this pair at h, level K - 1's at 1 - h
                                const float4 f = join2(v, Op, h);
                                const bool own = p >= z0 && p < z1;
                                const __amdgpu_buffer_rsrc_t ro =
                                    SD ? rsrc(sd_out, own)
                                       : __builtin_amdgcn_make_buffer_rsrc(a.out + (size_t)(own ? p : 0) * plane,
                                                                           (short)0,
                                                                           own ? (int)(plane * sizeof(float)) : 0,
                                                                           0x00020000);
                                const gv4f vv = {f.x, f.y, f.z, f.w};
                                __builtin_amdgcn_raw_buffer_store_b128(vv, ro, (int)so[j], 0, kStoreNt);
                            }
                          }
                        } else if (r >= l && r < NR - l) {
                            // level l-1 at planes p (c), p + 1 (U), p - 1 (D)
                            const float4 c = f4_of(l == 1 ? V[j][vs(0)] : Q[j][l - 1][qs(l - 1, 1)]);
                            const float4 U = f4_of(l == 1 ? V[j][vs(1)] : Q[j][l - 1][qs(l - 1, 2)]);
                            const float4 D = f4_of(l == 1 ? V[j][vs(-1)] : Q[j][l - 1][qs(l - 1, 0)]);
                            const LdsIn in = fetch(l, j);
                            // (lanes 0 / 63: the x-halo cells, as the GS branch)
                            const float wl = dpp_from_lower_old(in.wl, c.w);
                            const float er = dpp_from_upper_old(in.er, c.x);
                            float lm = 0.f;
                            // every lane (see the GS branch)
                            const float4 v = level4<MODE, PREL, K == 4>(c, wl, er, in.N, in.S, U, D,
                                                                f4_of(Rq[j][ROTR ? slk(R - l + 1, K) : l - 1]), x, nx,
                                                                irow[j] && !fx, a, (BPv ^ E ^ (j * NWR)) & 1,
                                                                orow[j] && p >= z0 && p < z1, lm);
                            fold(l, lm);
                            if (l < K) {
                                if constexpr (ROT) {
                                    Q[j][l][sl3(R - l + 1)] = toV(v);  // over plane p - 3, dead
                                } else {
                                    Q[j][l][0] = Q[j][l][1];
                                    Q[j][l][1] = Q[j][l][2];
                                    Q[j][l][2] = toV(v);
                                }
                            } else {
                                // unconditional buffer store: rows, lanes and planes this
                                // tile does not own fall out of range and are dropped
                                const bool own = p >= z0 && p < z1;
                                const __amdgpu_buffer_rsrc_t ro =
                                    SD ? rsrc(sd_out, own)
                                       : __builtin_amdgcn_make_buffer_rsrc(a.out + (size_t)(own ? p : 0) * plane,
                                                                           (short)0,
                                                                           own ? (int)(plane * sizeof(float)) : 0,
                                                                           0x00020000);
                                const gv4f vv = {v.x, v.y, v.z, v.w};
                                __builtin_amdgcn_raw_buffer_store_b128(vv, ro, (int)so[j], 0, kStoreNt);
                            }
                        }
                        if (EARLY && l == K && !(r >= l && r < NR - l)) {
                            // a row outside level K's range still issues its store
                            // (to an empty resource: dropped), so that every step
                            // has kNSK of them for EARLY's vmcnt count
                            const __amdgpu_buffer_rsrc_t ro =
                                __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, 0, 0x00020000);
                            __builtin_amdgcn_raw_buffer_store_b128(gv4f{0.f, 0.f, 0.f, 0.f}, ro, (int)kOob, 0, kStoreNt);
                        }
                        // one (level, row) at a time at K <= 3 (measured 0.4 % faster
                        // than letting the scheduler interleave them, r01); at K = 4
                        // the interleaved schedule is 0.3-0.4 % faster (r03)
                        if constexpr (K <= 3) __builtin_amdgcn_sched_barrier(0);
                    }
                }
                trace_mark(a.trace, wv, z - zs, 3);
                lds_barrier();
                trace_mark(a.trace, wv, z - zs, 4);
                if constexpr (SD) {
                    sd_in += pbytes;
                    sd_div += pbytes;
                    sd_out += pbytes;
                    sd_rhs += pbytes;
                    const int t_ = sd_oz;
                    sd_oz = sd_on;
                    sd_on = sd_od;
                    sd_od = t_;
                }
                if constexpr (!ROT) {
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        V[j][0] = V[j][1];
                        V[j][1] = V[j][2];
                    }
                }
            };
            // the z-march, instantiated per base colour parity BP (wave-uniform:
            // zoff + zs + y0 + K + wv + h0) so that every level's colour is a
            // compile-time constant in the GS (one copy for Jacobi)
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            auto march = [&](auto bpc) {
                if constexpr (!ROT) {
                    for (int zb = zs; zb <= zl; zb += 2) {
                        step(zb, I0{}, I0{}, bpc);
                        if (zb + 1 <= zl) step(zb + 1, I1{}, I0{}, bpc);
                    }
                    return;
                }
                for (int zb = zs; zb <= zl; zb += 6) {  // zl - zs + 1 is a multiple of 6
                    step(zb, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, bpc);
                    step(zb + 1, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}, bpc);
                    step(zb + 2, std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{}, bpc);
                    step(zb + 3, std::integral_constant<int, 1>{}, std::integral_constant<int, 3>{}, bpc);
                    step(zb + 4, std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{}, bpc);
                    step(zb + 5, std::integral_constant<int, 1>{}, std::integral_constant<int, 5>{}, bpc);
                }
            };
            if (MODE == kRbgs && ((a.zoff + zs + y0 + K + wv + a.h0) & 1))
                march(std::integral_constant<int, 1>{});
            else
                march(std::integral_constant<int, 0>{});
            wait_vmcnt<0>();  // no LDS-DMA outlives the wave
        } else {
            // ------------------------------------------------------------ row wave
            int rr[RPW];
            size_t ofs[RPW];
            bool ld[RPW], irow[RPW], orow[RPW];
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
                rr[j] = 1 + wv + j * NWR;
                const int y = y0 - K + rr[j];
                const bool rowin = y >= 0 && y <= ny - 1;
                ld[j] = xin && rowin;
                irow[j] = y >= 1 && y <= ny - 2;
                orow[j] = rr[j] >= K && rr[j] < NR - K && y <= ny - 2 && xin;
                ofs[j] = (size_t)(rowin ? y : 0) * nx + (xin ? x : 0);
            }
            auto ldp = [&](int j, int p) {
                return (ld[j] && p >= 0 && p <= nz - 1) ? ldg4(P(p) + ofs[j]) : z4;
            };
            auto ldr = [&](int j, int p) {
                return (ld[j] && p >= 0 && p <= nz - 1) ? ldg4(a.div + (size_t)p * plane + ofs[j]) : z4;
            };
            float4 Q[RPW][K][3];  // Q[j][l][i] = level l of plane (z - l) - 1 + i, row j
            float4 Rq[RPW][K];    // Rq[j][i] = rhs of plane z - i
            float4 Cq[RPW][PD], Rn[RPW][PD];
#pragma unroll
            for (int j = 0; j < RPW; ++j) {
#pragma unroll
                for (int l = 0; l < K; ++l) Q[j][l][0] = Q[j][l][1] = Q[j][l][2] = z4;
                Q[j][0][0] = ldp(j, zs - 1);
                Q[j][0][1] = ldp(j, zs);
                Q[j][0][2] = ldp(j, zs + 1);
#pragma unroll
                for (int i = 0; i < K; ++i) Rq[j][i] = ldr(j, zs - i);
#pragma unroll
                for (int i = 0; i + 1 < PD; ++i) {
                    Cq[j][i] = ldp(j, zs + 2 + i);
                    Rn[j][i] = ldr(j, zs + 1 + i);
                }
            }
            for (int z = zs; z <= zl; ++z) {
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    Cq[j][PD - 1] = ldp(j, z + 1 + PD);
                    Rn[j][PD - 1] = ldr(j, z + PD);
                }
                // phase W
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    if (ld[j]) sts4(T(0, rr[j]) + 4 + 4 * lane, Q[j][0][1]);
#pragma unroll
                    for (int l = 1; l < K; ++l)
                        if (xin && rr[j] >= l && rr[j] < NR - l) sts4(T(l, rr[j]) + 4 + 4 * lane, Q[j][l][2]);
                }
                __syncthreads();
                // phase R
#pragma unroll
                for (int l = 1; l <= K; ++l) {
                    const int p = z - l + 1;
                    const bool fx = fixedp(p);
#pragma unroll
                    for (int j = 0; j < RPW; ++j) {
                        const int r = rr[j];
                        if (r >= l && r < NR - l) {
                            const float4 c = Q[j][l - 1][1];
                            float wl = __shfl_up(c.w, 1, 64);
                            float er = __shfl_down(c.x, 1, 64);
                            const float *row = T(l - 1, r);
                            const float wl_l = row[3], er_l = row[260];
                            if (lane == 0) wl = wl_l;
                            if (lane == 63) er = er_l;
                            float4 v = c;
                            if (xin) {
                                const float4 N = lds4(T(l - 1, r + 1) + 4 + 4 * lane);
                                const float4 S = lds4(T(l - 1, r - 1) + 4 + 4 * lane);
                                const int y = y0 - K + r;
                                float lm = 0.f;
                                v = level4<MODE, PRE>(c, wl, er, N, S, Q[j][l - 1][2], Q[j][l - 1][0],
                                                      Rq[j][l - 1], x, nx, irow[j] && !fx, a,
                                                      (a.zoff + p + y + 1 + ((a.h0 + l - 1) & 1)) & 1,
                                                      orow[j] && p >= z0 && p < z1, lm);
                                fold(l, lm);
                            }
                            if (l < K) {
                                Q[j][l][0] = Q[j][l][1];
                                Q[j][l][1] = Q[j][l][2];
                                Q[j][l][2] = v;
                            } else if (orow[j] && p >= z0 && p < z1) {
                                stg4(a.out + (size_t)p * plane + ofs[j], v);
                            }
                        }
                    }
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < RPW; ++j) {
                    Q[j][0][0] = Q[j][0][1];
                    Q[j][0][1] = Q[j][0][2];
                    Q[j][0][2] = Cq[j][0];
#pragma unroll
                    for (int i = K - 1; i > 0; --i) Rq[j][i] = Rq[j][i - 1];
                    Rq[j][0] = Rn[j][0];
#pragma unroll
                    for (int i = 0; i + 1 < PD; ++i) {
                        Cq[j][i] = Cq[j][i + 1];
                        Rn[j][i] = Rn[j][i + 1];
                    }
                }
            }
        }
    } else {
        // the halo wave (see tbr_halo_wave_call).  Its global loads are plain
        // register loads; at K = 4 they run HPD = 2 planes ahead (the halo wave
        // is on that step's critical path: 2.976 -> 2.891 ms per pass); at
        // K <= 3 one plane (two: neutral for the Jacobi, -2 % for the GS,
        // which then spills a VGPR)
        constexpr int HPD = DMA && K == 4 ? 2 : PD;
        if constexpr (K == 4)
            tbr_halo_wave<K, NWR, RPW, PRE, HPD, MODE, F, SPLIT, PT, T0S>(a, smem, z0, z1, y0, xs, zl, slots);
        else
            tbr_halo_wave_call<K, NWR, RPW, PRE, HPD, MODE, F, SPLIT, PT, T0S>(a, smem, z0, z1, y0, xs, zl, slots);
    }
    if (MODE == kRbgs && a.maxc) {
        // level l is iteration (h0 >> 1) + q(l), q(l) = ((h0 & 1) + l - 1) >> 1
        float chg[NIT];
#pragma unroll
        for (int i = 0; i < NIT; ++i) chg[i] = 0.f;
#pragma unroll
        for (int l = 1; l <= (MODE == kRbgs ? K : 1); ++l) {
            const int q = ((a.h0 & 1) + l - 1) >> 1;
#pragma unroll
            for (int i = 0; i < NIT; ++i) chg[i] = q == i ? fmaxf(chg[i], chgl[slot(l)]) : chg[i];
        }
        __shared__ float red[NIT][NWR + 1];
#pragma unroll
        for (int i = 0; i < NIT; ++i)  // the iterations this pass touched (workgroup-uniform)
            if ((a.h0 >> 1) + i <= (a.h0 + K - 1) >> 1)
                block_reduce_max_store(chg[i], a.maxc + (a.h0 >> 1) + i, red[i]);
    }
}

// Output rows per tile of the tall-tile shape for K levels.
namespace {
struct TbrShape {
    int K, nwr, rpw;
    bool autopick;  // candidate for rows == 0
    int rows() const { return nwr * rpw + 2 - 2 * K; }
};
// K = 4: (4, 11, 2) -- 16 output rows, one round of 256 workgroups at 1024^2 --
// with the phi rows by LDS-DMA and the rhs by register prefetch, 161 VGPRs:
// 2.87 ms per pass at 1024^3 (r02), against 3.07 for (4, 10, 2) (292 tiles, a
// partial second round) and 4.0-4.2 for (4, 7, 3) (two waves per SIMD).
// K = 2 shapes serve the red-black GS passes (one iteration per pass); r01 at
// 1024^3: 20 rows 2.48 ms, 18 rows 2.51 ms, 28 rows 2.60 ms per iteration.
// (2, 9, 2): 16-row GS tiles, 256 workgroups at 1024^2 -- one full round;
// (2, 10, 2): 18-row, 228 workgroups, for the 240 CUs of a partitioned slab.
// K = 3 shapes also serve the red-black GS (three half-sweeps, 1.5 iterations,
// per pass: the r02 default); K = 1 only its rollback of one half-sweep.
constexpr TbrShape kShapes[] = {{3, 11, 2, true}, {3, 10, 2, true}, {3, 7, 3, false},
                                {4, 7, 3, false}, {4, 11, 2, true}, {4, 10, 2, false}, {2, 11, 2, true},
                                {2, 10, 2, true}, {2, 10, 3, false}, {2, 9, 2, true}, {1, 9, 2, true}};

int num_cus() {
    static int n = 0;
    if (n <= 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}
thread_local int g_cu_reserve = 0;
thread_local int g_last_shape[4] = {0, 0, 0, 0};  // K, row waves, rows per wave, z-chunk
}  // namespace

int tbr_cus() { return num_cus() - g_cu_reserve; }
void set_cu_reserve(int n) { g_cu_reserve = n; }

// rows = output rows per tile (0: pick the shape and z-chunk by a cost model).
// One workgroup fills a CU (LDS / VGPRs), so workgroups run in rounds of
// #CUs.  Model: rounds x (steps per workgroup + ~8 steps of pipeline fill) x
// rows loaded per step (a saturated chip gives each CU an equal byte rate).
// Calibrated on 1024^3, K = 3: 16-row tiles in one round of 256 workgroups
// (2.48 ms per pass) beat 18-row tiles in 9 rounds of 103 planes (2.62 ms)
// and in 5 rounds of 205 planes (2.79 ms); the model orders them the same.
// Pick the shape and z-chunk (see above) and launch.
// first: 0, or the kFirst* flags of a Jacobi first pass (K = 2..4 auto shapes).
template <int MODE>
static int tbr_launch(TbrArgs a, int K, int rows, int zchunk, bool pre, hipStream_t s, int first = 0) {
    const int pd = jacobi3d_tb_prefetch();
    if (first && (MODE != kJacobi || pre || pd != 1 || rows != 0 || K < 2)) {
        set_error("jacobi3d_tbr: a first pass needs Jacobi, raw div, prefetch 1, auto tiles, 2..4 levels");
        return CFD_E_INVALID;
    }
    if (a.nx % 4 != 0) {  // float4 rows; the levels' edge rule assumes it (level4)
        set_error("jacobi3d_tbr: nx must be a multiple of 4");
        return CFD_E_INVALID;
    }
    const int L = a.ze - a.zb;
    const int nseg = ceil_div(a.nx, 256);
    const int ncu = tbr_cus();
    const TbrShape *best = nullptr;
    int best_zlen = 0;
    double best_cost = 0.0;
    for (const TbrShape &sh : kShapes) {
        if (sh.K != K || (rows ? sh.rows() != rows : !sh.autopick)) continue;
        const int W = sh.rows(), NR = W + 2 * K;
        const long tiles = (long)nseg * ceil_div(a.ny - 2, W);
        for (int nzc = 1; nzc <= 64; ++nzc) {
            int zlen = zchunk > 0 ? zchunk : ceil_div(L, nzc);
            if (zlen > L) zlen = L;
            if (zchunk <= 0 && zlen < 8 && L >= 8) break;
            const long wgs = tiles * ceil_div(L, zlen);
            const double cost = (double)ceil_div(wgs, ncu) * (zlen + 2 * K - 2 + 8) * NR;
            if (!best || cost < best_cost) {
                best = &sh;
                best_cost = cost;
                best_zlen = zlen;
            }
            if (zchunk > 0) break;
        }
    }
    if (!best) {
        set_error("jacobi3d_tbr: no tile shape with %d rows for %d levels per pass", rows, K);
        return CFD_E_INVALID;
    }
    a.nseg = nseg;
    a.ntile_y = ceil_div(a.ny - 2, best->rows());
    a.trace = reinterpret_cast<unsigned long long *>(tuning().tbr_trace);
    a.zchunk = best_zlen;
    // CFD_TBR_XBW = w (A/B knob): each XCD takes a block of w x-segments x
    // (its share / w) tile rows instead of whole tile rows, which changes how
    // many halo rows / columns two XCDs both fetch; only for one z-chunk and
    // block counts that tile the plane exactly
    {
        static const int xbw_env = [] {
            const char *e = getenv("CFD_TBR_XBW");
            return e ? atoi(e) : 0;
        }();
        const int tiles = nseg * a.ntile_y, per = tiles / kNumXcd;
        a.xbw = 0;
        if (xbw_env > 0 && best_zlen >= L && tiles % kNumXcd == 0 && nseg % xbw_env == 0 && per % xbw_env == 0 &&
            (kNumXcd / (nseg / xbw_env)) * (per / xbw_env) == a.ntile_y && kNumXcd % (nseg / xbw_env) == 0)
            a.xbw = xbw_env;
    }
    g_last_shape[0] = best->K;
    g_last_shape[1] = best->nwr;
    g_last_shape[2] = best->rpw;
    g_last_shape[3] = best_zlen;
    const int blocks = a.nseg * a.ntile_y * ceil_div(L, best_zlen);
    // short Jacobi chunks whose step count (zlen + 2K - 2) is no multiple of
    // 6: shifting queues (SHIFTQ) run exactly their steps; the rotated ones
    // save ~2 % per step but would run up to 5 extra (the slab boundary
    // launches: 3 planes = 7 steps, 12 rotated)
    const int nsteps = best_zlen + 2 * best->K - 2;
    static const bool shiftq_all = [] {  // CFD_TBR_SHIFTQ=1 (A/B knob): shifting queues everywhere
        const char *e = getenv("CFD_TBR_SHIFTQ");
        return e && atoi(e) == 1;
    }();
    const bool shiftq = MODE == kJacobi && pd == 1 && best->K == 3 &&
                        (shiftq_all || (nsteps % 6 != 0 && nsteps < 216));
#define CFD_TBR_L(KV, NW, RP, PR, PDV) \
    hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, PR, PDV, MODE>), dim3(blocks), dim3((NW + 1) * 64), 0, s, a)
#define CFD_TBR(KV, NW, RP)                                                                   \
    do {                                                                                      \
        if constexpr (MODE == kRbgs) {                                                        \
            if (pd == 2) CFD_TBR_L(KV, NW, RP, false, 2); else CFD_TBR_L(KV, NW, RP, false, 1); \
        } else if (pd == 2) {                                                                 \
            if (pre) CFD_TBR_L(KV, NW, RP, true, 2); else CFD_TBR_L(KV, NW, RP, false, 2);      \
        } else {                                                                              \
            if (pre) CFD_TBR_L(KV, NW, RP, true, 1); else CFD_TBR_L(KV, NW, RP, false, 1);      \
        }                                                                                     \
    } while (0)
    // shapes with a first-pass variant (all on the LDS-DMA path); K = 3 ones
    // also with shifting queues
#define CFD_TBRF(KV, NW, RP)                                                                 \
    do {                                                                                     \
        if constexpr (MODE == kJacobi && KV == 3) {                                          \
            if (shiftq) {                                                                    \
                if (first == (kFirstRhs | kFirstZero))                                       \
                    hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, false, 1, MODE, kFirstRhs | kFirstZero, true>), \
                                       dim3(blocks), dim3((NW + 1) * 64), 0, s, a);          \
                else if (first == kFirstRhs)                                                 \
                    hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, false, 1, MODE, kFirstRhs, true>), \
                                       dim3(blocks), dim3((NW + 1) * 64), 0, s, a);          \
                else if (pre)                                                                \
                    hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, true, 1, MODE, 0, true>),   \
                                       dim3(blocks), dim3((NW + 1) * 64), 0, s, a);          \
                else                                                                         \
                    hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, false, 1, MODE, 0, true>),  \
                                       dim3(blocks), dim3((NW + 1) * 64), 0, s, a);          \
                break;                                                                       \
            }                                                                                \
        }                                                                                    \
        if constexpr (MODE == kJacobi) {                                                     \
            if (first == (kFirstRhs | kFirstZero)) {                                         \
                hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, false, 1, MODE, kFirstRhs | kFirstZero>), \
                                   dim3(blocks), dim3((NW + 1) * 64), 0, s, a);              \
                break;                                                                       \
            }                                                                                \
            if (first == kFirstRhs) {                                                        \
                hipLaunchKernelGGL((jacobi3d_tbr<KV, NW, RP, false, 1, MODE, kFirstRhs>),     \
                                   dim3(blocks), dim3((NW + 1) * 64), 0, s, a);              \
                break;                                                                       \
            }                                                                                \
        }                                                                                    \
        CFD_TBR(KV, NW, RP);                                                                 \
    } while (0)
    const int code = best->K * 100 + best->nwr * 10 + best->rpw;
    // only the CFD_TBRF shapes below have first-pass instantiations; a first
    // pass on any other shape would silently run as a plain pass (rhs_out
    // never written, phi read from `out`)
    if (first && code != 3 * 100 + 11 * 10 + 2 && code != 3 * 100 + 10 * 10 + 2 &&
        code != 4 * 100 + 11 * 10 + 2 && code != 2 * 100 + 11 * 10 + 2 && code != 2 * 100 + 10 * 10 + 2 &&
        code != 2 * 100 + 9 * 10 + 2) {
        set_error("jacobi3d_tbr: tile shape (%d levels, %d x %d rows) has no first-pass variant", best->K,
                  best->nwr, best->rpw);
        return CFD_E_INVALID;
    }
    switch (code) {
        case 3 * 100 + 11 * 10 + 2: CFD_TBRF(3, 11, 2); break;
        case 3 * 100 + 10 * 10 + 2: CFD_TBRF(3, 10, 2); break;
        case 1 * 100 + 9 * 10 + 2: if constexpr (MODE == kRbgs) CFD_TBR(1, 9, 2); break;
        case 3 * 100 + 7 * 10 + 3: if constexpr (MODE == kJacobi) CFD_TBR(3, 7, 3); break;
        case 4 * 100 + 7 * 10 + 3: CFD_TBR(4, 7, 3); break;
        case 4 * 100 + 11 * 10 + 2: CFD_TBRF(4, 11, 2); break;
        case 4 * 100 + 10 * 10 + 2: CFD_TBR(4, 10, 2); break;
        case 2 * 100 + 11 * 10 + 2: CFD_TBRF(2, 11, 2); break;
        case 2 * 100 + 10 * 10 + 2: CFD_TBRF(2, 10, 2); break;
        case 2 * 100 + 9 * 10 + 2: CFD_TBRF(2, 9, 2); break;
        default: CFD_TBR(2, 10, 3); break;
    }
#undef CFD_TBRF
#undef CFD_TBR
#undef CFD_TBR_L
    CFD_LAUNCH_CHECK();
    return CFD_OK;
}

int jacobi3d_tbr_pass(int K, int rows, const float *in, float *out, const float *div, int nz,
                      int ny, int nx, int zb, int ze, int fixed_lo, int fixed_hi, float h2,
                      float dt, int zchunk, bool pre, hipStream_t s) {
    if (ze <= zb || ny < 3) return CFD_OK;
    TbrArgs a{};
    a.in = in; a.out = out; a.div = div;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze;
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi; a.h2 = h2; a.dt = dt;
    return tbr_launch<kJacobi>(a, K, rows, zchunk, pre, s);
}

// The first pass of a solve (K = 2..4): raw div in, f32(h*h)*div/dt of the
// owned cells out to rhs_out for the later passes; zero != 0: level 0 is
// phi = 0 and `out` is the only array of phi touched (any of the pair).
int jacobi3d_tbr_first_pass(int K, float *out, const float *div, float *rhs_out, const float *in,
                            int nz, int ny, int nx, int zb, int ze, int fixed_lo, int fixed_hi,
                            float h2, float dt, int zchunk, bool zero, hipStream_t s) {
    if (ze <= zb || ny < 3) return CFD_OK;
    TbrArgs a{};
    a.in = zero ? out : in; a.out = out; a.div = div; a.rhs_out = rhs_out;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze;
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi; a.h2 = h2; a.dt = dt;
    return tbr_launch<kJacobi>(a, K, 0, zchunk, false, s, kFirstRhs | (zero ? kFirstZero : 0));
}

// Red-black GS passes on tall tiles: `levels` half-sweeps (1..4) from half-sweep
// h0 on (iteration h0 / 2, colour h0 & 1), planes [zb, ze) of `out` from `in`.
// A pass is skipped on the device when an iteration the previous pass
// completed met the tolerance (maxc of iterations h0/2 - 1 and h0/2 - 2, or
// `lag` earlier); each level's max|change| of owned cells goes to
// ws->maxc[its iteration] (a pass that ends inside an iteration leaves the
// rest to the next).  rollback = P != 0: the conditional re-run after a stop
// inside a pass of a solve of P half-sweeps per pass and nhalf in all (in =
// phi, out = phi_tmp as passed to the solve; the kernel reads the count in
// ws->flags[1], see rbgs_count, and picks h0 and the direction itself).
int rbgs3d_tbr_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                    int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int h0,
                    int levels, RbgsWs *ws, int rollback, int nhalf, int rows, hipStream_t s,
                    int lag) {
    if (ze <= zb || ny < 3) return CFD_OK;
    TbrArgs a{};
    a.in = in; a.out = out; a.div = div;
    a.nz = nz; a.ny = ny; a.nx = nx; a.zb = zb; a.ze = ze;
    a.fixed_lo = fixed_lo; a.fixed_hi = fixed_hi;
    a.cx = k.cx; a.cy = k.cy; a.cz = k.cz; a.cd = k.cd; a.dt_inv = k.dt_inv; a.tol = k.tol;
    a.zoff = zoff; a.h0 = h0;
    a.maxc = rollback ? nullptr : ws->maxc;
    a.rollback = rollback;
    a.nhalf = nhalf;
    a.count = &ws->flags[1];
    a.lag = lag;
    return tbr_launch<kRbgs>(a, levels, rows, jacobi3d_tb_zchunk(), false, s);
}

}  // namespace cfd

extern "C" int cfd_get_last_tbr_shape(int *levels, int *row_waves, int *rows_per_wave, int *zchunk) {
    CFD_REQUIRE(levels && row_waves && rows_per_wave && zchunk, "get_last_tbr_shape: null pointer");
    *levels = cfd::g_last_shape[0];
    *row_waves = cfd::g_last_shape[1];
    *rows_per_wave = cfd::g_last_shape[2];
    *zchunk = cfd::g_last_shape[3];
    return CFD_OK;
}
