// rbgs2d_persist.hip -- the small-grid 2-D red-black Gauss-Seidel solve
// (v5.py:202-226, the v5 cylinder's 600 x 180 pressure solve) as ONE
// persistent launch.
//
// Why: at 600 x 180 a GS launch is latency, not bytes.  The launch-per-block
// path (rbgs2d_wg, poisson2d.hip) pays per launch ~4.2 us of fixed cost (the
// kernel boundary, the tile's load latency, the stores and slot atomics) for
// 4 iterations; here the tiles stay resident for the whole solve and the
// kernel boundary between two blocks of iterations becomes a neighbour
// hand-off of 8-byte {value, tag} granules (~1 us, MI355X_MICROARCH.md,
// handoff-1to1), which needs no flag, fence or barrier: a granule is valid when
// its tag is the block that wrote it.
//
// Geometry and arithmetic are rbgs2d_wg's, so the two paths are bit-identical
// block for block: a workgroup is one 32-row x 64-column tile (16 waves x 2
// rows, one cell per lane) that advances NI iterations (L = 2 NI colour
// levels) per block, the intermediate levels eroding into an L-row / L-lane
// halo, and owns its inner (32 - 2L) x (64 - 2L) cells.  Own cells stay in
// registers from block to block; after a block the tile publishes them to a
// ring of granule planes (slot = block mod 3, tag = block + 1), and before the
// next block it polls its halo cells (all owned by its 8 neighbour tiles) in
// the previous block's slot.  Rows 0 and ny-1 and cells outside the grid never
// change, so they keep the values loaded at the start.
//
// Stop rule (v5.py:224-225): the solve stops after the first iteration whose
// max|change| < tol, i.e. the first iteration in which no cell changed by >=
// tol (a NaN change never raises the reference's max).  So a tile publishes,
// per block, one granule of flags (bit q: did any own cell change by >= tol in
// iteration q; ring of 8 blocks; block k's go out at block k + 1's start).  At the end
// of block k, after block k is published, wave 0 folds every tile's flags of
// block k - 3 by ballots (their loads were issued at the block's second level,
// so their latency hides behind the levels; two blocks of slack cover the
// tiles' skew, ~0.5 block); the first flag-free iteration n stops the solve:
// every tile then re-runs block B = n / NI from its input (block B - 1's slot,
// which no tile has overwritten: nobody publishes block k without having ruled
// out a stop in block k - 4, and the ring holds 5 blocks) for the n - B NI + 1
// iterations it needs.  The last three blocks are checked after the loop.  With tol <= 0 nothing is
// published or polled for the stop rule (it can never fire).
//
// Ordering of the granule ring (5 slots): a tile publishes block k (before
// its stop decision at the end of block k) over block k - 5's granules only
// after it has consumed its neighbours' block k - 1 output, which they
// published after reading their block k - 2 input, later than the last read
// of block k - 5's granules (their block k - 4 input, or the rollback of a
// stop in block k - 4, ruled out at the end of block k - 1).  The flag
// ring (8 blocks): block j's flags go out at block j + 1, after this tile
// ruled out a stop in block j - 2, so every tile has published block j - 2's
// flags, i.e. is in block j - 1 or later and reads flags of block j - 4 or
// later.  The launch (launch_persistent) is a plain one after the
// occupancy check by default, ordered after this process's previous persistent
// launch on the device; cfd_set_persistent_launch(1, ...) makes it cooperative
// (the runtime guarantees that every tile is resident at once, or refuses it
// and the launch-per-block path runs).  Every poll is still bounded (20 s of the 100
// MHz clock from the kernel's start by default, cfd_set_persistent_launch):
// an expired one ends the solve with phi all NaN, *iters_done = -1 and a
// failure counted for cfd_persistent_status, instead of a hang.
#include "internal.hpp"

#include <atomic>

namespace cfd {
namespace {

constexpr int kPW = 16, kPRW = 2, kPT0 = kPW * kPRW;  // waves, rows per wave, tile rows
#ifndef CFD_GS_LAG
#define CFD_GS_LAG 3
#endif
constexpr int kPLag = CFD_GS_LAG;                      // the stop test looks kPLag blocks back
constexpr int kPGSlots = kPLag + 2;                    // granule planes (block outputs)
constexpr int kPMSlots = 8;                            // per-block flag ring (>= kPLag + 2)
static_assert(kPMSlots >= kPLag + 2, "flag ring too short for the lag");
constexpr int kPMaxTiles = 256;                        // one tile per CU at most
constexpr int kPMaxNI = 5;

struct PersistArgs {
    const float *in;
    float *out;
    const float *div;
    const uint8_t *mask;
    unsigned long long *G;  // kPGSlots planes of ny * nx granules
    unsigned long long *M;  // kPMSlots x ntiles flag granules
    RbgsWs *ws;
    int *bad;  // a poll expired (a ring word, zeroed with the rings per solve)
    unsigned long long *trace;  // optional: 4 timestamps per tile and block
    unsigned long long spin;    // poll bound, 100 MHz ticks
    int ny, nx, nseg, ntiles, niters;
    float cx, cy, cd, dt_inv, tol;
};

__device__ inline unsigned long long gload(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load sc1
}
__device__ inline void gstore(unsigned long long *p, float v, unsigned tag) {
    __hip_atomic_store(p, ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store sc1
}
__device__ inline unsigned gtag(unsigned long long g) { return (unsigned)(g >> 32); }
__device__ inline float gval(unsigned long long g) { return __uint_as_float((unsigned)g); }
// LDS writes done, then the workgroup barrier; global loads stay in flight
// (the compiler's __syncthreads would wait for them too)
__device__ inline void lds_barrier_p() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool MASK, int NI, bool PAIRS>
__global__ __launch_bounds__(1024) void rbgs2d_persist(PersistArgs a) {
    constexpr int L = 2 * NI, HL = L, SOUT = 64 - 2 * HL, OUT = kPT0 - 2 * L;
    constexpr int MT = kPMaxTiles / 64;  // maxima granules per lane and iteration (wave 0)
    static_assert(OUT >= 2, "too many levels for the tile");
    // two buffers of the tile's rows; tile row i at S[.][i + 2], two zero
    // rows above and below (the halo-row reads need no test: each test was a
    // branch on a spilled lane mask, ~12 of an iteration's ~67 VALU, r06)
    __shared__ float S[2][kPT0 + 4][64];
    __shared__ int busy[NI];  // some own cell changed by >= tol in iteration q of the block
    __shared__ int sh_stop;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = bid % a.nseg, ty = bid / a.nseg;
    const int ytop = 1 + ty * OUT - L;  // global row of tile row 0
    const int x = seg * SOUT - HL + lane;
    const bool valid = x >= 0 && x < a.nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    const bool check = a.tol > 0.f;
    const unsigned long long t0 = wall_clock64();
    bool broken = false;  // a poll expired (per wave; the result is garbage then)
    auto expired = [&]() {
        broken = broken || (unsigned long long)(wall_clock64() - t0) > a.spin;
        return broken;
    };

    if (w == 0) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            S[b][0][lane] = S[b][1][lane] = 0.f;
            S[b][kPT0 + 2][lane] = S[b][kPT0 + 3][lane] = 0.f;
        }
    }

    float A[kPRW], RH[kPRW];
    bool U0[kPRW], U1[kPRW], own[kPRW], inner[kPRW];
    size_t off[kPRW];
#pragma unroll
    for (int j = 0; j < kPRW; ++j) {
        const int i = kPRW * w + j, y = ytop + i;
        const bool in_ = valid && y >= 0 && y <= a.ny - 1;
        off[j] = (size_t)min(max(y, 0), a.ny - 1) * a.nx + (valid ? x : 0);
        const float v = a.in ? a.in[off[j]] : 0.f;
        const float d = a.div[off[j]];
        const bool mk = MASK ? a.mask[off[j]] != 0 : false;
        const bool edge = y <= 0 || y >= a.ny - 1;
        A[j] = in_ ? v : 0.f;
        RH[j] = -(in_ ? d : 0.f) * a.dt_inv;
        const bool ok = in_ && !edge && x >= 1 && x < a.nx - 1 && !mk;
        const bool even = ((y + x + 1) & 1) == 0;
        U0[j] = ok && even;
        U1[j] = ok && !even;
        own[j] = writer && i >= L && i < kPT0 - L && y <= a.ny - 2;
        inner[j] = in_ && !edge;  // cells some tile owns (all others never change)
    }
    // PAIRS: the rhs and colour masks of the rows just outside the wave's two
    // (tile rows 2w - 1 and 2w + 2), which the pair schedule updates too
    float RHh[2] = {0.f, 0.f};
    bool U0h[2] = {false, false};
    if (PAIRS) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = kPRW * w + (h ? kPRW : -1), y = ytop + i;
            const bool in_ = valid && y >= 0 && y <= a.ny - 1 && i >= 0 && i < kPT0;
            const size_t o = (size_t)min(max(y, 0), a.ny - 1) * a.nx + (valid ? x : 0);
            const float d = a.div[o];
            const bool mk = MASK ? a.mask[o] != 0 : false;
            const bool edge = y <= 0 || y >= a.ny - 1;
            RHh[h] = -(in_ ? d : 0.f) * a.dt_inv;
            const bool ok = in_ && !edge && x >= 1 && x < a.nx - 1 && !mk;
            U0h[h] = ok && ((y + x + 1) & 1) == 0;  // these rows are updated only at colour-0 levels
        }
    }
    const size_t plane = (size_t)a.ny * a.nx;

    // cells of block k's input (block k-1's granules): the halo cells, or all
    // inner cells of the tile (a rollback, whose registers hold a later block)
    auto fetch = [&](int k, bool all) {
        const unsigned long long *Gk = a.G + (size_t)((k - 1) % kPGSlots) * plane;
        const unsigned want = (unsigned)k;
        bool need[kPRW];
#pragma unroll
        for (int j = 0; j < kPRW; ++j) need[j] = inner[j] && (all || !own[j]);
        while (true) {
            unsigned long long g[kPRW];
#pragma unroll
            for (int j = 0; j < kPRW; ++j) g[j] = need[j] ? gload(Gk + off[j]) : 0ull;
            bool more = false;
#pragma unroll
            for (int j = 0; j < kPRW; ++j) {
                if (need[j] && gtag(g[j]) == want) {
                    A[j] = gval(g[j]);
                    need[j] = false;
                }
                more = more || need[j];
            }
            if (!__any(more) || expired()) break;
            __builtin_amdgcn_s_sleep(1);
        }
    };

    // wave 0: the tile's flags of block kb as one granule (bit q: some own
    // cell changed by >= tol in iteration q of the block), then cleared
    auto publish_flags = [&](int kb) {
        if (lane == 0) {
            unsigned bits = 0;
#pragma unroll
            for (int q = 0; q < NI; ++q) bits |= busy[q] ? 1u << q : 0u;
            __hip_atomic_store(a.M + (size_t)(kb % kPMSlots) * a.ntiles + bid,
                               ((unsigned long long)(kb + 1) << 32) | bits, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane < NI) busy[lane] = 0;
    };
    // wave 0: every tile's flag granule of block kb (issued early, folded late)
    unsigned long long mg[MT];
    auto issue_maxima = [&](int kb) {
        const unsigned long long *Mk = a.M + (size_t)(kb % kPMSlots) * a.ntiles;
#pragma unroll
        for (int r = 0; r < MT; ++r) {
            const int t = lane + 64 * r;
            mg[r] = t < a.ntiles ? gload(Mk + t) : 0ull;
        }
    };
    // first iteration of block kb (m iterations) in which no tile was hot, else -1
    auto fold_maxima = [&](int kb, int m) {
        const unsigned long long *Mk = a.M + (size_t)(kb % kPMSlots) * a.ntiles;
        const unsigned want = (unsigned)(kb + 1);
        while (true) {
            bool late[MT], more = false;
#pragma unroll
            for (int r = 0; r < MT; ++r) {
                late[r] = lane + 64 * r < a.ntiles && gtag(mg[r]) != want;
                more = more || late[r];
            }
            if (!__any(more) || expired()) break;
            __builtin_amdgcn_s_sleep(1);
            // re-issue every late granule before waiting for any of them
#pragma unroll
            for (int r = 0; r < MT; ++r)
                if (late[r]) mg[r] = gload(Mk + lane + 64 * r);
        }
        unsigned bits = 0;
#pragma unroll
        for (int r = 0; r < MT; ++r) bits |= (unsigned)mg[r];
        int hit = -1;
#pragma unroll
        for (int q = NI - 1; q >= 0; --q)
            if (q < m && !__any((bits >> q) & 1u)) hit = q;
        return hit < 0 ? -1 : kb * NI + hit;
    };

    // colour levels 1..2m of one block (m = iterations, block-uniform).  The
    // wave's two rows go through the arithmetic as one packed pair (v_pk_*
    // f32: the same IEEE operations in the same order per element).  A wave
    // whose rows are both outside level l's live rows [l, 32 - l) skips the
    // level (nothing reads them at level l + 1).  Own-row waves note per
    // iteration whether an own cell changed by >= tol (hot).  Outside a
    // rollback (k >= 0): wave 0, whose rows die after level 1, publishes the
    // tile's flags of block k - 1 at the second level and folds every tile's
    // flags of block k - 3 after the last level (the stop decision, in sh_stop
    // after the block's last barrier).
    const int nb = (a.niters + NI - 1) / NI;
    bool hot[NI];  // per lane: an own cell changed by >= tol (a NaN change never counts, as in v5.py:221)
    const bool own_rows = kPRW * w + 1 >= L && kPRW * w < kPT0 - L;  // wave-uniform
    // the PAIRS levels' stop-test condition as a scalar int: as a bool it
    // stayed a 64-bit lane mask, spilled to VGPR lanes (two v_readlane per
    // use, twice per iteration)
    const int chk_own = __builtin_amdgcn_readfirstlane(check && own_rows ? 1 : 0);
    // PAIRS: the colour masks as VGPR bit masks (v_bfi_b32 selects) and the
    // stop threshold as a per-lane VGPR (tol on a lane of own cells, NaN
    // elsewhere: no compare is true).  As 64-bit lane masks they outgrew the
    // SGPRs, and every select read its mask back with two v_readlane.
    auto vmask = [](bool b) {
        uint32_t m = b ? ~0u : 0u;
        __asm__ volatile("" : "+v"(m));
        return m;
    };
    const uint32_t mU0h0 = vmask(U0h[0]), mU00 = vmask(U0[0]), mU01 = vmask(U0[1]), mU0h1 = vmask(U0h[1]);
    const uint32_t mU10 = vmask(U1[0]), mU11 = vmask(U1[1]);
    float tolv = own[0] ? a.tol : __int_as_float(0x7fc00000);
    __asm__ volatile("" : "+v"(tolv));
    auto bsel = [](uint32_t m, float t, float f) {  // (t & m) | (f & ~m), one v_bfi_b32
        float r;
        __asm__("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(t), "v"(f));
        return r;
    };
    auto levels = [&](int m, int k) {
#pragma unroll
        for (int q = 0; q < NI; ++q) hot[q] = false;
#pragma unroll
        for (int j = 0; j < kPRW; ++j) S[0][kPRW * w + 2 + j][lane] = A[j];
        lds_barrier_p();
        if (a.trace && k >= 0 && w == 0 && lane == 0) a.trace[((size_t)k * a.ntiles + bid) * 4 + 2] = wall_clock64();
        typedef float f2 __attribute__((ext_vector_type(2)));
        const int i0 = kPRW * w;
        const f2 rh = {RH[0], RH[1]};
        if (PAIRS) {
            // one LDS exchange per iteration: each wave reads two rows on
            // either side, computes the colour-0 level on its rows and the
            // two around them, then the colour-1 level on its own rows
            const f2 rhl = {RHh[0], RH[0]}, rhu = {RH[1], RHh[1]};
#pragma unroll
            for (int p = 1; p <= NI; ++p) {
                if (p > m) break;
                const int l = 2 * p - 1;
                const int rb = (p - 1) & 1, wb = p & 1;
                if (p == 1 && check && k >= 1 && w == 0) {
                    publish_flags(k - 1);
                    if (k >= kPLag) issue_maxima(k - kPLag);
                }
                // wave-uniform: an own row live at l + 1 (a scalar int, as chk_own)
                if (__builtin_amdgcn_readfirstlane(i0 + 1 >= l + 1 && i0 < kPT0 - (l + 1) ? 1 : 0)) {
                    const float dn2 = S[rb][i0][lane], dn1 = S[rb][i0 + 1][lane];
                    const float up1 = S[rb][i0 + 4][lane], up2 = S[rb][i0 + 5][lane];
                    // level l (colour 0): rows i0-1, i0 (pair lo) and i0+1, i0+2 (pair hi)
                    const f2 cl = {dn1, A[0]}, ch2 = {A[1], up1};
                    const f2 nl = ((a.cx * (f2{dpp_from_upper(dn1), dpp_from_upper(A[0])} +
                                            f2{dpp_from_lower(dn1), dpp_from_lower(A[0])}) +
                                    a.cy * (f2{A[0], A[1]} + f2{dn2, dn1})) - rhl) * a.cd;
                    const f2 nh = ((a.cx * (f2{dpp_from_upper(A[1]), dpp_from_upper(up1)} +
                                            f2{dpp_from_lower(A[1]), dpp_from_lower(up1)}) +
                                    a.cy * (f2{up1, up2} + f2{A[0], A[1]})) - rhu) * a.cd;
                    // no per-row liveness test: a row outside level l's live
                    // rows [l, 32 - l) is read at level l + 1 only by rows
                    // outside [l + 1, 31 - l), so updating it changes no live
                    // cell (and the masks stay loop-invariant)
                    const float q0 = bsel(mU0h0, nl[0], cl[0]), q1 = bsel(mU00, nl[1], cl[1]);
                    const float q2 = bsel(mU01, nh[0], ch2[0]), q3 = bsel(mU0h1, nh[1], ch2[1]);
                    // the stop test's largest change of the wave's own-row cells
                    // in this iteration: the change of the SELECTED values, 0
                    // for a cell the colour leaves alone; fmaxf drops a NaN
                    // change (it never counts, v5.py:221)
                    float dmax = 0.f;
                    if (chk_own) {
                        const f2 d0 = f2{q1, q2} - f2{cl[1], ch2[0]};
                        dmax = fmaxf(fmaxf(fabsf(d0[0]), fabsf(d0[1])), dmax);
                    }
                    // level l + 1 (colour 1): rows i0, i0 + 1 from q0..q3
                    const f2 c2 = {q1, q2};
                    const f2 nv = ((a.cx * (f2{dpp_from_upper(q1), dpp_from_upper(q2)} +
                                            f2{dpp_from_lower(q1), dpp_from_lower(q2)}) +
                                    a.cy * (f2{q2, q3} + f2{q0, q1})) - rh) * a.cd;
                    A[0] = bsel(mU10, nv[0], c2[0]);
                    A[1] = bsel(mU11, nv[1], c2[1]);
                    if (chk_own) {
                        const f2 d1 = f2{A[0], A[1]} - c2;
                        dmax = fmaxf(fmaxf(fabsf(d1[0]), fabsf(d1[1])), dmax);
                        // own[0] covers own[1] wherever row i0 + 1 can change
                        // (i0 and L even: both rows own or neither; past the
                        // last interior row nothing is updated)
                        hot[p - 1] = dmax >= tolv;
                    }
                    S[wb][i0 + 2][lane] = A[0];
                    S[wb][i0 + 3][lane] = A[1];
                }
                if (p < m) lds_barrier_p();
            }
        } else {
#pragma unroll
        for (int l = 1; l <= L; ++l) {
            if (l > 2 * m) break;
            const int par = (l - 1) & 1;  // colour of this level
            const int rb = (l - 1) & 1, wb = l & 1;
            if (l == 2 && check && k >= 1 && w == 0) {
                // wave 0 (its rows died after level 1): the tile's flags of
                // block k - 1, and the loads of every tile's flags of block k - 3
                publish_flags(k - 1);
                if (k >= kPLag) issue_maxima(k - kPLag);
            }
            if (i0 + 1 >= l && i0 < kPT0 - l) {  // wave-uniform: some row live
                const float up = S[rb][i0 + 4][lane], dn = S[rb][i0 + 1][lane];
                const f2 a2 = {A[0], A[1]};
                const f2 e2 = {dpp_from_upper(A[0]), dpp_from_upper(A[1])};
                const f2 w2 = {dpp_from_lower(A[0]), dpp_from_lower(A[1])};
                const f2 n2 = {A[1], up}, s2 = {dn, A[0]};
                const f2 nv = ((a.cx * (e2 + w2) + a.cy * (n2 + s2)) - rh) * a.cd;
                const f2 d2 = nv - a2;
                float B[kPRW];
#pragma unroll
                for (int j = 0; j < kPRW; ++j) {
                    const int i = i0 + j;
                    const bool live = i >= l && i < kPT0 - l;
                    const bool upd = live && (par ? U1[j] : U0[j]);
                    B[j] = upd ? nv[j] : A[j];
                    if (check && own_rows) hot[(l - 1) / 2] = hot[(l - 1) / 2] || (own[j] && upd && fabsf(d2[j]) >= a.tol);
                }
#pragma unroll
                for (int j = 0; j < kPRW; ++j) {
                    A[j] = B[j];
                    S[wb][i0 + 2 + j][lane] = B[j];
                }
            }
            if (l < 2 * m) lds_barrier_p();
        }
        }
        // block k's output goes out before the stop decision, so the fold
        // and the barrier do not delay the neighbours' next block.  It takes
        // the slot of block k - kPLag - 2: a stop in block k - kPLag - 1 or
        // earlier was ruled out at the end of block k - 1, and the rollback of
        // a stop in block k - kPLag (decided below) reads block k - kPLag - 1's
        // slot, hence kPLag + 2 slots
        if (k >= 0 && (k + 1 < nb || check)) {
#pragma unroll
            for (int j = 0; j < kPRW; ++j)
                if (own[j]) gstore(a.G + (size_t)(k % kPGSlots) * plane + off[j], A[j], (unsigned)(k + 1));
        }
        // the last level's barrier, behind the stop decision
        if (check && k >= kPLag && w == 0) {
            const int n = fold_maxima(k - kPLag, NI);
            if (lane == 0) sh_stop = n;
        }
        lds_barrier_p();
        if (a.trace && k >= 0 && w == 0 && lane == 0) a.trace[((size_t)k * a.ntiles + bid) * 4 + 3] = wall_clock64();
    };

    // diagnostics: in trace row nb, the kernel's entry, loop start, loop end and exit
    auto mark_end = [&](int e, unsigned long long t) {
        if (a.trace && w == 0 && lane == 0) a.trace[((size_t)nb * a.ntiles + bid) * 4 + e] = t;
    };
    mark_end(0, t0);
    mark_end(1, wall_clock64());
    int stop = -1;  // first iteration meeting the tolerance (workgroup-uniform)
    if (w == 0) sh_stop = -1;
    if (w == 0 && lane < NI) busy[lane] = 0;
    for (int k = 0; k < nb; ++k) {
        const int m = min(NI, a.niters - k * NI);
        if (a.trace && w == 0 && lane == 0) a.trace[((size_t)k * a.ntiles + bid) * 4] = wall_clock64();
        if (k > 0) fetch(k, false);
        if (a.trace && w == 0 && lane == 0) a.trace[((size_t)k * a.ntiles + bid) * 4 + 1] = wall_clock64();
        levels(m, k);
        if (check) {
            stop = sh_stop;
            if (stop >= 0) break;
            if (own_rows) {
#pragma unroll
                for (int q = 0; q < NI; ++q)
                    if (__any(hot[q]) && lane == 0) busy[q] = 1;
            }
        }
    }
    mark_end(2, wall_clock64());
    if (check && stop < 0) {
        // the last block's maxima, then the blocks no in-loop check covered
        lds_barrier_p();
        if (w == 0) publish_flags(nb - 1);
        for (int kb = max(0, nb - kPLag); kb < nb && stop < 0; ++kb) {
            if (w == 0) {
                issue_maxima(kb);
                const int n = fold_maxima(kb, min(NI, a.niters - kb * NI));
                if (lane == 0) sh_stop = n;
            }
            lds_barrier_p();
            stop = sh_stop;
            lds_barrier_p();  // every wave has read sh_stop before wave 0 may rewrite it
        }
    }
    if (stop >= 0) {
        // re-run block B from its input for the iterations up to the stop
        const int B = stop / NI, need = stop - B * NI + 1;
        if (B == 0) {
#pragma unroll
            for (int j = 0; j < kPRW; ++j)
                if (inner[j]) A[j] = a.in ? a.in[off[j]] : 0.f;
        } else {
            fetch(B, true);
        }
        levels(need, -1);
    }
#pragma unroll
    for (int j = 0; j < kPRW; ++j)
        if (own[j]) a.out[off[j]] = A[j];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ws->flags[1] = stop >= 0 ? stop + 1 : a.niters;
    if (broken) atomicOr(a.bad, 1);
    mark_end(3, wall_clock64());
}

// phi's rows 1 .. ny - 2 <- out's (the solve's result; rows 0 and ny - 1 never
// change, so phi keeps its own and out needs none), and the count; after an
// expired poll phi becomes all NaN instead (it cannot pass for a solution),
// the count -1, and the device's failure counter (cfd_persistent_status)
// counts the solve.  nx % 4 == 0 (the float4 path's condition).
__global__ void rbgs_persist_finish(const RbgsWs *__restrict__ ws, const int *__restrict__ badp, float *__restrict__ phi,
                                    const float *__restrict__ src, int ny, int nx, int zero, int *iters_done,
                                    int *fail) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const bool bad = *badp != 0;
    const float4 nan4 = make_float4(__int_as_float(0x7fc00000), __int_as_float(0x7fc00000),
                                    __int_as_float(0x7fc00000), __int_as_float(0x7fc00000));
    if (bad) {
        const size_t n4 = (size_t)ny * nx / 4;
        for (size_t k = t0; k < n4; k += stride) reinterpret_cast<float4 *>(phi)[k] = nan4;
    } else {
        const size_t b4 = (size_t)nx / 4, e4 = (size_t)(ny - 1) * nx / 4;
        for (size_t k = b4 + t0; k < e4; k += stride)
            reinterpret_cast<float4 *>(phi)[k] = reinterpret_cast<const float4 *>(src)[k];
        if (zero) {  // a zero start: rows 0 and ny - 1 are zeros too
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            for (size_t k = t0; k < b4; k += stride) {
                reinterpret_cast<float4 *>(phi)[k] = z4;
                reinterpret_cast<float4 *>(phi)[e4 + k] = z4;
            }
        }
    }
    if (t0 == 0 && iters_done) *iters_done = bad ? -1 : ws->flags[1];
    if (t0 == 0 && bad && fail) atomicAdd(fail, 1);
}

int tiles_for(int NI, int ny, int nx, int *nseg) {
    const int L = 2 * NI, OUT = kPT0 - 2 * L, SOUT = 64 - 2 * L;
    *nseg = ceil_div(nx, SOUT);
    return *nseg * ceil_div(ny - 2, OUT);
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// workgroups of rbgs2d_persist<MASK, NI, PAIRS> the chip holds at once (-1: query failed)
// (an idle device's count, cached per device)
template <bool MASK, int NI, bool PAIRS>
int resident_tiles() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    int r = cache[dev].load(std::memory_order_relaxed);
    if (r == 0) {
        int per_cu = 0, cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rbgs2d_persist<MASK, NI, PAIRS>, 1024, 0) != hipSuccess)
            return -1;
        r = per_cu * cus;
        cache[dev].store(r, std::memory_order_relaxed);
    }
    return r;
}

}  // namespace

size_t rbgs2d_persist_extra_bytes(int ny, int nx) {
    int nseg;
    const int nt = tiles_for(kPMaxNI, ny, nx, &nseg);  // the most tiles of any NI
    return align256(sizeof(unsigned long long) * kPGSlots * (size_t)ny * nx) +
           sizeof(unsigned long long) * kPMSlots * (size_t)nt + 256;
}

int rbgs2d_persist_solve(float *phi, const float *div, const uint8_t *mask, int ny, int nx, float cx,
                         float cy, float cd, float dt_inv, float tol, float *phi_tmp, RbgsWs *ws,
                         size_t ws_bytes, int iterations, int *iters_done, hipStream_t s, int *rc, bool zero) {
    *rc = CFD_OK;
    if (!tuning().gs_persist || !tuning().gs_wg || !phi_tmp || iterations < 1 || ny < 3 || nx < 3) return 0;
    const size_t base = align256(rbgs_base_bytes(iterations));
    if (ws_bytes < base + rbgs2d_persist_extra_bytes(ny, nx)) return 0;
    PersistArgs a;
    a.in = zero ? nullptr : phi;  // null: a zero start (v5.py:337), nothing of phi read (a field
                                  // of its own cost the loop SGPR spills: 57 -> 65 VALU per iteration)
    a.out = phi_tmp;
    a.div = div;
    a.mask = mask;
    a.ws = ws;
    a.ny = ny;
    a.nx = nx;
    a.niters = iterations;
    // every tile must be resident at once (they wait on each other): the most
    // iterations per block, at most gs_ni, whose tiles all fit on the chip
    // (5 at 600 x 180: 210 tiles; the block's fixed cost, the hand-off, is
    // spread over 5 iterations instead of 4)
    const bool pairs = tuning().gs_pairs != 0;
#define CFD_PERS_N(F)                                         \
    switch (NI) {                                             \
        case 5: F(5); break;                                  \
        case 4: F(4); break;                                  \
        case 3: F(3); break;                                  \
        case 2: F(2); break;                                  \
        default: F(1); break;                                 \
    }
#define CFD_RES(N_)                                                                        \
    resident = pairs ? (mask ? resident_tiles<true, N_, true>() : resident_tiles<false, N_, true>()) \
                     : (mask ? resident_tiles<true, N_, false>() : resident_tiles<false, N_, false>())
    int NI = tuning().gs_ni;
    for (; NI >= 1; --NI) {
        int resident = 0;
        CFD_PERS_N(CFD_RES)
        if (resident < 0) {
            *rc = CFD_E_HIP;
            set_error("rbgs2d persistent: occupancy query failed");
            return 1;
        }
        a.ntiles = tiles_for(NI, ny, nx, &a.nseg);
        if (a.ntiles <= resident && a.ntiles <= kPMaxTiles) break;
    }
#undef CFD_RES
    if (NI < 1) return 0;  // the launch-per-block path
    {
        const size_t need = 32 * (size_t)a.ntiles * (size_t)((iterations + NI - 1) / NI + 1);
        a.trace = tuning().gs_trace_bytes >= need ? reinterpret_cast<unsigned long long *>(tuning().gs_trace) : nullptr;
    }
    a.cx = cx;
    a.cy = cy;
    a.cd = cd;
    a.dt_inv = dt_inv;
    a.tol = tol;
    char *p = reinterpret_cast<char *>(ws) + base;
    a.G = reinterpret_cast<unsigned long long *>(p);
    const size_t gbytes = align256(sizeof(unsigned long long) * kPGSlots * (size_t)ny * nx);
    a.M = reinterpret_cast<unsigned long long *>(p + gbytes);
    const size_t mbytes = sizeof(unsigned long long) * kPMSlots * (size_t)a.ntiles;
    a.bad = reinterpret_cast<int *>(p + gbytes + mbytes);  // (within the extra bytes' last 256)
    // a stale granule of an earlier solve carries a valid-looking tag: reset
    // the rings (and the failure word)
    if (hipMemsetAsync(p, 0, gbytes + mbytes + sizeof(int), s) != hipSuccess) {
        *rc = CFD_E_HIP;
        set_error("rbgs2d persistent: ring reset failed");
        return 1;
    }
    a.spin = persist_poll_ticks();
    const void *f = nullptr;
#define CFD_KF(N_)                                                                                    \
    f = pairs ? (mask ? (const void *)rbgs2d_persist<true, N_, true> : (const void *)rbgs2d_persist<false, N_, true>) \
              : (mask ? (const void *)rbgs2d_persist<true, N_, false> : (const void *)rbgs2d_persist<false, N_, false>)
    CFD_PERS_N(CFD_KF)
#undef CFD_KF
#undef CFD_PERS_N
    const int lr = launch_persistent(f, a.ntiles, 1024, &a, s);
    if (lr == 0) return 0;  // not co-resident now: the launch-per-block path (the rings are re-reset there)
    if (lr < 0) {
        *rc = CFD_E_HIP;
        return 1;
    }
    const size_t n = (size_t)ny * nx;
    hipLaunchKernelGGL(rbgs_persist_finish, dim3(ceil_div((long)(n / 4 + 1), 256)), dim3(256), 0, s, ws, a.bad, phi,
                       phi_tmp, ny, nx, zero ? 1 : 0, iters_done, persist_fail_word(s));
    const hipError_t e2 = hipGetLastError();
    if (e2 != hipSuccess) {
        *rc = CFD_E_HIP;
        set_error("rbgs2d persistent finish failed: %s", hipGetErrorString(e2));
    }
    return 1;
}

}  // namespace cfd
