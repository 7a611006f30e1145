// jacobi2d_persist.hip -- the small-grid 2-D Jacobi solve (v5.py:336-346, the
// NumPy branch of solve_pressure_fast on the 600 x 180 cylinder: 1500 sweeps,
// masked cells forced to 0 after each) as ONE persistent launch.
//
// The launch-per-pass path (jacobi2d_small, poisson2d.hip) pays ~4 us of
// kernel boundary and load latency per 4 sweeps at 600 x 180.  Here, as in
// rbgs2d_persist.hip (whose hand-off this is), the tiles stay resident for
// the whole solve: a workgroup is one 32-row x 64-column tile (16 waves x 2
// rows, one cell per lane) that advances NI sweeps per block, the
// intermediate levels eroding into an NI-row / NI-lane halo, and owns its
// inner (32 - 2 NI) x (64 - 2 NI) cells (NI: the most of 10, 8, 6, 4 whose
// tiles all fit on the chip; 210 tiles of 10 sweeps at 600 x 180).  Own cells stay in registers from
// block to block; after a block the tile publishes them as 8-byte {value,
// tag} granules (sc1 stores, tag = solve epoch << 16 | block + 1) into a ring of granule planes,
// and before the next block it polls its halo cells (owned by its 8
// neighbour tiles) until their tags match.  A pair of levels is one LDS
// exchange of the waves' rows (double-buffered: one barrier per pair, below);
// x-neighbours by DPP.
// There is no stop rule in this branch of the reference (a fixed count).
//
// Arithmetic: jac5's order, ((E + W) + N + S - rhs) * 0.25 with rhs =
// f32(dx^2) * div / dt formed as k_rhs2d forms it, two rows per wave as one
// packed pair (v_pk_add / v_pk_mul: the same IEEE operation per element); a
// masked cell becomes 0 at every sweep (v5.py:345), rows 0 and ny - 1 and
// columns 0 and nx - 1 keep their values.  Bit-identical to the single
// sweep, sweep for sweep.
//
// Ring ordering (kJGSlots planes): a tile publishes block k over block
// k - kJGSlots's granules after it consumed all its neighbours' block k - 1
// output, which each published after reading its own block k - 1 input
// (block k - 2 granules): nobody reads a granule plane older than k - 2 then.
// The result: every tile writes its own cells into phi after its last block;
// a neighbour read phi only at its start, which preceded its block 0 output
// that this tile consumed (hence nb >= 2 blocks, iterations > NI).  Every poll
// is bounded (20 s of the 100 MHz clock by default, cfd_set_persistent_launch);
// an expired one leaves phi all NaN and counts a failure (cfd_persistent_status):
// the last workgroup to finish (a ticket counter) checks and resets the status,
// so a solve is this one launch with no prologue or epilogue kernel.
// The launch (launch_persistent) is a plain one after the occupancy check by
// default (every tile fits on an otherwise idle chip), ordered after this
// process's previous persistent launch on the device; cfd_set_persistent_launch
// (1, ...) makes it cooperative, where the runtime guarantees that every tile
// is resident at once or refuses and the launch-per-pass path runs.
#include "internal.hpp"

#include <atomic>

namespace cfd {
namespace {

constexpr int kJT0 = 32;  // tile rows (32 / RW waves of RW rows)
constexpr int kJGSlots = 3;
constexpr int kJMaxTiles = 256;
constexpr int kMaxDevices = 64;

struct JPersistArgs {
    float *phi;         // in: the initial guess; out: the own cells of the result
    const float *src;   // div, or the precomputed rhs (pre)
    const uint8_t *mask;
    unsigned long long *G;  // kJGSlots planes of ny * nx granules
    int *status;            // [0]: bit 0 a poll expired; [1]: workgroups finished (both 0 between solves)
    int *fail;              // the device's persistent-failure counter (cfd_persistent_status)
    unsigned epoch;         // this solve's tag prefix: granule tags are epoch << 16 | block + 1
    unsigned long long spin;  // poll bound, 100 MHz ticks
    unsigned long long *trace;  // optional (cfd_set_small2d_gs_trace): 4 timestamps per tile and block
    int ny, nx, nseg, niters, pre;
    int zero;  // start from phi = 0 (v5.py:337): read nothing of phi, write the edge rows' zeros too
    float dx2, dtv;
};

__device__ inline unsigned long long jgload(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load sc1
}
__device__ inline void jgstore(unsigned long long *p, float v, unsigned tag) {
    __hip_atomic_store(p, ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store sc1
}
__device__ inline void lds_barrier_j() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// PAIRS (r06): the levels in pairs with ONE LDS exchange per pair: each wave
// reads rows i0 - 2, i0 - 1, i0 + RW, i0 + RW + 1 of level l - 1, computes
// level l on its RW rows and one halo row on either side (redundantly with the
// neighbouring waves) and level l + 1 on its own rows from registers, so a
// pair costs one barrier and one LDS round trip instead of two.  600 x 180,
// 10 sweeps per block (scripts/j2_trace.py): levels 2.64 -> 1.72 us per
// block, the solve 0.684 -> 0.557 ms.  RW = 4 (8 waves) computes 1.25 row
// sweeps per own row and level against 1.5 and its levels are faster
// (1.6 us), but its halo waits grow more (1.44 against 0.96 us): RW = 2 is
// the one instantiated.  Every row's update is the single sweep's, in its
// order: the same bits.
template <bool MASK, int NI, bool PAIRS, int RW>
__global__ __launch_bounds__(1024) void jacobi2d_persist(JPersistArgs a) {
    static_assert(RW == 2 || RW == 4, "rows per wave");
    constexpr int HL = NI, SOUT = 64 - 2 * HL, OUT = kJT0 - 2 * NI;
    static_assert(OUT >= 2, "too many sweeps per block for the tile");
    // two buffers of the tile's rows; tile row i at S[.][i + 2], two zero
    // rows above and below (the reads of rows -2 .. kJT0 + 1 need no test)
    __shared__ float S[2][kJT0 + 4][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = xcd_swizzle(blockIdx.x, gridDim.x);
    const int seg = bid % a.nseg, ty = bid / a.nseg;
    const int ytop = 1 + ty * OUT - NI;  // global row of tile row 0
    const int x = seg * SOUT - HL + lane;
    const bool valid = x >= 0 && x < a.nx;
    const bool writer = lane >= HL && lane < 64 - HL && valid;
    const unsigned long long t0 = wall_clock64();
    bool broken = false;
    if (w == 0) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            S[b][0][lane] = S[b][1][lane] = 0.f;
            S[b][kJT0 + 2][lane] = S[b][kJT0 + 3][lane] = 0.f;
        }
    }

    typedef float f2 __attribute__((ext_vector_type(2)));
    const int i0 = RW * w;
    float A[RW];
    f2 rh[RW / 2];
    bool upd[RW], zero[RW], own[RW], inner[RW], edgez[RW];
    size_t off[RW];
#pragma unroll
    for (int j = 0; j < RW; ++j) {
        const int i = i0 + j, y = ytop + i;
        const bool in_ = valid && y >= 0 && y <= a.ny - 1;
        off[j] = (size_t)min(max(y, 0), a.ny - 1) * a.nx + (valid ? x : 0);
        const float v = a.zero ? 0.f : a.phi[off[j]], d = a.src[off[j]];
        const bool mk = MASK ? a.mask[off[j]] != 0 : false;
        A[j] = in_ ? v : 0.f;
        const float dd = in_ ? d : 0.f;
        rh[j / 2][j % 2] = a.pre ? dd : (a.dx2 * dd) / a.dtv;
        upd[j] = in_ && y >= 1 && y <= a.ny - 2 && x >= 1 && x <= a.nx - 2;
        zero[j] = in_ && mk;  // v5.py:345: after the interior, masked cells <- 0
        own[j] = writer && i >= NI && i < kJT0 - NI && y <= a.ny - 2;
        inner[j] = in_ && y >= 1 && y <= a.ny - 2;  // the cells some tile owns
        // a masked cell of row 0 or ny - 1 (no tile owns it) becomes 0 too,
        // and with a zero start every cell of those rows
        edgez[j] = writer && in_ && !inner[j] && (mk || a.zero);
    }
    const size_t plane = (size_t)a.ny * a.nx;
    // PAIRS: the halo rows i0 - 1 (.x) and i0 + RW (.y): their rhs and update rules
    f2 rhH = {0.f, 0.f};
    bool updH[2] = {false, false}, zeroH[2] = {false, false};
    if constexpr (PAIRS) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int i = q ? i0 + RW : i0 - 1, y = ytop + i;
            const bool in_ = valid && i >= 0 && i < kJT0 && y >= 0 && y <= a.ny - 1;
            const size_t o = (size_t)min(max(y, 0), a.ny - 1) * a.nx + (valid ? x : 0);
            const float d = in_ ? a.src[o] : 0.f;
            const bool mk = MASK && in_ ? a.mask[o] != 0 : false;
            rhH[q] = a.pre ? d : (a.dx2 * d) / a.dtv;
            updH[q] = in_ && y >= 1 && y <= a.ny - 2 && x >= 1 && x <= a.nx - 2;
            zeroH[q] = in_ && mk;
        }
    }

    // block k's halo cells (block k - 1's granules)
    auto fetch = [&](int k) {
        const unsigned long long *Gk = a.G + (size_t)((k - 1) % kJGSlots) * plane;
        bool need[RW];
#pragma unroll
        for (int j = 0; j < RW; ++j) need[j] = inner[j] && !own[j];
        while (true) {
            unsigned long long g[RW];
#pragma unroll
            for (int j = 0; j < RW; ++j) g[j] = need[j] ? jgload(Gk + off[j]) : 0ull;
            bool more = false;
#pragma unroll
            for (int j = 0; j < RW; ++j) {
                if (need[j] && (unsigned)(g[j] >> 32) == (a.epoch << 16 | (unsigned)k)) {
                    A[j] = __uint_as_float((unsigned)g[j]);
                    need[j] = false;
                }
                more = more || need[j];
            }
            broken = broken || (unsigned long long)(wall_clock64() - t0) > a.spin;
            if (!__any(more) || broken) break;
            __builtin_amdgcn_s_sleep(1);
        }
    };

    // sweeps 1..m of one block: level l keeps the tile rows [l, 32 - l)
    // (s - rh) * 0.25 on two rows as two packed ops: left to itself the
    // compiler splits both into scalar pairs (v_pk_mul_f32 takes no literal,
    // and the selects that follow are per row); the same IEEE operations
    f2 quarter = {0.25f, 0.25f};
    __asm__ volatile("" : "+v"(quarter));
    auto pk_quarter_diff = [&](f2 s2v, f2 rr) {
        f2 d, r;
        __asm__("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(s2v), "v"(rr));
        __asm__("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(d), "v"(quarter));
        return r;
    };
    // one sweep of two rows x0, x1 with north (n0, n1) and south (s0, s1)
    // neighbours: ((E + W) + N + S - rhs) * 0.25, E and W by DPP
    auto sweep2 = [&](float x0, float x1, float n0, float n1, float s0, float s1, f2 rr) {
        f2 t = f2{dpp_from_upper(x0), dpp_from_upper(x1)} + f2{dpp_from_lower(x0), dpp_from_lower(x1)};
        t = t + f2{n0, n1};
        t = t + f2{s0, s1};
        return pk_quarter_diff(t, rr);
    };
    // after the first sweep every masked cell of the tile holds 0 (each wave
    // has a live row at sweep 1, halo cells arrive zeroed from their owners,
    // cells no tile owns keep their sweep-1 zero), so later sweeps need one
    // select: upd && !zero ? new : old
    bool updnz[RW], updnzH[2];
#pragma unroll
    for (int j = 0; j < RW; ++j) updnz[j] = upd[j] && !zero[j];
#pragma unroll
    for (int q = 0; q < 2; ++q) updnzH[q] = updH[q] && !zeroH[q];
    // the new own rows from nv (first: the block-uniform first sweep's select and zeroing)
    auto select_own = [&](const f2 (&nv)[RW / 2], bool first) {
#pragma unroll
        for (int j = 0; j < RW; ++j) {
            if (first) {
                float b = upd[j] ? nv[j / 2][j % 2] : A[j];
                if (zero[j]) b = 0.f;
                A[j] = b;
            } else {
                A[j] = (MASK ? updnz[j] : upd[j]) ? nv[j / 2][j % 2] : A[j];
            }
        }
    };
    // one level of the own rows, the rows below / above them being dn / up
    auto level_own = [&](float dn, float up, bool first) {
        f2 nv[RW / 2];
#pragma unroll
        for (int p = 0; p < RW / 2; ++p) {
            const int j = 2 * p;
            nv[p] = sweep2(A[j], A[j + 1], A[j + 1], j + 2 < RW ? A[j + 2] : up, j > 0 ? A[j - 1] : dn, A[j], rh[p]);
        }
        select_own(nv, first);
    };
    // one pair of levels (l, l + 1) from buffer rb into buffer wb (PAIRS)
    auto pair = [&](int l, int k, int rb, int wb) {
        const bool first = MASK && k == 0 && l == 1;
        // (a wave whose rows are dead at level l + 1 needs neither level, except
        // for the first sweep's zeroing: an edge row (no tile owns it, it is
        // never fetched) keeps its zeroed masked cells from block 0 on)
        if (!first && !(i0 + RW - 1 >= l + 1 && i0 < kJT0 - (l + 1))) return;
        const float sm2 = S[rb][i0][lane], sm1 = S[rb][i0 + 1][lane];
        const float spa = S[rb][i0 + RW + 2][lane], spb = S[rb][i0 + RW + 3][lane];
        // level l: the halo rows (row i0 - 1: N A[0], S sm2; row i0 + RW: N spb, S A[RW - 1]) ...
        const f2 nh = sweep2(sm1, spa, A[0], spb, sm2, A[RW - 1], rhH);
        float H0, H1;
        if (first) {
            H0 = updH[0] ? nh.x : sm1;
            if (zeroH[0]) H0 = 0.f;
            H1 = updH[1] ? nh.y : spa;
            if (zeroH[1]) H1 = 0.f;
        } else {
            H0 = (MASK ? updnzH[0] : updH[0]) ? nh.x : sm1;
            H1 = (MASK ? updnzH[1] : updH[1]) ? nh.y : spa;
        }
        // ... and the own rows; level l + 1 on the own rows, all operands in registers
        level_own(sm1, spa, first);
        level_own(H0, H1, false);
#pragma unroll
        for (int j = 0; j < RW; ++j) S[wb][i0 + 2 + j][lane] = A[j];
    };
    auto levels = [&](int m, int k) {
#pragma unroll
        for (int j = 0; j < RW; ++j) S[0][i0 + 2 + j][lane] = A[j];
        lds_barrier_j();
        if constexpr (PAIRS) {
            // pairs from buffer 0; an odd m ends with one single level below
#pragma unroll
            for (int l = 1; l + 1 <= NI; l += 2) {
                if (l + 1 > m) break;
                const int rb = ((l - 1) >> 1) & 1;
                pair(l, k, rb, rb ^ 1);
                if (l + 1 < m) lds_barrier_j();
            }
            if ((m & 1) == 0) return;
        }
#pragma unroll
        for (int l = 1; l <= NI; ++l) {
            if (PAIRS && l < m) continue;  // (PAIRS: only the odd last level)
            if (l > m) break;
            // (PAIRS: the (l - 1) / 2 pairs before it left level l - 1 in buffer ((l - 1) / 2) & 1)
            const int rb = PAIRS ? ((l - 1) >> 1) & 1 : (l - 1) & 1, wb = rb ^ 1;
            if (i0 + RW - 1 >= l && i0 < kJT0 - l) {
                level_own(S[rb][i0 + 1][lane], S[rb][i0 + RW + 2][lane], MASK && k == 0 && l == 1);
#pragma unroll
                for (int j = 0; j < RW; ++j) S[wb][i0 + 2 + j][lane] = A[j];
            }
            if (l < m) lds_barrier_j();
        }
    };

    const int nb = (a.niters + NI - 1) / NI;
    const int ntl = gridDim.x;
    // diagnostics: wave 0's timestamps (100 MHz) per block k, and in row nb
    // the kernel's entry, loop start, loop end and exit
    auto mark_at = [&](int k, int e, unsigned long long t) {
        if (a.trace && w == 0 && lane == 0) a.trace[((size_t)k * ntl + bid) * 4 + e] = t;
    };
    auto mark = [&](int k, int e) { mark_at(k, e, wall_clock64()); };
    mark_at(nb, 0, t0);
    mark(nb, 1);
    for (int k = 0; k < nb; ++k) {
        const int m = min(NI, a.niters - k * NI);
        mark(k, 0);
        if (k > 0) fetch(k);
        mark(k, 1);
        levels(m, k);
        mark(k, 2);
        if (k + 1 < nb) {
#pragma unroll
            for (int j = 0; j < RW; ++j)
                if (own[j])
                    jgstore(a.G + (size_t)(k % kJGSlots) * plane + off[j], A[j], a.epoch << 16 | (unsigned)(k + 1));
        }
        mark(k, 3);
        lds_barrier_j();  // the next block's LDS writes follow every wave's last reads
    }
#pragma unroll
    for (int j = 0; j < RW; ++j) {
        if (own[j]) a.phi[off[j]] = A[j];
        if (edgez[j]) a.phi[off[j]] = 0.f;
    }
    mark(nb, 2);
    // The last workgroup to finish reads the status: an expired poll left
    // garbage, so the whole result becomes NaN (it cannot pass for a solution:
    // the health check, v5.py:601, sees it) and the device's failure counter
    // counts the solve.  It then zeroes both words for the ring's next solve.
    __shared__ int last;
    // every thread's phi stores at agent scope before the workgroup's ticket:
    // each wave waits for its own stores (vmcnt counts stores on CDNA), then
    // ONE agent fence per workgroup (its L2 write-back covers the CU's waves)
    // after the barrier.  A fence in every thread, each an L2 write-back, cost
    // the launch up to 55 us at 600 x 180 (r06 trace, scripts/j2_trace.py).
    wait_vmcnt<0>();
    const int any_broken = __syncthreads_or(broken ? 1 : 0);
    if (threadIdx.x == 0) {
        __threadfence();
        if (any_broken) atomicOr(a.status, 1);
        __threadfence();  // the status before the ticket
        last = atomicAdd(a.status + 1, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    mark(nb, 3);
    if (!last) return;
    __threadfence();
    if (__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        for (size_t c = threadIdx.x; c < plane; c += blockDim.x) a.phi[c] = __int_as_float(0x7fc00000);
        if (threadIdx.x == 0 && a.fail) atomicAdd(a.fail, 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.status, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.status + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int jtiles_for(int NI, int ny, int nx, int *nseg) {
    const int OUT = kJT0 - 2 * NI, SOUT = 64 - 2 * NI;
    *nseg = ceil_div(nx, SOUT);
    return *nseg * ceil_div(ny - 2, OUT);
}

// workgroups of jacobi2d_persist<MASK, NI, PAIRS, RW> the current device holds
// at once (an idle device; -1: query failed), cached per device
template <bool MASK, int NI, bool PAIRS, int RW>
int jresident_tiles() {
    static std::atomic<int> cache[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return -1;
    int r = cache[dev].load(std::memory_order_relaxed);
    if (r == 0) {
        int per_cu = 0, cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, jacobi2d_persist<MASK, NI, PAIRS, RW>,
                                                         64 * (kJT0 / RW), 0) != hipSuccess)
            return -1;
        r = per_cu * cus;
        cache[dev].store(r, std::memory_order_relaxed);
    }
    return r;
}

// The granule ring and the status word live in a library-owned device buffer,
// one per host thread and device (the Jacobi entry points take no exchange
// workspace: 24 B per cell, 2.6 MB at 600 x 180), grown on demand and kept
// for the life of the process (a destructor at thread exit could run after
// the HIP runtime's teardown; a thread that exits leaves its ring).  Solves that
// share a ring are ordered: a solve on another stream than the ring's last
// user first waits for that solve (an event), so two streams of one thread
// never run on the same granules at once.
struct JRing {
    void *p[kMaxDevices] = {};
    size_t bytes[kMaxDevices] = {};
    unsigned epoch[kMaxDevices] = {};  // the last solve's tag prefix (0: reset the ring first)
    hipEvent_t done[kMaxDevices] = {};
    hipStream_t last[kMaxDevices] = {};
};
thread_local JRing t_ring;

// the ring for device dev, at least `bytes`, ordered after its last user
void *ring_acquire(int dev, size_t bytes, hipStream_t s, int *rc) {
    JRing &r = t_ring;
    if (r.bytes[dev] < bytes) {
        if (r.p[dev]) {
            // the old ring may still be in use by queued work
            if (r.done[dev]) (void)hipEventSynchronize(r.done[dev]);
            (void)hipFree(r.p[dev]);
        }
        r.p[dev] = nullptr;
        r.bytes[dev] = 0;
        r.epoch[dev] = 0;
        if (hipMalloc(&r.p[dev], bytes) != hipSuccess) {
            *rc = CFD_E_HIP;
            set_error("jacobi2d persistent: ring allocation of %zu bytes failed", bytes);
            return nullptr;
        }
        r.bytes[dev] = bytes;
    }
    if (!r.done[dev] && hipEventCreateWithFlags(&r.done[dev], hipEventDisableTiming) != hipSuccess) {
        *rc = CFD_E_HIP;
        set_error("jacobi2d persistent: event creation failed");
        return nullptr;
    }
    if (r.last[dev] != s && hipStreamWaitEvent(s, r.done[dev], 0) != hipSuccess) {
        *rc = CFD_E_HIP;
        set_error("jacobi2d persistent: stream ordering failed");
        return nullptr;
    }
    return r.p[dev];
}
unsigned &t_ring_epoch(int dev) { return t_ring.epoch[dev]; }
void ring_release(int dev, hipStream_t s) {
    JRing &r = t_ring;
    if (hipEventRecord(r.done[dev], s) == hipSuccess) r.last[dev] = s;
}

}  // namespace

void release_thread_rings() {
    JRing &r = t_ring;
    for (int d = 0; d < kMaxDevices; ++d) {
        if (r.done[d]) (void)hipEventSynchronize(r.done[d]);
        if (r.p[d]) (void)hipFree(r.p[d]);
        if (r.done[d]) (void)hipEventDestroy(r.done[d]);
        r.p[d] = nullptr;
        r.bytes[d] = 0;
        r.epoch[d] = 0;
        r.done[d] = nullptr;
        r.last[d] = nullptr;
    }
}

int jacobi2d_persist_solve(float *phi, const float *src, bool pre, const uint8_t *mask, int ny, int nx,
                           float dx2, float dtv, int iterations, hipStream_t s, int *rc, bool zero) {
    *rc = CFD_OK;
    if (!tuning().j2_persist || ny < 3 || nx < 3) return 0;
    const bool pairs = tuning().j2p_pairs;
    JPersistArgs a;
    a.phi = phi;
    a.src = src;
    a.mask = mask;
    a.ny = ny;
    a.nx = nx;
    a.niters = iterations;
    a.pre = pre ? 1 : 0;
    a.zero = zero ? 1 : 0;
    a.dx2 = dx2;
    a.dtv = dtv;
    // the most sweeps per block (at most j2p_ni) whose tiles all fit on the
    // chip at once: more sweeps per block are fewer hand-offs, but smaller
    // tile outputs (32 - 2 NI rows), so more tiles
#define CFD_JN(F)                   \
    switch (NI) {                   \
        case 10: F(10, RW_); break; \
        case 8: F(8, RW_); break;   \
        case 6: F(6, RW_); break;   \
        default: F(4, RW_); break;  \
    }
#define CFD_RES(N_, R_)                                                                                         \
    resident = pairs ? (mask ? jresident_tiles<true, N_, true, R_>() : jresident_tiles<false, N_, true, R_>()) \
                     : (mask ? jresident_tiles<true, N_, false, R_>() : jresident_tiles<false, N_, false, R_>())
    constexpr int RW_ = 2;  // rows per wave (RW = 4, 8 waves: 0.674 against 0.625 ms per v5 step, r06)
    int NI = 0, ntiles = 0;
    for (const int cand : {10, 8, 6, 4}) {
        if (cand > tuning().j2p_ni || iterations <= cand) continue;
        if ((iterations + cand - 1) / cand >= 0xffff) continue;  // block numbers are 16-bit tag fields
        NI = cand;
        int resident = 0;
        CFD_JN(CFD_RES)
        if (resident < 0) {
            *rc = CFD_E_HIP;
            set_error("jacobi2d persistent: occupancy query failed");
            return 1;
        }
        ntiles = jtiles_for(NI, ny, nx, &a.nseg);
        if (ntiles <= resident && ntiles <= kJMaxTiles) break;
        NI = 0;
    }
#undef CFD_RES
    if (NI == 0) return 0;  // the launch-per-pass path
    const size_t plane = (size_t)ny * nx;
    const size_t gbytes = sizeof(unsigned long long) * kJGSlots * plane;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        *rc = CFD_E_HIP;
        set_error("jacobi2d persistent: no device");
        return 1;
    }
    char *p = static_cast<char *>(ring_acquire(dev, gbytes + 256, s, rc));
    if (!p) return 1;
    // the status words first, at a place no grid size moves: behind the
    // granules they sat where a larger grid's solve had left granules, so a
    // smaller grid after a larger one on the same ring read garbage there
    // (its last workgroup never found itself last; an expired poll then went
    // unreported, r06)
    a.status = reinterpret_cast<int *>(p);
    a.G = reinterpret_cast<unsigned long long *>(p + 256);
    // Granule tags carry a per-ring solve epoch, so a granule left by an earlier
    // solve never matches a poll of this one.  The ring is zeroed only when it
    // is new or the 16-bit epoch wraps (a plane a run of short solves leaves
    // alone could otherwise hold a same-tag granule 65536 solves old).
    unsigned &ep = t_ring_epoch(dev);
    if (ep == 0 || ep == 0xffffu) {
        if (hipMemsetAsync(p, 0, gbytes + 256, s) != hipSuccess) {
            *rc = CFD_E_HIP;
            set_error("jacobi2d persistent: ring reset failed");
            return 1;
        }
        ep = 0;
    }
    a.epoch = ++ep;
    a.fail = persist_fail_word(s);
    {
        const size_t need = 32 * (size_t)ntiles * (size_t)((iterations + NI - 1) / NI + 1);
        a.trace = tuning().gs_trace_bytes >= need ? reinterpret_cast<unsigned long long *>(tuning().gs_trace) : nullptr;
    }
    a.spin = persist_poll_ticks();
    const void *f = nullptr;
#define CFD_KF(N_, R_)                                                                                       \
    f = pairs ? (mask ? (const void *)jacobi2d_persist<true, N_, true, R_>                                    \
                      : (const void *)jacobi2d_persist<false, N_, true, R_>)                                  \
              : (mask ? (const void *)jacobi2d_persist<true, N_, false, R_>                                   \
                      : (const void *)jacobi2d_persist<false, N_, false, R_>)
    CFD_JN(CFD_KF)
#undef CFD_KF
#undef CFD_JN
    const int lr = launch_persistent(f, ntiles, 64 * (kJT0 / RW_), &a, s);
    if (lr == 0) return 0;  // not co-resident now: the launch-per-pass path
    if (lr < 0) {
        *rc = CFD_E_HIP;
        return 1;
    }
    ring_release(dev, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        *rc = CFD_E_HIP;
        set_error("jacobi2d persistent launch failed: %s", hipGetErrorString(e));
    }
    return 1;
}

}  // namespace cfd
