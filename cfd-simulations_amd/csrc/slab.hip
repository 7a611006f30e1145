// slab.hip -- multi-GPU slab decomposition of the 3-D Jacobi sweep.
//
// One process per GPU.  The (nz, ny, nx) grid is cut on z; each rank's local
// array is (nz_local + 2G, ny, nx) with G ghost planes per side (G = 1..4).
// A pass performs up to G sweeps (the K-level blocked kernels recompute the
// inner ghost planes' intermediate levels); after every pass the G owned
// boundary planes per side go to the z-neighbours with RCCL send/recv
// (point-to-point over xGMI: one direct link per neighbour pair).
// With overlap on, the boundary planes are swept first, their exchange runs on
// a second HIP stream, and the interior planes sweep concurrently on the main
// stream; the main stream waits on the exchange before the next sweep.  The
// decomposition is exact: every cell sees the same neighbour values as in the
// single-GPU sweep, so results are bit-identical for any rank count.
//
// The exchange plan (peers, which planes are updated) is computed on the host
// (SlabPlan in the Python package) and tested there on CPU with gloo.
//
// Transport: RCCL (cfd_comm_init), or -- for tests and rehearsals on a single
// GPU, where RCCL refuses several ranks per device -- an in-process group of N
// ranks driven by N host threads (cfd_comm_init_local): the same drivers, the
// same pass / exchange / reduce sequence, with the send/recv pairs replaced by
// device copies ordered by HIP events and host barriers.
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "internal.hpp"

namespace cfd {

struct LocalGroup {
    struct Slot {
        float *buf[2] = {nullptr, nullptr};
        float *maxc = nullptr;
        int nzl = 0, G = 0;
        size_t plane = 0;
        hipEvent_t ready = nullptr, done = nullptr;
    };
    explicit LocalGroup(int n_) : n(n_), slot(n_) {}
    // all ranks meet; false if a rank did not arrive within the timeout (it
    // failed): the group is then broken and every later call fails fast
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const long gen = generation;
        if (++arrived == n) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen || broken; })) {
            broken = true;
            cv.notify_all();
            return false;
        }
        return !broken;
    }
    int n;
    std::vector<Slot> slot;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long generation = 0;
    bool broken = false;
};

// ---------------------------------------------------------------------------
// Copy-engine transport (cfd_comm_init_ipc): the halo exchange without CUs.
// Each rank maps its z-neighbours' field buffers (IPC handles of their
// allocations, exchanged once by the caller: cfd_comm_ipc_export / _import)
// and writes its boundary planes straight into their ghost planes with the
// copy engines (hipMemcpyDeviceToDeviceNoCU: SDMA, ~58 GB/s per stream on
// MI355X, measured by scripts/sdma_probe.hip), one stream per direction so the
// two directions run on two engines.  Behind each copy, on the same stream, a
// hipStreamWriteValue32 bumps a sequence word in the receiver's flag block
// (uncached device memory).  The receiver's compute stream runs a one-wave
// sync kernel (k_ce_sync) after each pass: it waits, with a bounded spin,
// until both neighbours' words reach the expected count, so the next pass's
// boundary launches, dispatched after it, read complete ghosts.  Why this
// replaces RCCL here: RCCL's send/recv kernel needs 132 VGPRs and 20 KB of
// LDS per block, which no CU has free beside the one-workgroup-per-CU tall-tile
// interior, so it needed a CU partition (16 CUs reserved, 240-CU tile plans:
// 13 % slower interiors, and the 256-workgroup 4-level GS tile in two rounds).
// The copy engines take no CU at all, so the interior keeps the single-GPU
// plan.  Ordering: counts are monotonic per direction and every rank runs the
// same exchanges, so no host handshake is needed; inside a solve a copy into
// a neighbour's buffer can only start after that neighbour's previous sync
// (its boundary launches, the only readers of ghost planes, precede the planes
// it sends, which our next pass waits for), so no ghost plane is overwritten
// while read.  Across solves nothing orders a neighbour's first copy after
// this rank's earlier work on its buffers (a zero start has no initial
// exchange; a fill of phi_tmp queued just before the solve was seen to land
// over the ghosts a fast neighbour had already sent), so each solve begins
// with a ready word per direction: written to the neighbour's flag block on
// the compute stream behind all earlier work (ce_begin), and waited for on
// the copy stream before that solve's first copy into the neighbour.
// The red-black GS stop rule needs the global max|change| of each iteration:
// the same sync kernel stores this rank's maxima into every rank's gather ring
// (8-byte {tag, value} granules, system-scope stores into the uncached flag
// blocks) and waits for every rank's granule of the pass, max-reduces them and
// writes the global value back to the workspace before the next pass's stop
// test reads it.
constexpr int kCeMaxRanks = 16;
constexpr int kCeRing = 256;             // gather slots, iterations in flight
constexpr int kCeFromLo = 0;             // u32 word: exchanges received from the lo neighbour
constexpr int kCeFromHi = 32;            // ... from the hi neighbour (own 128-B line)
constexpr int kCeReadyFromLo = 64;       // solves the lo neighbour has begun (its buffers free)
constexpr int kCeReadyFromHi = 96;       // ... the hi neighbour
constexpr int kCeGatherWord = 256;       // gather ring (u64 granules) at byte 1024
constexpr size_t kCeFlagBytes = 4 * (size_t)kCeGatherWord + 8 * (size_t)kCeRing * kCeMaxRanks;
constexpr uint32_t kCeMagic = 0x43464445u;  // "CFDE"

// Landing buffers (r06).  hipIpcOpenMemHandle of an allocation past 2 GiB
// never returns on this stack (r06 probe, scripts/ipc_size_probe.py: 2046 MiB
// maps, 2050 MiB hangs the importing process) -- the 1024^3 grid at two ranks
// holds 2.2 GB arrays.  A rank whose pair is that large (or any rank with
// CFD_CE_LANDING=1) exports instead a small landing buffer of 2 slots x 2
// sides x G planes: its neighbours' copies land there, and after the sync
// kernel its compute stream copies the slot into the ghost planes.  Slots
// alternate with the exchange count of each direction (the sender's count
// and the receiver's are equal), so the neighbours' exchange k + 2, which
// needs this rank's exchange k + 1 -- sent after this rank's landing copy k
// on the compute stream -- never overwrites a slot still being copied.
constexpr size_t kIpcMapMax = (size_t)2 << 30;  // allocations at or past this are not mapped

// What a rank exports for its peers (host bytes, cfd_comm_ipc_blob_bytes)
struct CeBlob {
    uint32_t magic, version;
    int32_t rank, nranks;
    hipIpcMemHandle_t buf_h[2];  // allocations holding phi and phi_tmp
    uint64_t buf_off[2];         // byte offset of the array in its allocation
    uint64_t buf_n[2];           // elements of each array
    hipIpcMemHandle_t flags_h;   // the flag block
    hipIpcMemHandle_t land_h;    // the landing buffer (land_n > 0)
    uint64_t land_n;             // elements per (slot, side) of the landing buffer; 0: none
};

struct CeState {
    unsigned *flags = nullptr;      // this rank's flag block (uncached)
    unsigned **peers_dev = nullptr; // every rank's flag block, as mapped here (device array)
    int *status = nullptr;          // bit 0: a sync kernel timed out
    hipStream_t xs[2] = {nullptr, nullptr};  // copy streams: to lo, to hi
    hipEvent_t xev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    struct Map {
        int rank;
        hipIpcMemHandle_t h;
        char *base;
    };
    std::vector<Map> maps;          // IPC mappings opened by this process
    std::vector<unsigned *> peer_flags;  // every rank's flag block, mapped (after the first import)
    // attached buffer pairs, in the (collective) order of their imports: a
    // solve finds its pair among them; every rank holds the same list
    struct Attachment {
        float *mine[2];
        size_t n;
        std::vector<CeBlob> blobs;  // every rank's export of this pair
        float *land = nullptr;      // this rank's landing buffer (land_n > 0)
        size_t land_n = 0;
    };
    std::vector<Attachment> att;
    int cur = -1;                   // the attachment of the solve in progress
    float *pend[2] = {nullptr, nullptr};  // exported, not yet imported
    size_t pend_n = 0;
    float *pend_land = nullptr;
    size_t pend_land_n = 0;
    std::vector<float *> lands;     // every landing buffer allocated (freed with the comm)
    // the exchange of the pass in flight (exchange_ce -> ce_sync): the array,
    // its owned planes, ghost depth and plane size
    float *x_a = nullptr;
    int x_nzl = 0, x_G = 0;
    size_t x_plane = 0;
    unsigned sent[2] = {0, 0}, recvd[2] = {0, 0}, gathered = 0;
    // solves begun per direction: every rank begins the same solves, so the
    // neighbour's ready word reaches this count when it has begun this one
    unsigned ready_sent[2] = {0, 0};
    bool need_ready[2] = {false, false};  // the solve's first copy in that direction is pending
};

struct SlabComm {
    ncclComm_t comm = nullptr;
    std::unique_ptr<CeState> ce;      // copy-engine transport instead of RCCL
    std::shared_ptr<LocalGroup> grp;  // in-process transport instead of RCCL
    int rank = 0, nranks = 1;
    hipEvent_t ev_boundary = nullptr, ev_comm = nullptr;
    // CU partition of an overlapped solve (see partition_streams): a compute
    // stream on all CUs but `reserve`, an exchange stream on those
    int part_state = 0;  // 0 not tried, 1 ready, -1 off / unavailable
    int reserve = 0;
    hipStream_t cstream = nullptr, xstream = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

// Why a CU partition: the tall-tile kernels fill a CU per workgroup (VGPRs
// and LDS), so an RCCL send/recv kernel launched beside the interior finds no
// CU with room for its blocks and runs only after the interior -- the
// exchange would be serialised, not overlapped (seen in rocprof traces of the
// self-peered rehearsal: the RCCL kernel ends right after the interior).
// The overlapped drivers therefore run their launches on a stream masked to
// all CUs but R and the exchange on a stream masked to those R: R/8 per XCD
// (workgroups are dealt round-robin to the 8 XCDs), with bit positions that
// stay spread over the XCDs whether the queue's CU-mask bits map to CUs
// XCD-major or interleaved.  The tile cost model plans for the remaining CUs
// (16-row tiles become 18-row, one round of 228 workgroups at 1024^2).
// CFD_SLAB_COMM_CUS = R (default 16, 0 = off).
}  // namespace cfd

extern "C" int cfd_slab_cu_partition(int ncu, int reserve, uint32_t *compute_mask,
                                     uint32_t *exchange_mask, int words) {
    CFD_REQUIRE(compute_mask && exchange_mask && ncu > 0 && words >= (ncu + 31) / 32,
                "slab_cu_partition: bad arguments");
    const int per = ncu / 8, R = reserve;
    // (x + 8j) % per is distinct for j < per / 8: at most per / 8 CUs per XCD
    CFD_REQUIRE(ncu % 8 == 0 && per % 8 == 0 && R > 0 && R % 8 == 0 && R <= per,
                "slab_cu_partition: need ncu %% 64 == 0 and reserve (%d) = 8k <= ncu / 8", R);
    for (int w = 0; w < words; ++w) compute_mask[w] = exchange_mask[w] = 0u;
    for (int b = 0; b < ncu; ++b) compute_mask[b / 32] |= 1u << (b % 32);
    for (int x = 0; x < 8; ++x)
        for (int j = 0; j < R / 8; ++j) {
            // R/8 CUs of XCD x under both bit orders: b / per == x and b % 8 == x
            const int b = x * per + (x + 8 * j) % per;
            exchange_mask[b / 32] |= 1u << (b % 32);
            compute_mask[b / 32] &= ~(1u << (b % 32));
        }
    return CFD_OK;
}

namespace cfd {

static int partition_streams(SlabComm *c) {
    if (c->part_state) return c->part_state;
    c->part_state = -1;
    int R = 16;
    if (const char *e = getenv("CFD_SLAB_COMM_CUS")) R = atoi(e);
    int dev = 0, ncu = 0;
    if (R <= 0 || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return c->part_state;
    if (ncu <= 0 || ncu > 1024) return c->part_state;
    std::vector<uint32_t> cm((ncu + 31) / 32, 0u), xm((ncu + 31) / 32, 0u);
    if (cfd_slab_cu_partition(ncu, R, cm.data(), xm.data(), (int)cm.size()) != CFD_OK)
        return c->part_state;
    if (hipExtStreamCreateWithCUMask(&c->cstream, (uint32_t)cm.size(), cm.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&c->xstream, (uint32_t)xm.size(), xm.data()) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        return c->part_state;
    }
    c->reserve = R;
    c->part_state = 1;
    return c->part_state;
}

// Runs a solve on the partitioned streams: forks from the caller's stream on
// entry, joins back (and clears the CU reserve) on every exit path.
struct PartitionScope {
    SlabComm *c = nullptr;
    hipStream_t caller = nullptr;
    bool on = false;
    PartitionScope(SlabComm *c_, bool want, hipStream_t &s, hipStream_t &cs) : c(c_), caller(s) {
        // not for an in-process group: its ranks share one GPU's CUs anyway,
        // and 2 masked queues per rank oversubscribe the hardware queues; not
        // for the copy-engine transport, whose exchange takes no CUs
        if (!want || c->grp || c->ce || partition_streams(c) != 1) return;
        if (hipEventRecord(c->ev_fork, s) != hipSuccess ||
            hipStreamWaitEvent(c->cstream, c->ev_fork, 0) != hipSuccess)
            return;
        on = true;
        s = c->cstream;
        cs = c->xstream;
        set_cu_reserve(c->reserve);
    }
    ~PartitionScope() {
        if (!on) return;
        set_cu_reserve(0);
        (void)hipEventRecord(c->ev_join, c->cstream);
        (void)hipStreamWaitEvent(caller, c->ev_join, 0);
    }
};

#define CFD_GROUP_BARRIER(g)                                                       \
    do {                                                                           \
        if (!(g)->barrier()) {                                                     \
            ::cfd::set_error("local slab group: a rank did not reach the barrier"); \
            return CFD_E_COMM;                                                     \
        }                                                                          \
    } while (0)

// each rank of a local group publishes its two field buffers and maxima
static int register_local(SlabComm *c, float *phi, float *phi_tmp, RbgsWs *ws, int nzl, int G,
                          size_t plane) {
    LocalGroup::Slot &me = c->grp->slot[c->rank];
    me.buf[0] = phi;
    me.buf[1] = phi_tmp;
    me.maxc = ws ? ws->maxc : nullptr;
    me.nzl = nzl;
    me.G = G;
    me.plane = plane;
    CFD_GROUP_BARRIER(c->grp);
    return CFD_OK;
}

// send/recv of G planes with each neighbour, as device copies: wait until the
// neighbour's pass has produced its planes (and stopped reading its ghosts),
// copy ours into its ghosts, and let it wait for our copies in turn
static int exchange_local(SlabComm *c, float *a, int nzl, int G, size_t plane, int lo, int hi,
                          hipStream_t s) {
    LocalGroup *g = c->grp.get();
    LocalGroup::Slot &me = g->slot[c->rank];
    const int bi = a == me.buf[0] ? 0 : a == me.buf[1] ? 1 : -1;
    CFD_REQUIRE(bi >= 0, "local slab group: exchange of an unregistered buffer");
    CFD_CHECK_HIP(hipEventRecord(me.ready, s));
    CFD_GROUP_BARRIER(g);
    const size_t n = (size_t)G * plane * sizeof(float);
    for (int peer : {lo, hi}) {
        if (peer < 0) continue;
        const LocalGroup::Slot &p = g->slot[peer];
        CFD_REQUIRE(p.G == G && p.plane == plane, "local slab group: ranks disagree on the layout");
        CFD_CHECK_HIP(hipStreamWaitEvent(s, p.ready, 0));
        const float *src = peer == lo ? a + (size_t)G * plane : a + (size_t)nzl * plane;
        float *dst = peer == lo ? p.buf[bi] + (size_t)(p.nzl + G) * plane : p.buf[bi];
        CFD_CHECK_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s));
    }
    CFD_CHECK_HIP(hipEventRecord(me.done, s));
    CFD_GROUP_BARRIER(g);
    for (int peer : {lo, hi})
        if (peer >= 0) CFD_CHECK_HIP(hipStreamWaitEvent(s, g->slot[peer].done, 0));
    return CFD_OK;
}

struct MaxcPtrs {
    const float *p[16];
};
__global__ void k_group_max(MaxcPtrs ptrs, int n, int off, int cnt, float *dst) {
    const int i = threadIdx.x;
    if (i >= cnt) return;
    float m = 0.f;
    for (int r = 0; r < n; ++r) m = fmaxf(m, ptrs.p[r][off + i]);
    dst[off + i] = m;
}

// allreduce(max) of maxc[off .. off+cnt) over the group (idempotent: a rank
// may read a peer's entry before or after the peer overwrote it with the max)
static int allreduce_local(SlabComm *c, int off, int cnt, hipStream_t s) {
    LocalGroup *g = c->grp.get();
    CFD_REQUIRE(g->n <= 16, "local slab group: at most 16 ranks");
    LocalGroup::Slot &me = g->slot[c->rank];
    CFD_CHECK_HIP(hipEventRecord(me.ready, s));
    CFD_GROUP_BARRIER(g);
    MaxcPtrs ptrs{};
    for (int r = 0; r < g->n; ++r) {
        CFD_CHECK_HIP(hipStreamWaitEvent(s, g->slot[r].ready, 0));
        ptrs.p[r] = g->slot[r].maxc;
    }
    hipLaunchKernelGGL(k_group_max, dim3(1), dim3(64), 0, s, ptrs, g->n, off, cnt, me.maxc);
    CFD_LAUNCH_CHECK();
    // no rank reuses its ready event before every rank has enqueued its waits
    CFD_GROUP_BARRIER(g);
    return CFD_OK;
}

#define CFD_CHECK_NCCL(expr)                                                              \
    do {                                                                                  \
        ncclResult_t _r = (expr);                                                         \
        if (_r != ncclSuccess) {                                                          \
            ::cfd::set_error("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r),       \
                             __FILE__, __LINE__);                                         \
            return CFD_E_COMM;                                                            \
        }                                                                                 \
    } while (0)

// Ghost exchange of array `a` (local planes 0 .. nzl+2G-1, owned G .. G+nzl-1):
// the G owned planes next to each neighbour go into that neighbour's G ghost
// planes; each direction is one contiguous message of G planes.
static int exchange(SlabComm *c, float *a, int nzl, int G, size_t plane, int lo, int hi,
                    hipStream_t s) {
    if (c->grp) return exchange_local(c, a, nzl, G, plane, lo, hi, s);
    if (lo < 0 && hi < 0) return CFD_OK;
    const size_t n = (size_t)G * plane;
    CFD_CHECK_NCCL(ncclGroupStart());
    if (lo >= 0) {
        CFD_CHECK_NCCL(ncclSend(a + (size_t)G * plane, n, ncclFloat32, lo, c->comm, s));
        CFD_CHECK_NCCL(ncclRecv(a, n, ncclFloat32, lo, c->comm, s));
    }
    if (hi >= 0) {
        CFD_CHECK_NCCL(ncclSend(a + (size_t)nzl * plane, n, ncclFloat32, hi, c->comm, s));
        CFD_CHECK_NCCL(ncclRecv(a + (size_t)(nzl + G) * plane, n, ncclFloat32, hi, c->comm, s));
    }
    CFD_CHECK_NCCL(ncclGroupEnd());
    return CFD_OK;
}

// ------------------------------------------------- copy-engine transport
static const hipMemcpyKind kCopyEngine = (hipMemcpyKind)1024;  // hipMemcpyDeviceToDeviceNoCU
// bounded spins: a peer that never signals ends the wait (status bit 0, the
// solve's result is then garbage and cfd_comm_status reports it) instead of
// hanging the GPU.  s_memrealtime ticks at 100 MHz: 20 s.
constexpr unsigned long long kCeSpinLimit = 2000000000ull;

struct CeSyncArgs {
    const unsigned *flags;           // this rank's flag block
    unsigned want_lo, want_hi;       // counts to wait for (0: no such neighbour)
    float *maxc;                     // GS maxima: publish, gather, write back
    int it0, cnt;                    // iterations it0 .. it0 + cnt - 1 (cnt 0: none)
    unsigned tag0;                   // gather tag of iteration it0
    int nranks, rank;
    unsigned *const *peers;          // every rank's flag block
    int *status;
};

__global__ __launch_bounds__(64) void k_ce_sync(CeSyncArgs a) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    bool ok = true;
    // once one wait has expired the comm is broken: later syncs return at
    // once (the solve's result is garbage either way), so a stopped peer costs
    // one timeout, not one per pass
    const bool broken = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    auto expired = [&]() { return broken || wall_clock64() - t0 > kCeSpinLimit; };
    // publish first, so that no peer waits on this rank's own waits
    for (int q = 0; q < a.cnt; ++q) {
        const unsigned tag = a.tag0 + (unsigned)q;
        const unsigned long long g =
            ((unsigned long long)__float_as_uint(a.maxc[a.it0 + q]) << 32) | (unsigned long long)tag;
        if (lane < a.nranks) {
            unsigned long long *ring = reinterpret_cast<unsigned long long *>(a.peers[lane] + kCeGatherWord);
            __hip_atomic_store(ring + (size_t)(tag % kCeRing) * kCeMaxRanks + a.rank, g, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // the neighbours' ghost planes of the pass
    if ((lane == 0 && a.want_lo) || (lane == 1 && a.want_hi)) {
        const unsigned *w = a.flags + (lane == 0 ? kCeFromLo : kCeFromHi);
        const unsigned want = lane == 0 ? a.want_lo : a.want_hi;
        while ((int)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - want) < 0) {
            if (expired()) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    // every rank's maxima of the pass -> the global max
    for (int q = 0; q < a.cnt; ++q) {
        const unsigned tag = a.tag0 + (unsigned)q;
        float m = 0.f;
        if (lane < a.nranks) {
            const unsigned long long *g = reinterpret_cast<const unsigned long long *>(a.flags + kCeGatherWord) +
                                          (size_t)(tag % kCeRing) * kCeMaxRanks + lane;
            unsigned long long v;
            while ((unsigned)(v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != tag) {
                if (expired()) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            m = __uint_as_float((unsigned)(v >> 32));
        }
        for (int off = 32; off; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        if (lane == 0) a.maxc[a.it0 + q] = m;
    }
    if (!ok) atomicOr(a.status, 1);
}

// a copy stream's wait for a neighbour's ready word (bounded, as k_ce_sync)
__global__ __launch_bounds__(64) void k_ce_wait_ready(const unsigned *w, unsigned want, int *status) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    while ((int)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - want) < 0) {
        if (wall_clock64() - t0 > kCeSpinLimit) {
            atomicOr(status, 1);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

static int ce_map(CeState &ce, int rank, const hipIpcMemHandle_t &h, char **base) {
    for (const CeState::Map &m : ce.maps)
        if (m.rank == rank && !memcmp(&m.h, &h, sizeof h)) {
            *base = m.base;
            return CFD_OK;
        }
    void *p = nullptr;
    CFD_CHECK_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    ce.maps.push_back({rank, h, static_cast<char *>(p)});
    *base = static_cast<char *>(p);
    return CFD_OK;
}

// buffer bi (0 = phi, 1 = phi_tmp as attached) of rank `peer`, as mapped here
static int ce_peer_buf(SlabComm *c, int peer, int bi, float **buf, size_t *n) {
    CeState &ce = *c->ce;
    const CeState::Attachment &at = ce.att[ce.cur];
    if (peer == c->rank) {
        *buf = at.mine[bi];
        *n = at.n;
        return CFD_OK;
    }
    const CeBlob &b = at.blobs[peer];
    char *base = nullptr;
    if (b.land_n) {  // the peer takes its ghosts through its landing buffer
        int rc = ce_map(ce, peer, b.land_h, &base);
        if (rc) return rc;
        *buf = reinterpret_cast<float *>(base);
        *n = 4 * (size_t)b.land_n;
        return CFD_OK;
    }
    int rc = ce_map(ce, peer, b.buf_h[bi], &base);
    if (rc) return rc;
    *buf = reinterpret_cast<float *>(base + b.buf_off[bi]);
    *n = b.buf_n[bi];
    return CFD_OK;
}

// the copy-engine exchange of array `a` (phi or phi_tmp as attached): the G
// owned planes next to each neighbour go into its ghost planes once `ready`
// (recorded on the compute stream after the boundary planes) has fired, then
// the neighbour's sequence word is bumped
static int exchange_ce(SlabComm *c, const float *a, int nzl, int G, size_t plane, int lo, int hi,
                       hipEvent_t ready) {
    CeState &ce = *c->ce;
    const CeState::Attachment &at = ce.att[ce.cur];
    const int bi = a == at.mine[0] ? 0 : a == at.mine[1] ? 1 : -1;
    CFD_REQUIRE(bi >= 0, "slab (copy engines): exchange of a buffer that was not attached");
    const size_t n = (size_t)G * plane;
    for (int d = 0; d < 2; ++d) {
        const int peer = d == 0 ? lo : hi;
        if (peer < 0) continue;
        float *dst = nullptr;
        size_t pn = 0;
        int rc = ce_peer_buf(c, peer, bi, &dst, &pn);
        if (rc) return rc;
        // to lo: our first owned planes -> its last (hi) ghost planes, its
        // from-hi word; to hi: our last owned planes -> its first ghost planes
        const float *src = d == 0 ? a + n : a + (size_t)nzl * plane;
        const size_t land_n = at.blobs[peer].land_n;
        if (land_n) {
            // its landing buffer: slot (this exchange's count) & 1, side hi (d
            // = 0: our planes are its hi ghosts) or lo
            CFD_REQUIRE(land_n >= n, "slab (copy engines): rank %d's landing buffer is smaller than its ghosts",
                        peer);
            const unsigned k = ce.sent[d] + 1;
            dst += ((size_t)(k & 1u) * 2 + (d == 0 ? 1 : 0)) * land_n;
        } else {
            CFD_REQUIRE(pn >= 2 * n, "slab (copy engines): rank %d's buffer is smaller than its ghosts", peer);
            if (d == 0) dst += pn - n;
        }
        unsigned *word = ce.peer_flags[peer] + (d == 0 ? kCeFromHi : kCeFromLo);
        CFD_CHECK_HIP(hipStreamWaitEvent(ce.xs[d], ready, 0));
        if (ce.need_ready[d]) {  // the neighbour has begun this solve (ce_begin)
            hipLaunchKernelGGL(k_ce_wait_ready, dim3(1), dim3(64), 0, ce.xs[d],
                               ce.flags + (d == 0 ? kCeReadyFromLo : kCeReadyFromHi), ce.ready_sent[d],
                               ce.status);
            CFD_LAUNCH_CHECK();
            ce.need_ready[d] = false;
        }
        CFD_CHECK_HIP(hipMemcpyAsync(dst, src, n * sizeof(float), kCopyEngine, ce.xs[d]));
        CFD_CHECK_HIP(hipStreamWriteValue32(ce.xs[d], word, ++ce.sent[d], 0));
        ce.used[d] = true;
    }
    ce.x_a = const_cast<float *>(a);
    ce.x_nzl = nzl;
    ce.x_G = G;
    ce.x_plane = plane;
    return CFD_OK;
}

// on stream s: wait for the ghosts of the last exchange (and, cnt > 0, make
// maxc[it0 .. it0+cnt) the global maxima)
static int ce_sync(SlabComm *c, hipStream_t s, int lo, int hi, float *maxc, int it0, int cnt) {
    CeState &ce = *c->ce;
    CeSyncArgs a{};
    a.flags = ce.flags;
    a.want_lo = lo >= 0 ? ++ce.recvd[0] : 0u;
    a.want_hi = hi >= 0 ? ++ce.recvd[1] : 0u;
    a.maxc = maxc;
    a.it0 = it0;
    a.cnt = maxc ? cnt : 0;
    a.tag0 = ce.gathered + 1;
    ce.gathered += (unsigned)a.cnt;
    a.nranks = c->nranks;
    a.rank = c->rank;
    a.peers = ce.peers_dev;
    a.status = ce.status;
    if (!a.want_lo && !a.want_hi && !a.cnt) return CFD_OK;
    hipLaunchKernelGGL(k_ce_sync, dim3(1), dim3(64), 0, s, a);
    CFD_LAUNCH_CHECK();
    const CeState::Attachment &at = ce.att[ce.cur];
    if (at.land_n && ce.x_a) {
        // the neighbours' planes landed in this rank's landing slots: into the
        // ghost planes of the exchanged array, behind the sync on s
        const size_t n = (size_t)ce.x_G * ce.x_plane;
        CFD_REQUIRE(at.land_n >= n, "slab (copy engines): landing buffer smaller than the ghosts");
        if (a.want_lo)
            CFD_CHECK_HIP(hipMemcpyAsync(ce.x_a, at.land + (size_t)(a.want_lo & 1u) * 2 * at.land_n,
                                         n * sizeof(float), hipMemcpyDeviceToDevice, s));
        if (a.want_hi)
            CFD_CHECK_HIP(hipMemcpyAsync(ce.x_a + (size_t)(ce.x_nzl + ce.x_G) * ce.x_plane,
                                         at.land + ((size_t)(a.want_hi & 1u) * 2 + 1) * at.land_n,
                                         n * sizeof(float), hipMemcpyDeviceToDevice, s));
    }
    return CFD_OK;
}

// start of a solve, after ce_check_attached: tell each neighbour, behind
// everything queued on s so far, that this rank's buffers may be written
static int ce_begin(SlabComm *c, hipStream_t s, int lo, int hi) {
    CeState &ce = *c->ce;
    for (int d = 0; d < 2; ++d) {
        const int peer = d == 0 ? lo : hi;
        if (peer < 0) continue;
        // to lo: we are its hi neighbour
        unsigned *word = ce.peer_flags[peer] + (d == 0 ? kCeReadyFromHi : kCeReadyFromLo);
        CFD_CHECK_HIP(hipStreamWriteValue32(s, word, ++ce.ready_sent[d], 0));
        ce.need_ready[d] = true;
    }
    return CFD_OK;
}

// end of a solve: the caller's stream covers this rank's outgoing copies
static int ce_join(SlabComm *c, hipStream_t s) {
    CeState &ce = *c->ce;
    for (int d = 0; d < 2; ++d) {
        if (!ce.used[d]) continue;
        CFD_CHECK_HIP(hipEventRecord(ce.xev[d], ce.xs[d]));
        CFD_CHECK_HIP(hipStreamWaitEvent(s, ce.xev[d], 0));
        ce.used[d] = false;
    }
    return CFD_OK;
}

// selects the attachment of phi / phi_tmp (either order; phi_tmp NULL: any
// pair holding phi) for the solve that follows
static int ce_check_attached(SlabComm *c, const float *phi, const float *phi_tmp) {
    CeState &ce = *c->ce;
    ce.cur = -1;
    for (int k = (int)ce.att.size() - 1; k >= 0 && ce.cur < 0; --k) {
        const CeState::Attachment &at = ce.att[k];
        if ((phi == at.mine[0] || phi == at.mine[1]) &&
            (!phi_tmp || phi_tmp == (phi == at.mine[0] ? at.mine[1] : at.mine[0])))
            ce.cur = k;
    }
    CFD_REQUIRE(ce.cur >= 0,
                "slab (copy engines): phi / phi_tmp are not a pair attached with cfd_comm_ipc_import");
    return CFD_OK;
}

}  // namespace cfd

using namespace cfd;

extern "C" {

int cfd_comm_unique_id(void *out, size_t bytes) {
    CFD_REQUIRE(out && bytes >= sizeof(ncclUniqueId), "comm_unique_id: need %zu bytes",
                sizeof(ncclUniqueId));
    ncclUniqueId id;
    CFD_CHECK_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return CFD_OK;
}

int cfd_comm_init(const void *unique_id, int nranks, int rank, void **comm) {
    CFD_REQUIRE(unique_id && comm && nranks >= 1 && rank >= 0 && rank < nranks,
                "comm_init: bad arguments");
    SlabComm *c = new SlabComm();
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        delete c;
        return CFD_E_COMM;
    }
    if (hipEventCreateWithFlags(&c->ev_boundary, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming) != hipSuccess) {
        set_error("comm_init: hipEventCreate failed");
        ncclCommDestroy(c->comm);
        delete c;
        return CFD_E_HIP;
    }
    *comm = c;
    return CFD_OK;
}

int cfd_comm_init_local(int nranks, void **comms) {
    CFD_REQUIRE(comms && nranks >= 1 && nranks <= 16, "comm_init_local: 1..16 ranks");
    auto g = std::make_shared<LocalGroup>(nranks);
    for (int r = 0; r < nranks; ++r) {
        SlabComm *c = new SlabComm();
        c->grp = g;
        c->rank = r;
        c->nranks = nranks;
        if (hipEventCreateWithFlags(&c->ev_boundary, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->slot[r].ready, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->slot[r].done, hipEventDisableTiming) != hipSuccess) {
            set_error("comm_init_local: hipEventCreate failed");
            return CFD_E_HIP;
        }
        comms[r] = c;
    }
    return CFD_OK;
}

int cfd_comm_init_ipc(int nranks, int rank, void **comm) {
    CFD_REQUIRE(comm && nranks >= 1 && nranks <= kCeMaxRanks && rank >= 0 && rank < nranks,
                "comm_init_ipc: 1..%d ranks, 0 <= rank < nranks", kCeMaxRanks);
    std::unique_ptr<SlabComm> c(new SlabComm());
    c->rank = rank;
    c->nranks = nranks;
    c->ce.reset(new CeState());
    CeState &ce = *c->ce;
    CFD_CHECK_HIP(hipExtMallocWithFlags((void **)&ce.flags, kCeFlagBytes, hipDeviceMallocUncached));
    CFD_CHECK_HIP(hipMemset(ce.flags, 0, kCeFlagBytes));
    CFD_CHECK_HIP(hipMalloc((void **)&ce.peers_dev, sizeof(unsigned *) * kCeMaxRanks));
    CFD_CHECK_HIP(hipMalloc((void **)&ce.status, sizeof(int)));
    CFD_CHECK_HIP(hipMemset(ce.status, 0, sizeof(int)));
    for (int d = 0; d < 2; ++d) {
        CFD_CHECK_HIP(hipStreamCreateWithFlags(&ce.xs[d], hipStreamNonBlocking));
        CFD_CHECK_HIP(hipEventCreateWithFlags(&ce.xev[d], hipEventDisableTiming));
    }
    CFD_CHECK_HIP(hipEventCreateWithFlags(&c->ev_boundary, hipEventDisableTiming));
    CFD_CHECK_HIP(hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming));
    CFD_CHECK_HIP(hipDeviceSynchronize());
    *comm = c.release();
    return CFD_OK;
}

size_t cfd_comm_ipc_blob_bytes(void) { return sizeof(CeBlob); }

int cfd_comm_ipc_export(void *comm, const float *phi, const float *phi_tmp, size_t n, void *blob) {
    return cfd_comm_ipc_export_ghost(comm, phi, phi_tmp, n, 0, blob);
}

int cfd_comm_ipc_export_ghost(void *comm, const float *phi, const float *phi_tmp, size_t n, size_t ghost_elems,
                              void *blob) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && c->ce && phi && phi_tmp && phi != phi_tmp && n > 0 && blob,
                "comm_ipc_export: needs a copy-engine comm, two distinct buffers and a blob");
    CFD_REQUIRE(2 * ghost_elems <= n, "comm_ipc_export: %zu ghost elements per side of a %zu-element array",
                ghost_elems, n);
    CeState &ce = *c->ce;
    CeBlob b;
    memset(&b, 0, sizeof b);
    b.magic = kCeMagic;
    b.version = 2;
    b.rank = c->rank;
    b.nranks = c->nranks;
    const float *bufs[2] = {phi, phi_tmp};
    static const bool force_landing = [] {  // CFD_CE_LANDING=1: landing buffers at any size (tests)
        const char *e = getenv("CFD_CE_LANDING");
        return e && atoi(e) == 1;
    }();
    bool big = false;
    for (int i = 0; i < 2; ++i) {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        CFD_CHECK_HIP(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)bufs[i]));
        const size_t off = (size_t)((const char *)bufs[i] - (const char *)base);
        CFD_REQUIRE(off + n * sizeof(float) <= size, "comm_ipc_export: buffer %d overruns its allocation", i);
        big |= size >= kIpcMapMax;
        CFD_CHECK_HIP(hipIpcGetMemHandle(&b.buf_h[i], (void *)base));
        b.buf_off[i] = off;
        b.buf_n[i] = n;
    }
    CFD_REQUIRE(!big || ghost_elems > 0, "comm_ipc_export: an allocation of 2 GiB or more cannot be mapped by "
                "the peers (hipIpcOpenMemHandle hangs past 2 GiB); export it with its ghost size "
                "(cfd_comm_ipc_export_ghost) so that its ghosts arrive through a landing buffer");
    float *land = nullptr;
    const size_t land_n = (big || force_landing) ? ghost_elems : 0;
    if (land_n) {
        CFD_CHECK_HIP(hipMalloc((void **)&land, 4 * land_n * sizeof(float)));
        CFD_CHECK_HIP(hipMemset(land, 0, 4 * land_n * sizeof(float)));
        ce.lands.push_back(land);
        CFD_CHECK_HIP(hipIpcGetMemHandle(&b.land_h, land));
        b.land_n = land_n;
    }
    CFD_CHECK_HIP(hipIpcGetMemHandle(&b.flags_h, ce.flags));
    ce.pend[0] = const_cast<float *>(phi);
    ce.pend[1] = const_cast<float *>(phi_tmp);
    ce.pend_n = n;
    ce.pend_land = land;
    ce.pend_land_n = land_n;
    memcpy(blob, &b, sizeof b);
    return CFD_OK;
}

int cfd_comm_ipc_import(void *comm, const void *blobs, int nblobs) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && c->ce && blobs && nblobs == c->nranks,
                "comm_ipc_import: needs a copy-engine comm and one blob per rank (%d)", c ? c->nranks : 0);
    CeState &ce = *c->ce;
    CFD_REQUIRE(ce.pend[0], "comm_ipc_import: export this rank's buffers first");
    std::vector<CeBlob> in((size_t)nblobs);
    memcpy(in.data(), blobs, sizeof(CeBlob) * (size_t)nblobs);
    for (int r = 0; r < nblobs; ++r)
        CFD_REQUIRE(in[r].magic == kCeMagic && in[r].version == 2 && in[r].rank == r &&
                        in[r].nranks == c->nranks,
                    "comm_ipc_import: blob %d is not rank %d's export of a %d-rank comm", r, r, c->nranks);
    // every rank's flag block, mapped once (it lives as long as the comm)
    if (ce.peer_flags.empty()) {
        ce.peer_flags.assign((size_t)c->nranks, nullptr);
        for (int r = 0; r < c->nranks; ++r) {
            if (r == c->rank) {
                ce.peer_flags[r] = ce.flags;
                continue;
            }
            char *base = nullptr;
            int rc = ce_map(ce, r, in[r].flags_h, &base);
            if (rc) return rc;
            ce.peer_flags[r] = reinterpret_cast<unsigned *>(base);
        }
        CFD_CHECK_HIP(hipMemcpy(ce.peers_dev, ce.peer_flags.data(), sizeof(unsigned *) * c->nranks,
                                hipMemcpyHostToDevice));
    }
    // a re-attached pair replaces its entry (its peers' buffers may be new)
    CeState::Attachment at{{ce.pend[0], ce.pend[1]}, ce.pend_n, std::move(in), ce.pend_land, ce.pend_land_n};
    int k = 0;
    while (k < (int)ce.att.size() && !(ce.att[k].mine[0] == at.mine[0] && ce.att[k].mine[1] == at.mine[1])) ++k;
    if (k == (int)ce.att.size())
        ce.att.push_back(std::move(at));
    else
        ce.att[k] = std::move(at);
    ce.pend[0] = ce.pend[1] = nullptr;
    ce.pend_land = nullptr;
    ce.pend_land_n = 0;
    // the z-neighbours' buffers are mapped now (others on first use)
    ce.cur = k;
    for (int r : {c->rank - 1, c->rank + 1}) {
        if (r < 0 || r >= c->nranks) continue;
        for (int bi = 0; bi < 2; ++bi) {
            float *p = nullptr;
            size_t n = 0;
            int rc = ce_peer_buf(c, r, bi, &p, &n);
            if (rc) return rc;
        }
    }
    return CFD_OK;
}

int cfd_comm_status(void *comm, int *timeouts) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && timeouts, "comm_status: null argument");
    *timeouts = 0;
    if (!c->ce) return CFD_OK;
    CFD_CHECK_HIP(hipDeviceSynchronize());
    CFD_CHECK_HIP(hipMemcpy(timeouts, c->ce->status, sizeof(int), hipMemcpyDeviceToHost));
    if (*timeouts) {
        set_error("slab (copy engines): a wait for a neighbour timed out");
        return CFD_E_COMM;
    }
    return CFD_OK;
}

int cfd_comm_destroy(void *comm) {
    if (!comm) return CFD_OK;
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    if (c->ce) {
        CeState &ce = *c->ce;
        (void)hipDeviceSynchronize();
        for (const CeState::Map &m : ce.maps) (void)hipIpcCloseMemHandle(m.base);
        for (int d = 0; d < 2; ++d) {
            if (ce.xs[d]) (void)hipStreamDestroy(ce.xs[d]);
            if (ce.xev[d]) (void)hipEventDestroy(ce.xev[d]);
        }
        for (float *p : ce.lands) (void)hipFree(p);
        if (ce.flags) (void)hipFree(ce.flags);
        if (ce.peers_dev) (void)hipFree(ce.peers_dev);
        if (ce.status) (void)hipFree(ce.status);
    }
    if (c->ev_boundary) (void)hipEventDestroy(c->ev_boundary);
    if (c->ev_comm) (void)hipEventDestroy(c->ev_comm);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->xstream) (void)hipStreamDestroy(c->xstream);
    if (c->grp) {
        LocalGroup::Slot &me = c->grp->slot[c->rank];
        if (me.ready) (void)hipEventDestroy(me.ready);
        if (me.done) (void)hipEventDestroy(me.done);
        me.ready = me.done = nullptr;
    }
    ncclResult_t r = c->comm ? ncclCommDestroy(c->comm) : ncclSuccess;
    delete c;
    if (r != ncclSuccess) {
        set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return CFD_E_COMM;
    }
    return CFD_OK;
}

// The slab Jacobi solve (cfd_slab_jacobi3d_f32 / _zero_f32).  zero: phi starts
// as zeros (every rank's, ghosts included), so nothing of phi is read before
// the first pass writes it: no fill, no initial ghost exchange.  With a
// workspace and the blocked kernels, the first pass of each plane range is the
// fused one (jacobi3d_tbr_first_pass: raw div in, rhs of its planes out); the
// planes outside the update range (ghosts, global Dirichlet planes) get theirs
// from the RHS kernel, which the pass' halo levels read.
static int slab_jacobi3d(SlabComm *c, const float *div, float *phi, float *phi_tmp, float *rhs_ws,
                         const uint8_t *mask, int nz_local, int G, int ny, int nx, int lo_peer,
                         int hi_peer, int z_update_begin, int z_update_end, double h, float dt,
                         int iters, int overlap, void *stream, void *comm_stream, bool zero) {
    const int ghost = G;
    if (iters == 0) {
        if (zero) CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(float) * (size_t)(nz_local + 2 * G) * ny * nx,
                                               as_stream(stream)));
        return CFD_OK;
    }
    hipStream_t s = as_stream(stream);
    hipStream_t cs = comm_stream ? as_stream(comm_stream) : s;
    PartitionScope part(c, overlap && (lo_peer >= 0 || hi_peer >= 0) &&
                               z_update_end - z_update_begin >= 2 * ghost + 1, s, cs);
    const int nzt = nz_local + 2 * G;
    const size_t plane = (size_t)ny * nx;
    const float h2 = (float)(h * h);
    int rc;
    // Dirichlet faces of the owned planes: rows y=0, ny-1, and the global
    // boundary planes (owned planes outside the update range) in full.
    // Ghost planes arrive whole from the neighbours.
    const int full_lo = z_update_begin > G ? G : -1;
    const int full_hi = z_update_end < nz_local + G ? nz_local + G - 1 : -1;
    const int zb = z_update_begin, ze = z_update_end;
    const bool pre = rhs_ws != nullptr;
    const bool vec_ok = nx % 4 == 0 && aligned16(phi) && aligned16(phi_tmp) && aligned16(div) &&
                        (!pre || aligned16(rhs_ws));
    // k sweeps per pass need k-deep ghosts (and no mask): k = min(G, configured levels)
    const bool tb = G >= 2 && jacobi3d_tb_enabled() && !mask && vec_ok && ny >= 3;
    const int K = tb ? (jacobi3d_tb_levels() < G ? jacobi3d_tb_levels() : G) : 1;
    // the fused first pass (see above); its depth k1 makes the later passes
    // whole passes of K where it can (as in the single-GPU blocked solve)
    const bool first = pre && K >= 2 && jacobi3d_tb_prefetch() == 1 && iters >= 2;
    int k1 = K;
    if (first) {
        const int r = iters % K;
        k1 = (r == 2 || r == 3) ? r : r == 0 ? K : (K < 3 ? K : 3);
        if (k1 > iters) k1 = iters;
    }
    const int npass = first ? 1 + (iters - k1 + K - 1) / K : (iters + K - 1) / K;
    if (zero && !first) {  // the zero fill, then the general solve
        CFD_CHECK_HIP(hipMemsetAsync(phi, 0, sizeof(float) * plane * nzt, s));
        zero = false;
    }
    if (zero) {
        // phi = zeros: the Dirichlet faces of both buffers are zero, phi is
        // never read, and the first pass writes the buffer that makes the
        // last pass land in phi
        if ((rc = launch_fix_faces3d(nullptr, phi, nullptr, ny, nx, G, nz_local + G, full_lo, full_hi, s)) ||
            (rc = launch_fix_faces3d(nullptr, phi_tmp, nullptr, ny, nx, G, nz_local + G, full_lo, full_hi, s)))
            return rc;
    } else if ((rc = launch_fix_faces3d(phi, phi_tmp, mask, ny, nx, G, nz_local + G, full_lo, full_hi, s))) {
        return rc;
    }
    const float *src = div;
    if (pre) {
        if (first) {  // planes the first pass does not own: ghosts, global Dirichlet planes
            if ((rc = launch_rhs_f32(div, rhs_ws, plane * zb, h2, dt, s)) ||
                (rc = launch_rhs_f32(div + plane * ze, rhs_ws + plane * ze, plane * (nzt - ze), h2, dt, s)))
                return rc;
        } else if ((rc = launch_rhs_f32(div, rhs_ws, plane * nzt, h2, dt, s))) {
            return rc;
        }
        src = rhs_ws;
    }
    if (c->grp && (rc = register_local(c, phi, phi_tmp, nullptr, nz_local, G, plane))) return rc;
    if (c->ce && ((rc = ce_check_attached(c, phi, phi_tmp)) || (rc = ce_begin(c, s, lo_peer, hi_peer)))) return rc;
    // ghosts of the initial guess (a zero start reads none)
    if (!zero) {
        if (c->ce) {
            CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
            if ((rc = exchange_ce(c, phi, nz_local, G, plane, lo_peer, hi_peer, c->ev_boundary)) ||
                (rc = ce_sync(c, s, lo_peer, hi_peer, nullptr, 0, 0)))
                return rc;
        } else if ((rc = exchange(c, phi, nz_local, G, plane, lo_peer, hi_peer, s))) {
            return rc;
        }
    }
    const int fixed_lo = zb > G, fixed_hi = ze < nz_local + G;
    // owned planes a neighbour needs after each pass: the G next to it
    const bool lo_b = lo_peer >= 0, hi_b = hi_peer >= 0;
    const bool can_overlap = overlap && (lo_peer >= 0 || hi_peer >= 0) && (ze - zb) >= 2 * G + 1;
    float *a = phi, *b = phi_tmp;
    if (zero && npass % 2 == 1) {
        a = phi_tmp;
        b = phi;
    }
    const int tk = timing_begin(s);
    int done = 0;
    while (done < iters) {
        const int k = done == 0 && first ? k1 : iters - done < K ? iters - done : K;
        auto run = [&](int z0, int z1) -> int {
            if (z1 <= z0) return CFD_OK;
            if (done == 0 && first)
                return jacobi3d_tbr_first_pass(k, b, div, rhs_ws, a, nzt, ny, nx, z0, z1,
                                               z0 == zb && fixed_lo, z1 == ze && fixed_hi, h2, dt,
                                               jacobi3d_tb_zchunk(), zero, s);
            if (k == 1)
                return jacobi3d_sweep(a, b, src, mask, nzt, ny, nx, z0, z1, h2, dt, pre, nullptr, s);
            return jacobi3d_blocked_pass(k, a, b, src, nzt, ny, nx, z0, z1, z0 == zb && fixed_lo,
                                         z1 == ze && fixed_hi, h2, dt, pre, s);
        };
        if (!can_overlap) {
            if ((rc = run(zb, ze))) return rc;
            if (c->ce) {
                CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
                if ((rc = exchange_ce(c, b, nz_local, G, plane, lo_peer, hi_peer, c->ev_boundary)) ||
                    (rc = ce_sync(c, s, lo_peer, hi_peer, nullptr, 0, 0)))
                    return rc;
            } else if ((rc = exchange(c, b, nz_local, G, plane, lo_peer, hi_peer, s))) {
                return rc;
            }
        } else {
            // boundary planes first, their exchange on the comm stream, the
            // interior meanwhile on the main stream
            int ib = zb, ie = ze;
            if (lo_b) {
                if ((rc = run(zb, zb + G))) return rc;
                ib = zb + G;
            }
            if (hi_b) {
                if ((rc = run(ze - G, ze))) return rc;
                ie = ze - G;
            }
            // the interior is enqueued before the exchange: the RCCL calls
            // cost the host tens of microseconds, and the interior does not
            // depend on them (a wait captures the event as recorded so far)
            CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
            if ((rc = run(ib, ie))) return rc;
            if (c->ce) {
                // copy engines: no CUs, so nothing to reserve; the next pass
                // waits for the neighbours' planes behind the interior
                if ((rc = exchange_ce(c, b, nz_local, G, plane, lo_peer, hi_peer, c->ev_boundary)) ||
                    (rc = ce_sync(c, s, lo_peer, hi_peer, nullptr, 0, 0)))
                    return rc;
            } else {
                CFD_CHECK_HIP(hipStreamWaitEvent(cs, c->ev_boundary, 0));
                if ((rc = exchange(c, b, nz_local, G, plane, lo_peer, hi_peer, cs))) return rc;
                CFD_CHECK_HIP(hipEventRecord(c->ev_comm, cs));
                CFD_CHECK_HIP(hipStreamWaitEvent(s, c->ev_comm, 0));
            }
        }
        // after the first pass, the other buffer gets the final owned faces too
        if (done == 0 && !zero &&
            (rc = launch_fix_faces3d(phi_tmp, phi, nullptr, ny, nx, G, nz_local + G, full_lo, full_hi, s)))
            return rc;
        done += k;
        float *t = a;
        a = b;
        b = t;
    }
    if (c->ce && (rc = ce_join(c, s))) return rc;
    timing_end(tk, s, iters);
    if (a != phi)
        CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(float) * plane * nzt, hipMemcpyDeviceToDevice, s));
    return CFD_OK;
}

int cfd_slab_jacobi3d_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                          float *rhs_ws, const uint8_t *mask, int nz_local, int ghost, int ny,
                          int nx, int lo_peer, int hi_peer, int z_update_begin, int z_update_end,
                          double h, float dt, int iters, int overlap, void *stream,
                          void *comm_stream) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && div && phi && phi_tmp, "slab_jacobi3d: null pointer");
    CFD_REQUIRE(ghost >= 1 && ghost <= 4, "slab_jacobi3d: ghost depth must be 1..4");
    CFD_REQUIRE(nz_local >= ghost && ny >= 1 && nx >= 1 && iters >= 0, "slab_jacobi3d: bad shape");
    const int G = ghost;
    CFD_REQUIRE(z_update_begin >= G && z_update_end <= nz_local + G &&
                    z_update_begin <= z_update_end,
                "slab_jacobi3d: update range [%d,%d) outside owned planes %d..%d", z_update_begin,
                z_update_end, G, nz_local + G - 1);
    CFD_REQUIRE(lo_peer < c->nranks && hi_peer < c->nranks, "slab_jacobi3d: bad peer");
    if (iters == 0) return CFD_OK;
    return slab_jacobi3d(c, div, phi, phi_tmp, rhs_ws, mask, nz_local, G, ny, nx, lo_peer, hi_peer,
                         z_update_begin, z_update_end, h, dt, iters, overlap, stream, comm_stream, false);
}

int cfd_slab_jacobi3d_zero_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                               float *rhs_ws, int nz_local, int ghost, int ny, int nx, int lo_peer,
                               int hi_peer, int z_update_begin, int z_update_end, double h, float dt,
                               int iters, int overlap, void *stream, void *comm_stream) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && div && phi && phi_tmp, "slab_jacobi3d_zero: null pointer");
    CFD_REQUIRE(ghost >= 1 && ghost <= 4, "slab_jacobi3d_zero: ghost depth must be 1..4");
    CFD_REQUIRE(nz_local >= ghost && ny >= 1 && nx >= 1 && iters >= 0, "slab_jacobi3d_zero: bad shape");
    CFD_REQUIRE(z_update_begin >= ghost && z_update_end <= nz_local + ghost &&
                    z_update_begin <= z_update_end,
                "slab_jacobi3d_zero: update range [%d,%d) outside owned planes %d..%d", z_update_begin,
                z_update_end, ghost, nz_local + ghost - 1);
    CFD_REQUIRE(lo_peer < c->nranks && hi_peer < c->nranks, "slab_jacobi3d_zero: bad peer");
    return slab_jacobi3d(c, div, phi, phi_tmp, rhs_ws, nullptr, nz_local, ghost, ny, nx, lo_peer, hi_peer,
                         z_update_begin, z_update_end, h, dt, iters, overlap, stream, comm_stream, true);
}

// Distributed red-black GS (config 5).  Colours are global: local plane k is
// global plane z_global_offset + k, so the decomposed sweep updates exactly
// the cells the single-GPU sweep updates, from the same neighbour values
// (bit-identical for every rank count).  The stop rule needs the GLOBAL
// max|change| of each iteration: one ncclAllReduce(max) of 4 bytes per
// iteration (skipped when tolerance <= 0, which can never stop).
//  * fused (ghost >= 2, no mask): one out-of-place pass per iteration (two per
//    pass with ghost 4 and blocking depth 4); its G owned boundary planes per
//    side go out while the interior runs.
//  * otherwise: in-place colour passes, a G-plane exchange after each colour.
int cfd_slab_rbgs3d_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                        const uint8_t *mask, int nz_local, int ghost, int ny, int nx, int lo_peer,
                        int hi_peer, int z_update_begin, int z_update_end, int z_global_offset,
                        double dx, double dy, double dz, float dt, int iterations,
                        double tolerance, void *ws, int *iters_done, int overlap, void *stream,
                        void *comm_stream) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && div && phi && ws, "slab_rbgs3d: null pointer");
    CFD_REQUIRE(ghost >= 1 && ghost <= 4, "slab_rbgs3d: ghost depth must be 1..4");
    CFD_REQUIRE(nz_local >= ghost && ny >= 1 && nx >= 1 && iterations >= 0, "slab_rbgs3d: bad shape");
    const int G = ghost;
    CFD_REQUIRE(z_update_begin >= G && z_update_end <= nz_local + G &&
                    z_update_begin <= z_update_end,
                "slab_rbgs3d: update range [%d,%d) outside owned planes %d..%d", z_update_begin,
                z_update_end, G, nz_local + G - 1);
    CFD_REQUIRE(lo_peer < c->nranks && hi_peer < c->nranks, "slab_rbgs3d: bad peer");
    hipStream_t s = as_stream(stream);
    hipStream_t cs = comm_stream ? as_stream(comm_stream) : s;
    PartitionScope part(c, overlap && (lo_peer >= 0 || hi_peer >= 0) &&
                               z_update_end - z_update_begin >= 2 * ghost + 1, s, cs);
    RbgsWs *w = reinterpret_cast<RbgsWs *>(ws);
    const RbgsConsts k = rbgs3d_consts(dx, dy, dz, dt, tolerance);
    int rc = launch_rbgs_init(w, iterations, k.tol, iters_done, s);
    if (rc || iterations == 0 || ny < 3 || nx < 3) return rc;
    const int nzt = nz_local + 2 * G;
    const size_t plane = (size_t)ny * nx;
    const int zb = z_update_begin, ze = z_update_end, zoff = z_global_offset;
    const int fixed_lo = zb > G, fixed_hi = ze < nz_local + G;
    // a one-rank comm peered with itself (the per-rank rehearsal) reduces too
    const bool self_peered = !c->grp && (lo_peer == c->rank || hi_peer == c->rank);
    const bool reduce = (c->nranks > 1 || self_peered) && k.tol > 0.0f;
    auto allreduce = [&](int it, int cnt, hipStream_t st) -> int {
        if (reduce && c->grp) return allreduce_local(c, it, cnt, st);
        if (reduce)
            CFD_CHECK_NCCL(ncclAllReduce(w->maxc + it, w->maxc + it, cnt, ncclFloat32, ncclMax, c->comm, st));
        return CFD_OK;
    };
    if (c->grp && (rc = register_local(c, phi, phi_tmp, w, nz_local, G, plane))) return rc;
    // copy engines: the exchange of `a` and the next pass's wait for it (with
    // the global maxima of iterations it .. it+cnt-1 when cnt > 0)
    auto ce_step = [&](float *a, int it, int cnt) -> int {
        int r;
        CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
        if ((r = exchange_ce(c, a, nz_local, G, plane, lo_peer, hi_peer, c->ev_boundary))) return r;
        return ce_sync(c, s, lo_peer, hi_peer, reduce ? w->maxc : nullptr, it, cnt);
    };
    if (c->ce && ((rc = ce_check_attached(c, phi, phi_tmp)) || (rc = ce_begin(c, s, lo_peer, hi_peer)))) return rc;
    // ghosts of the initial guess
    if (c->ce) {
        if ((rc = ce_step(phi, 0, 0))) return rc;
    } else if ((rc = exchange(c, phi, nz_local, G, plane, lo_peer, hi_peer, s))) {
        return rc;
    }
    const int tk = timing_begin(s);
    const bool fused = G >= 2 && rbgs3d_fused_ok(phi, phi_tmp, div, mask, nx);
    if (!fused) {
        for (int it = 0; it < iterations; ++it) {
            for (int colour = 0; colour < 2; ++colour) {
                if ((rc = rbgs3d_colour_pass(colour, phi, div, mask, ny, nx, zb, ze, zoff, k, w, it, s)))
                    return rc;
                if (c->ce) {
                    if ((rc = ce_step(phi, it, colour))) return rc;  // maxima after colour 1
                } else if ((rc = exchange(c, phi, nz_local, G, plane, lo_peer, hi_peer, s))) {
                    return rc;
                }
            }
            if (!c->ce && (rc = allreduce(it, 1, s))) return rc;
        }
        if (c->ce && (rc = ce_join(c, s))) return rc;
        timing_end(tk, s, iterations);
        return launch_rbgs_finish(w, phi, nullptr, plane * nzt, iters_done, s);
    }
    // pp iterations per pass need 2*pp-deep ghosts (the pass recomputes the
    // inner ghost planes' intermediate colours)
    const int pp = rbgs3d_iters_per_pass() == 2 && G >= 4 ? 2 : 1;
    // owned faces the passes never write, in both buffers
    const int full_lo = fixed_lo ? G : -1;
    const int full_hi = fixed_hi ? nz_local + G - 1 : -1;
    if ((rc = launch_fix_faces3d(phi, phi_tmp, nullptr, ny, nx, G, nz_local + G, full_lo, full_hi, s)))
        return rc;
    const bool can_overlap = overlap && (lo_peer >= 0 || hi_peer >= 0) && (ze - zb) >= 2 * G + 1;
    // Lagged stop test (overlapped, one iteration per pass): pass j tests
    // maxc[j-2] and maxc[j-3] instead of maxc[j-1] and maxc[j-2], so the
    // allreduce of iteration j-1 runs beside pass j's boundary launches
    // instead of between the passes.  A stop at iteration n then costs one
    // wasted pass n+1; it writes the buffer of iteration n-1, so iteration n's
    // result is intact, and maxc of a skipped pass stays 0 (< tol), which keeps
    // every later pass skipped.  rbgs_count / rbgs_copy are unchanged.
    const int lag = can_overlap && reduce && pp == 1 && !c->ce ? 1 : 0;
    float *a = phi, *b = phi_tmp;
    for (int it = 0; it < iterations;) {
        const int m = iterations - it >= pp ? pp : 1;
        auto run = [&](int z0, int z1) -> int {
            if (z1 <= z0) return CFD_OK;
            return rbgs3d_fused_pass(a, b, div, nzt, ny, nx, z0, z1, z0 == zb && fixed_lo,
                                     z1 == ze && fixed_hi, zoff, k, it, m, w, s, lag);
        };
        if (!can_overlap) {
            if ((rc = run(zb, ze))) return rc;
            if (c->ce) {
                if ((rc = ce_step(b, it, m))) return rc;
            } else if ((rc = exchange(c, b, nz_local, G, plane, lo_peer, hi_peer, s)) ||
                       (rc = allreduce(it, m, s))) {
                return rc;
            }
        } else {
            int ib = zb, ie = ze;
            if (lo_peer >= 0) {
                if ((rc = run(zb, zb + G))) return rc;
                ib = zb + G;
            }
            if (hi_peer >= 0) {
                if ((rc = run(ze - G, ze))) return rc;
                ie = ze - G;
            }
            // interior enqueued before the exchange (see the Jacobi driver)
            CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
            if ((rc = run(ib, ie))) return rc;
            if (c->ce) {
                // copies started after the boundary planes; the sync behind
                // the interior waits for the ghosts and combines the maxima
                if ((rc = exchange_ce(c, b, nz_local, G, plane, lo_peer, hi_peer, c->ev_boundary)) ||
                    (rc = ce_sync(c, s, lo_peer, hi_peer, reduce ? w->maxc : nullptr, it, m)))
                    return rc;
                it += m;
                float *t = a;
                a = b;
                b = t;
                continue;
            }
            CFD_CHECK_HIP(hipStreamWaitEvent(cs, c->ev_boundary, 0));
            if ((rc = exchange(c, b, nz_local, G, plane, lo_peer, hi_peer, cs))) return rc;
            // lagged: the next pass waits for the exchange only (and, through
            // the in-order exchange stream, for the previous allreduce)
            if (lag) CFD_CHECK_HIP(hipEventRecord(c->ev_comm, cs));
            if (reduce) {
                // the global max needs the interior's contribution too
                CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
                CFD_CHECK_HIP(hipStreamWaitEvent(cs, c->ev_boundary, 0));
                if ((rc = allreduce(it, m, cs))) return rc;
            }
            if (!lag) CFD_CHECK_HIP(hipEventRecord(c->ev_comm, cs));
            CFD_CHECK_HIP(hipStreamWaitEvent(s, c->ev_comm, 0));
        }
        it += m;
        float *t = a;
        a = b;
        b = t;
    }
    if (lag) {  // the last allreduce
        CFD_CHECK_HIP(hipEventRecord(c->ev_comm, cs));
        CFD_CHECK_HIP(hipStreamWaitEvent(s, c->ev_comm, 0));
    }
    if (c->ce && (rc = ce_join(c, s))) return rc;
    timing_end(tk, s, iterations);
    // count (same on every rank: the maxima are global), re-run a pair
    // pass's first iteration if the stop fell inside it, pick the buffer
    if ((rc = launch_rbgs_count(w, iters_done, s))) return rc;
    if (pp == 2 &&
        (rc = rbgs3d_tbr_pass(phi, phi_tmp, div, nzt, ny, nx, zb, ze, fixed_lo, fixed_hi, zoff, k, 0, 2,
                              w, 4, 2 * iterations, 0, s)))
        return rc;
    return launch_rbgs_copy(w, phi, phi_tmp, plane * nzt, 2 * pp, s);
}

}  // extern "C"
