// capi.hip -- error reporting, identification and sweep timing of libcfdsim.
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "internal.hpp"

namespace cfd {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Sweep timing for the bench harness: each solve brackets its sweep launches
// with a HIP event pair recorded on the stream it launches on.
// The event pool is reused after each cfd_timing_read(reset) / enable and
// capped: past kMaxPairs unread solves, further solves are not timed and the
// next read reports the overflow.  Nothing here runs at thread or process
// exit: a destructor calling hipEventDestroy would run from exit(), where the
// HIP runtime's own teardown (an exit handler of libamdhip64) may already have
// released the device (the r05 exit-time SIGSEGV).  The events
// are released by cfd_release_thread_resources, or with the process.
struct Timing {
    static constexpr size_t kMaxPairs = 1 << 14;
    bool on = false, overflow = false;
    std::vector<hipEvent_t> start, stop;
    std::vector<long long> sweeps;
    std::vector<int> channel;
    size_t used = 0;
};
static thread_local Timing g_timing;  // per host thread, like the tuning knobs

static void release_thread_timing() {
    for (size_t k = 0; k < g_timing.start.size(); ++k) {
        (void)hipEventSynchronize(g_timing.stop[k]);
        (void)hipEventDestroy(g_timing.start[k]);
        (void)hipEventDestroy(g_timing.stop[k]);
    }
    g_timing.start.clear();
    g_timing.stop.clear();
    g_timing.sweeps.clear();
    g_timing.channel.clear();
    g_timing.used = 0;
    g_timing.overflow = false;
}

// Process defaults of the tuning knobs: the CFD_* environment variables (A/B
// knobs of the bench scripts), validated, read once.
static int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
}
static Tuning process_defaults() {
    static const Tuning d = [] {
        Tuning t;
        const int k = env_int("CFD_J2_SMALL_K", 4);
        t.j2s_k = k >= 1 && k <= 8 ? k : 4;
        t.j2s_rw = env_int("CFD_J2_SMALL_RW", 1) == 2 ? 2 : 1;
        t.j2s_vec = env_int("CFD_J2_SMALL_VEC", 1) == 1 ? 1 : 0;  // 0: 16 bytes per lane
        const int dd = env_int("CFD_J2_DMA", t.j2_dma);
        t.j2_dma = dd == 0 || dd == 4 || dd == 6 ? dd : t.j2_dma;
        t.gs_rw = env_int("CFD_GS_SMALL_RW", 2) == 1 ? 1 : 2;
        t.gs_vec = env_int("CFD_GS_SMALL_VEC", 1) == 4 ? 4 : 1;
        t.gs_wpb = env_int("CFD_GS_SMALL_WPB", 4) == 16 ? 16 : 4;
        t.gs_wg = env_int("CFD_GS_SMALL_WG", t.gs_wg) != 0;
        t.gs_persist = env_int("CFD_GS_PERSIST", t.gs_persist) != 0;
        t.j2_persist = env_int("CFD_J2_PERSIST", t.j2_persist) != 0;
        const int jn = env_int("CFD_J2P_NI", t.j2p_ni);
        t.j2p_ni = jn == 4 || jn == 6 || jn == 8 || jn == 10 ? jn : t.j2p_ni;
        t.j2p_pairs = env_int("CFD_J2P_PAIRS", t.j2p_pairs) != 0;
        t.gs_pairs = env_int("CFD_GS_PAIRS", t.gs_pairs) != 0;
        const int pv = env_int("CFD_PRED_VARIANT", t.pred_variant);
        t.pred_variant = pv >= 0 && pv <= 2 ? pv : t.pred_variant;
        const int pw = env_int("CFD_PRED_VEC", t.pred_vec);
        t.pred_vec = pw == 1 || pw == 2 || pw == 4 ? pw : t.pred_vec;
        const int pr = env_int("CFD_PRED_ROWS", t.pred_rows);
        t.pred_rows = pr >= 0 ? pr : t.pred_rows;
        const int ni = env_int("CFD_GS_SMALL_NI", t.gs_ni);
        t.gs_ni = ni >= 1 && ni <= 5 ? ni : t.gs_ni;
        return t;
    }();
    return d;
}
Tuning &tuning() {
    static thread_local Tuning t = process_defaults();
    return t;
}

int timing_begin(hipStream_t s, int channel) {
    if (!g_timing.on) return -1;
    if (g_timing.used >= Timing::kMaxPairs) {
        g_timing.overflow = true;
        return -1;
    }
    if (g_timing.used == g_timing.start.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
        g_timing.start.push_back(a);
        g_timing.stop.push_back(b);
        g_timing.sweeps.push_back(0);
        g_timing.channel.push_back(0);
    }
    const int k = (int)g_timing.used++;
    g_timing.channel[k] = channel;
    if (hipEventRecord(g_timing.start[k], s) != hipSuccess) return -1;
    return k;
}

// a timing_begin whose work did not run (the last pair only)
void timing_cancel(int k) {
    if (k >= 0 && (size_t)k + 1 == g_timing.used) --g_timing.used;
}

void timing_end(int k, hipStream_t s, long long sweeps) {
    if (k < 0) return;
    g_timing.sweeps[k] = sweeps;
    (void)hipEventRecord(g_timing.stop[k], s);
}

// Failure words of the persistent solves, one per (device, stream): a solve
// counts its expired waits into the word of the stream it runs on, and
// cfd_persistent_status_stream reads and clears that word with an async copy
// on the same stream (no device-wide synchronisation, no other stream's
// failures consumed).  Kept for the life of the process (never freed at exit).
namespace {
struct FailWords {
    std::mutex mu;
    std::map<std::pair<int, hipStream_t>, int *> words;
};
FailWords &fail_words() {
    static FailWords *f = new FailWords;  // never destroyed: no exit-time teardown
    return *f;
}
}  // namespace

int *persist_fail_word(hipStream_t s, bool create) {
    thread_local int c_dev = -1;
    thread_local hipStream_t c_s = nullptr;
    thread_local int *c_w = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (c_w && c_dev == dev && c_s == s) return c_w;
    FailWords &f = fail_words();
    std::lock_guard<std::mutex> lk(f.mu);
    auto it = f.words.find({dev, s});
    int *p = it == f.words.end() ? nullptr : it->second;
    if (!p && create) {
        if (hipMalloc(&p, 256) != hipSuccess) return nullptr;
        // zeroed on the stream that will use it, ahead of its first solve
        if (hipMemsetAsync(p, 0, 256, s) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        f.words[{dev, s}] = p;
    }
    if (p) {
        c_dev = dev;
        c_s = s;
        c_w = p;
    }
    return p;
}

unsigned *energy_scratch(hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, unsigned *> bufs;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    unsigned *&p = bufs[{dev, s}];
    if (!p) {
        const size_t bytes = 64 + kEnergyBlocks * sizeof(double);
        if (hipMalloc(&p, bytes) != hipSuccess) return p = nullptr;
        // on s, ahead of the first k_energy_mean_mb (s may be a non-blocking
        // stream, which the null stream does not order)
        if (hipMemsetAsync(p, 0, bytes, s) != hipSuccess) {
            (void)hipFree(p);
            return p = nullptr;
        }
    }
    return p;
}

// Persistent launches of this process on one device run one at a time: each
// waits (on the device) for the previous one, whatever stream or host thread
// launched it.  A plain launch rests on the occupancy check, which assumes the
// chip is otherwise free of persistent tiles; two persistent solves on two
// streams could each end up partly resident, every resident tile waiting for a
// neighbour that cannot start until the poll bound expires.  The chain costs
// one event record per solve.  (Across processes on one device nothing orders
// them: cfd_set_persistent_launch(1, ...) -- cooperative launches -- is the
// setting for that.)
namespace {
struct PersistOrder {
    std::mutex mu;
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool any = false;
};
PersistOrder *persist_order(int dev) {
    static PersistOrder *o = new PersistOrder[64];  // never destroyed
    return dev >= 0 && dev < 64 ? &o[dev] : nullptr;
}
}  // namespace

int launch_persistent(const void *f, int nblocks, int threads, void *args, hipStream_t s) {
    void *kargs[] = {args};
    int dev = 0;
    PersistOrder *o = hipGetDevice(&dev) == hipSuccess ? persist_order(dev) : nullptr;
    if (!o) {
        set_error("persistent launch: no device");
        return -1;
    }
    std::lock_guard<std::mutex> lk(o->mu);
    if (!o->ev && hipEventCreateWithFlags(&o->ev, hipEventDisableTiming) != hipSuccess) {
        o->ev = nullptr;
        set_error("persistent launch: event creation failed");
        return -1;
    }
    if (o->any && o->last != s && hipStreamWaitEvent(s, o->ev, 0) != hipSuccess) {
        set_error("persistent launch: ordering after the previous persistent solve failed");
        return -1;
    }
    hipError_t e;
    if (tuning().persist_coop) {
        e = hipLaunchCooperativeKernel(f, dim3(nblocks), dim3(threads), kargs, 0, s);
        if (e == hipErrorCooperativeLaunchTooLarge) {
            (void)hipGetLastError();  // clear it: the caller runs the launch-per-pass path
            return 0;
        }
    } else {
        e = hipLaunchKernel(f, dim3(nblocks), dim3(threads), kargs, 0, s);
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        set_error("persistent launch failed: %s", hipGetErrorString(e));
        return -1;
    }
    if (hipEventRecord(o->ev, s) == hipSuccess) {
        o->last = s;
        o->any = true;
    } else {
        o->any = false;  // nothing to wait for: the next launch orders by its stream only
    }
    return 1;
}
}  // namespace cfd

using namespace cfd;

extern "C" {
int cfd_abi_version(void) { return CFD_ABI_VERSION; }
const char *cfd_last_error(void) { return cfd::g_err; }
const char *cfd_device_arch(void) { return "gfx950"; }

int cfd_reset_tuning(void) {
    tuning() = process_defaults();
    return CFD_OK;
}

int cfd_set_persistent_launch(int cooperative, long long poll_ticks) {
    CFD_REQUIRE(cooperative == 0 || cooperative == 1, "persistent launch: cooperative must be 0 or 1");
    CFD_REQUIRE(poll_ticks >= 0, "persistent launch: poll_ticks must be >= 0 (0 = the 20 s default)");
    tuning().persist_coop = cooperative;
    tuning().persist_poll = (unsigned long long)poll_ticks;
    return CFD_OK;
}

int cfd_persistent_status(int *expired) {
    CFD_REQUIRE(expired, "persistent_status: null pointer");
    *expired = 0;
    int dev = 0;
    CFD_CHECK_HIP(hipGetDevice(&dev));
    CFD_CHECK_HIP(hipDeviceSynchronize());
    FailWords &f = fail_words();
    std::lock_guard<std::mutex> lk(f.mu);
    for (auto &kv : f.words) {
        if (kv.first.first != dev) continue;
        int h = 0;
        CFD_CHECK_HIP(hipMemcpy(&h, kv.second, sizeof(int), hipMemcpyDeviceToHost));
        if (h) CFD_CHECK_HIP(hipMemset(kv.second, 0, sizeof(int)));
        *expired += h;
    }
    return CFD_OK;
}

int cfd_persistent_status_stream(void *stream, int *expired) {
    CFD_REQUIRE(expired, "persistent_status_stream: null pointer");
    *expired = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    int *w = persist_fail_word(s, false);
    if (!w) return CFD_OK;  // no persistent solve has run on this stream
    thread_local int *host = nullptr;  // pinned: the copy is a true async one
    if (!host) CFD_CHECK_HIP(hipHostMalloc(reinterpret_cast<void **>(&host), 64, hipHostMallocDefault));
    CFD_CHECK_HIP(hipMemcpyAsync(host, w, sizeof(int), hipMemcpyDeviceToHost, s));
    CFD_CHECK_HIP(hipMemsetAsync(w, 0, sizeof(int), s));
    CFD_CHECK_HIP(hipStreamSynchronize(s));
    *expired = *host;
    return CFD_OK;
}

int cfd_release_thread_resources(void) {
    release_thread_rings();
    release_thread_timing();
    return CFD_OK;
}

int cfd_set_small2d_shape(int j2_k, int j2_rw, int j2_vec, int gs_rw, int gs_vec, int gs_wpb) {
    CFD_REQUIRE(j2_k >= 0 && j2_k <= 8, "small-grid Jacobi sweeps per launch must be 0 (default) or 1..8");
    CFD_REQUIRE(j2_rw >= 0 && j2_rw <= 2, "small-grid Jacobi rows per wave must be 0 (default), 1 or 2");
    CFD_REQUIRE(j2_vec == 0 || j2_vec == 1 || j2_vec == 4,
                "small-grid Jacobi cells per lane must be 0 (default), 1 or 4 (16 bytes)");
    CFD_REQUIRE(gs_rw >= 0 && gs_rw <= 2, "small-grid GS rows per wave must be 0 (default), 1 or 2");
    CFD_REQUIRE(gs_vec == 0 || gs_vec == 1 || gs_vec == 4, "small-grid GS cells per lane must be 0, 1 or 4");
    CFD_REQUIRE(gs_wpb == 0 || gs_wpb == 4 || gs_wpb == 16, "small-grid GS waves per workgroup must be 0, 4 or 16");
    const Tuning d = process_defaults();
    Tuning &t = tuning();
    t.j2s_k = j2_k ? j2_k : d.j2s_k;
    t.j2s_rw = j2_rw ? j2_rw : d.j2s_rw;
    t.j2s_vec = j2_vec ? (j2_vec == 1 ? 1 : 0) : d.j2s_vec;
    t.gs_rw = gs_rw ? gs_rw : d.gs_rw;
    t.gs_vec = gs_vec ? gs_vec : d.gs_vec;
    t.gs_wpb = gs_wpb ? gs_wpb : d.gs_wpb;
    return CFD_OK;
}

int cfd_set_small2d_gs_iters(int iters_per_launch, int shared_rows) {
    CFD_REQUIRE(iters_per_launch >= 0 && iters_per_launch <= 5,
                "small-grid GS iterations per launch must be 0 (default) or 1..5");
    CFD_REQUIRE(shared_rows >= 0 && shared_rows <= 2, "small-grid GS shared_rows must be 0 (default), 1 or 2");
    const Tuning d = process_defaults();
    tuning().gs_ni = iters_per_launch ? iters_per_launch : d.gs_ni;
    tuning().gs_wg = shared_rows ? shared_rows == 2 : d.gs_wg;
    return CFD_OK;
}

int cfd_set_tbr_trace(void *buf, size_t bytes) {
    CFD_REQUIRE(!buf || bytes >= (size_t)16 * 64 * 5 * 8, "tbr trace buffer: 40 KiB");
    tuning().tbr_trace = buf;
    return CFD_OK;
}

int cfd_set_small2d_gs_trace(void *buf, size_t bytes) {
    tuning().gs_trace = buf;
    tuning().gs_trace_bytes = buf ? bytes : 0;
    return CFD_OK;
}

int cfd_set_small2d_gs_persistent(int mode) {
    CFD_REQUIRE(mode >= 0 && mode <= 3,
                "small-grid GS persistent mode must be 0 (default), 1 (off), 2 (on) or 3 (on, one exchange per level)");
    const Tuning d = process_defaults();
    tuning().gs_persist = mode ? mode >= 2 : d.gs_persist;
    tuning().gs_pairs = mode >= 2 ? mode == 2 : d.gs_pairs;
    return CFD_OK;
}

int cfd_set_small2d_jacobi_persistent(int on, int sweeps_per_block) {
    CFD_REQUIRE(on >= 0 && on <= 3,
                "small-grid Jacobi persistent: on must be 0 (default), 1 (off), 2 (on) or 3 (on, one exchange per sweep)");
    CFD_REQUIRE(sweeps_per_block == 0 || sweeps_per_block == 4 || sweeps_per_block == 6 || sweeps_per_block == 8 ||
                    sweeps_per_block == 10,
                "small-grid Jacobi persistent: sweeps per block must be 0 (default), 4, 6, 8 or 10");
    const Tuning d = process_defaults();
    tuning().j2_persist = on ? on >= 2 : d.j2_persist;
    tuning().j2p_pairs = on >= 2 ? on == 2 : d.j2p_pairs;
    tuning().j2p_ni = sweeps_per_block ? sweeps_per_block : d.j2p_ni;
    return CFD_OK;
}

int cfd_timing_enable(int enable) {
    g_timing.on = enable != 0;
    g_timing.used = 0;
    g_timing.overflow = false;
    return CFD_OK;
}

int cfd_timing_read(double *ms, long long *sweeps, int reset) {
    return cfd_timing_read_channel(kTimingSolve, ms, sweeps, reset);
}

int cfd_timing_read_channel(int channel, double *ms, long long *sweeps, int reset) {
    CFD_REQUIRE(ms && sweeps, "timing_read: null pointer");
    CFD_REQUIRE(channel == kTimingSolve || channel == kTimingPredictor, "timing_read: channel 0 or 1");
    CFD_REQUIRE(!g_timing.overflow, "timing_read: more than %zu solves were timed without a read",
                Timing::kMaxPairs);
    double total = 0.0;
    long long n = 0;
    for (size_t k = 0; k < g_timing.used; ++k) {
        if (g_timing.channel[k] != channel) continue;
        CFD_CHECK_HIP(hipEventSynchronize(g_timing.stop[k]));
        float t = 0.f;
        CFD_CHECK_HIP(hipEventElapsedTime(&t, g_timing.start[k], g_timing.stop[k]));
        total += t;
        n += g_timing.sweeps[k];
    }
    *ms = total;
    *sweeps = n;
    if (reset) {
        // drop this channel's pairs only: the other channel's unread timings stay
        size_t j = 0;
        for (size_t k = 0; k < g_timing.used; ++k) {
            if (g_timing.channel[k] == channel) continue;
            if (j != k) {
                std::swap(g_timing.start[j], g_timing.start[k]);
                std::swap(g_timing.stop[j], g_timing.stop[k]);
                std::swap(g_timing.sweeps[j], g_timing.sweeps[k]);
                std::swap(g_timing.channel[j], g_timing.channel[k]);
            }
            ++j;
        }
        g_timing.used = j;
        g_timing.overflow = false;
    }
    return CFD_OK;
}
}
