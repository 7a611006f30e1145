// capi.hip -- error reporting, identification and sweep timing of libcfdsim.
#include <cstring>
#include <vector>

#include "common.hpp"

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
struct Timing {
    bool on = false;
    std::vector<hipEvent_t> start, stop;
    std::vector<long long> sweeps;
    size_t used = 0;
};
static Timing g_timing;

int timing_begin(hipStream_t s) {
    if (!g_timing.on) return -1;
    if (g_timing.used == g_timing.start.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1;
        g_timing.start.push_back(a);
        g_timing.stop.push_back(b);
        g_timing.sweeps.push_back(0);
    }
    const int k = (int)g_timing.used++;
    if (hipEventRecord(g_timing.start[k], s) != hipSuccess) return -1;
    return k;
}

void timing_end(int k, hipStream_t s, long long sweeps) {
    if (k < 0) return;
    g_timing.sweeps[k] = sweeps;
    (void)hipEventRecord(g_timing.stop[k], s);
}
}  // namespace cfd

using namespace cfd;

extern "C" {
int cfd_abi_version(void) { return CFD_ABI_VERSION; }
const char *cfd_last_error(void) { return cfd::g_err; }
const char *cfd_device_arch(void) { return "gfx950"; }

int cfd_timing_enable(int enable) {
    g_timing.on = enable != 0;
    g_timing.used = 0;
    return CFD_OK;
}

int cfd_timing_read(double *ms, long long *sweeps, int reset) {
    CFD_REQUIRE(ms && sweeps, "timing_read: null pointer");
    double total = 0.0;
    long long n = 0;
    for (size_t k = 0; k < g_timing.used; ++k) {
        CFD_CHECK_HIP(hipEventSynchronize(g_timing.stop[k]));
        float t = 0.f;
        CFD_CHECK_HIP(hipEventElapsedTime(&t, g_timing.start[k], g_timing.stop[k]));
        total += t;
        n += g_timing.sweeps[k];
    }
    *ms = total;
    *sweeps = n;
    if (reset) g_timing.used = 0;
    return CFD_OK;
}
}
