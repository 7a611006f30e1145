// sdma_probe.hip -- measures the pieces of a CU-free slab halo exchange on one
// MI355X before the slab drivers rely on them:
//   A. copy-engine (hipMemcpyDeviceToDeviceNoCU) vs shader (blit) device copies
//      of 4 / 12 / 16 MiB;
//   B. a full-chip, one-workgroup-per-CU streaming kernel alone and with copies
//      running beside it on a second stream (does the copy progress without CUs,
//      and what does it cost the kernel);
//   C. per-op stream overheads between dependent launches: a tiny kernel, a
//      satisfied hipStreamWaitValue32, a 4-byte copy-engine copy, a poll kernel;
//   D. two processes (forked before any HIP call) on the same GPU exchanging
//      IPC handles: each copies a pattern into the other's buffer with the copy
//      engine, then a sequence number into the other's uncached flag word; the
//      receiver's bounded poll kernel waits for the flag, a check kernel counts
//      wrong words.  Round-trip time per ping-pong and any mismatches.
// Every spin is bounded (wall clock) and reports a timeout instead of hanging.
//   hipcc --offload-arch=gfx950 -O2 scripts/sdma_probe.hip -o scripts/sdma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "[%d] %s failed: %s (line %d)\n", (int)getpid(), #x,          \
                    hipGetErrorString(e_), __LINE__);                                     \
            exit(3);                                                                      \
        }                                                                                 \
    } while (0)

static const hipMemcpyKind kNoCU = (hipMemcpyKind)1024;  // hipMemcpyDeviceToDeviceNoCU

// streaming kernel: out = in * 1.0001f + 1, grid-stride, one workgroup per CU
// forced by a large dynamic LDS request
__global__ __launch_bounds__(1024) void k_stream(const float4 *in, float4 *out, size_t n4) {
    extern __shared__ float lds[];
    if (threadIdx.x == 0) lds[0] = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = in[i];
        v.x = v.x * 1.0001f + 1.f;
        v.y = v.y * 1.0001f + 1.f;
        v.z = v.z * 1.0001f + 1.f;
        v.w = v.w * 1.0001f + 1.f;
        out[i] = v;
    }
}

__global__ void k_tiny(int *p) {
    if (threadIdx.x == 0 && p) p[0] += 1;
}

// bounded poll of an uncached flag: status[0] = 1 on timeout
__global__ void k_wait(const unsigned *flag, unsigned want, unsigned *status, unsigned long long limit) {
    if (threadIdx.x == 0) {
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > limit) {
                __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
    }
    __syncthreads();
}

__global__ void k_fill(unsigned *p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v ^ (unsigned)i;
}

__global__ void k_check(const unsigned *p, size_t n, unsigned v, unsigned *bad) {
    unsigned b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += p[i] != (v ^ (unsigned)i);
    if (b) atomicAdd(bad, b);
}

static float ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

static void test_copies() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t big = 64ull << 20;
    char *a, *b;
    CK(hipMalloc(&a, big));
    CK(hipMalloc(&b, big));
    CK(hipMemset(a, 1, big));
    for (size_t mib : {4, 12, 16, 48}) {
        const size_t n = mib << 20;
        for (int kind = 0; kind < 2; ++kind) {
            const hipMemcpyKind k = kind ? kNoCU : hipMemcpyDeviceToDevice;
            for (int w = 0; w < 3; ++w) CK(hipMemcpyAsync(b, a, n, k, s));
            CK(hipEventRecord(e0, s));
            const int reps = 20;
            for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(b, a, n, k, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            const float ms = ms_between(e0, e1) / reps;
            printf("{\"test\": \"copy\", \"kind\": \"%s\", \"mib\": %zu, \"us\": %.1f, \"GBps\": %.1f}\n",
                   kind ? "nocu" : "blit", mib, ms * 1e3, n / (ms * 1e-3) / 1e9);
        }
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipStreamDestroy(s));
}

static void test_overlap() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s, cs;
    CK(hipStreamCreate(&s));
    CK(hipStreamCreate(&cs));
    hipEvent_t k0, k1, c0, c1;
    for (hipEvent_t *e : {&k0, &k1, &c0, &c1}) CK(hipEventCreate(e));
    const size_t n = 1ull << 30;  // 1 GiB in, 1 GiB out
    float *in, *out;
    CK(hipMalloc(&in, n));
    CK(hipMalloc(&out, n));
    CK(hipMemset(in, 0, n));
    const size_t cn = 12ull << 20;
    char *ca, *cb;
    CK(hipMalloc(&ca, cn));
    CK(hipMalloc(&cb, cn));
    const size_t lds = 144 * 1024;
    CK(hipFuncSetAttribute((const void *)k_stream, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    auto kernel = [&](int reps) {
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(k_stream, dim3(ncu), dim3(1024), lds, s, (const float4 *)in, (float4 *)out,
                               n / 16);
        CK(hipGetLastError());
    };
    kernel(3);
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(k0, s));
    kernel(reps);
    CK(hipEventRecord(k1, s));
    CK(hipDeviceSynchronize());
    const float alone = ms_between(k0, k1) / reps;
    printf("{\"test\": \"overlap\", \"what\": \"kernel alone\", \"ms\": %.4f, \"GBps\": %.1f}\n", alone,
           2.0 * n / (alone * 1e-3) / 1e9);
    for (int kind = 0; kind < 2; ++kind) {
        const hipMemcpyKind k = kind ? kNoCU : hipMemcpyDeviceToDevice;
        const int ncopies = 200;
        CK(hipEventRecord(k0, s));
        CK(hipStreamWaitEvent(cs, k0, 0));
        CK(hipEventRecord(c0, cs));
        kernel(reps);
        CK(hipEventRecord(k1, s));
        for (int r = 0; r < ncopies; ++r) CK(hipMemcpyAsync(cb, ca, cn, k, cs));
        CK(hipEventRecord(c1, cs));
        CK(hipDeviceSynchronize());
        const float kms = ms_between(k0, k1) / reps, cms = ms_between(c0, c1);
        printf("{\"test\": \"overlap\", \"what\": \"kernel + %d x 12 MiB %s copies\", \"kernel_ms\": %.4f, "
               "\"kernel_slowdown\": %.4f, \"copies_ms\": %.3f, \"copy_GBps\": %.1f, \"kernels_ms\": %.3f}\n",
               ncopies, kind ? "nocu" : "blit", kms, kms / alone, cms, ncopies * (double)cn / (cms * 1e-3) / 1e9,
               kms * reps);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(ca));
    CK(hipFree(cb));
}

static void test_overheads() {
    hipStream_t s, s2;
    CK(hipStreamCreate(&s));
    CK(hipStreamCreate(&s2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int *ctr;
    CK(hipMalloc(&ctr, 256));
    CK(hipMemset(ctr, 0, 256));
    unsigned *flag, *status;
    CK(hipExtMallocWithFlags((void **)&flag, 256, hipDeviceMallocUncached));
    CK(hipMemset(flag, 0, 256));
    CK(hipMalloc(&status, 256));
    CK(hipMemset(status, 0, 256));
    void *sig = nullptr;
    const bool have_sig = hipExtMallocWithFlags(&sig, 256, hipMallocSignalMemory) == hipSuccess;
    if (have_sig) CK(hipMemset(sig, 0, 8));
    (void)hipGetLastError();
    unsigned *seq;
    CK(hipMalloc(&seq, 4096 * 4));
    unsigned hseq[4096];
    for (int i = 0; i < 4096; ++i) hseq[i] = i + 1;
    CK(hipMemcpy(seq, hseq, sizeof(hseq), hipMemcpyHostToDevice));
    const int reps = 400;
    for (int mode = 0; mode < 6; ++mode) {
        if (mode == 2 && !have_sig) continue;
        CK(hipMemset(flag, 0, 256));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, ctr);
            if (mode == 1) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, ctr);
            if (mode == 2) CK(hipStreamWaitValue32(s, sig, 0, hipStreamWaitValueGte, 0xffffffffu));
            if (mode == 3) CK(hipMemcpyAsync(flag, seq + (r % 4096), 4, kNoCU, s));
            if (mode == 4) hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, 0u, status, 100000000ull);
            if (mode == 5) {  // a flag written on another stream, waited on by a poll kernel
                CK(hipMemcpyAsync(flag, seq + (r % 4096), 4, kNoCU, s2));
                hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, (unsigned)(r + 1), status,
                                   100000000ull);
            }
        }
        CK(hipEventRecord(e1, s));
        CK(hipDeviceSynchronize());
        static const char *names[] = {"tiny kernel", "2 tiny kernels", "tiny + satisfied WaitValue32",
                                      "tiny + 4 B nocu copy", "tiny + satisfied poll kernel",
                                      "tiny + poll kernel on a flag copied from stream 2"};
        printf("{\"test\": \"overhead\", \"what\": \"%s\", \"us_per_rep\": %.2f}\n", names[mode],
               ms_between(e0, e1) * 1e3 / reps);
    }
    unsigned st = 0;
    CK(hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost));
    printf("{\"test\": \"overhead\", \"poll_timeouts\": %u}\n", st);
    if (have_sig) CK(hipFree(sig));
    CK(hipFree(flag));
    CK(hipFree(status));
    CK(hipFree(seq));
    CK(hipFree(ctr));
}

// D: two processes on one GPU
static int rd(int fd, void *p, size_t n) {
    char *c = (char *)p;
    while (n) {
        ssize_t r = read(fd, c, n);
        if (r <= 0) return -1;
        c += r;
        n -= r;
    }
    return 0;
}
static int wr(int fd, const void *p, size_t n) {
    const char *c = (const char *)p;
    while (n) {
        ssize_t r = write(fd, c, n);
        if (r <= 0) return -1;
        c += r;
        n -= r;
    }
    return 0;
}

static int ipc_side(int me, int rfd, int wfd, size_t mib, int rounds, int wv, int split) {
    CK(hipSetDevice(0));
    const size_t n = mib << 20, nw = n / 4;
    unsigned *recv, *send, *flag, *status, *bad, *seq;
    CK(hipMalloc(&recv, n));
    CK(hipMalloc(&send, n));
    CK(hipExtMallocWithFlags((void **)&flag, 4096, hipDeviceMallocUncached));
    CK(hipMemset(flag, 0, 4096));
    CK(hipMalloc(&status, 256));
    CK(hipMemset(status, 0, 256));
    CK(hipMalloc(&bad, 256));
    CK(hipMemset(bad, 0, 256));
    CK(hipMalloc(&seq, 4 * (rounds + 2)));
    {
        unsigned *h = (unsigned *)malloc(4 * (rounds + 2));
        for (int i = 0; i < rounds + 2; ++i) h[i] = i + 1;
        CK(hipMemcpy(seq, h, 4 * (rounds + 2), hipMemcpyHostToDevice));
        free(h);
    }
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t hr, hf, pr, pf;
    CK(hipIpcGetMemHandle(&hr, recv));
    CK(hipIpcGetMemHandle(&hf, flag));
    if (wr(wfd, &hr, sizeof hr) || wr(wfd, &hf, sizeof hf) || rd(rfd, &pr, sizeof pr) || rd(rfd, &pf, sizeof pf)) {
        fprintf(stderr, "[%d] handle exchange failed\n", me);
        return 4;
    }
    unsigned *peer_recv = nullptr, *peer_flag = nullptr;
    CK(hipIpcOpenMemHandle((void **)&peer_recv, pr, hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle((void **)&peer_flag, pf, hipIpcMemLazyEnablePeerAccess));
    hipStream_t s, cs, cs2;
    CK(hipStreamCreate(&s));
    CK(hipStreamCreate(&cs));
    CK(hipStreamCreate(&cs2));
    hipEvent_t e0, e1, ev, ev_sent, ev_half;
    CK(hipEventCreateWithFlags(&ev_half, hipEventDisableTiming));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_sent, hipEventDisableTiming));
    char go = 1;
    // start together
    if (wr(wfd, &go, 1) || rd(rfd, &go, 1)) return 4;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < rounds; ++i) {
        // produce round i's payload (once the last send has read the buffer),
        // send it, then its sequence number
        if (i) CK(hipStreamWaitEvent(s, ev_sent, 0));
        hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, s, send, nw, (unsigned)(i * 2 + me));
        CK(hipEventRecord(ev, s));
        CK(hipStreamWaitEvent(cs, ev, 0));
        if (split) {
            CK(hipStreamWaitEvent(cs2, ev, 0));
            CK(hipMemcpyAsync(peer_recv + nw / 2, send + nw / 2, n / 2, kNoCU, cs2));
            CK(hipEventRecord(ev_half, cs2));
            CK(hipMemcpyAsync(peer_recv, send, n / 2, kNoCU, cs));
            CK(hipStreamWaitEvent(cs, ev_half, 0));
        } else {
            CK(hipMemcpyAsync(peer_recv, send, n, kNoCU, cs));
        }
        if (wv)
            CK(hipStreamWriteValue32(cs, peer_flag, (unsigned)(i + 1), 0));
        else
            CK(hipMemcpyAsync(peer_flag, seq + i, 4, kNoCU, cs));
        CK(hipEventRecord(ev_sent, cs));
        // wait for the peer's round i, check it
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s, flag, (unsigned)(i + 1), status,
                           2000000000ull);
        hipLaunchKernelGGL(k_check, dim3(256), dim3(256), 0, s, recv, nw, (unsigned)(i * 2 + (1 - me)), bad);
        // the peer may overwrite recv only after our check: tell it via the
        // second flag word (the next round's copy waits for it on the peer)
        CK(hipEventRecord(ev, s));
        CK(hipStreamWaitEvent(cs, ev, 0));
        if (wv)
            CK(hipStreamWriteValue32(cs, peer_flag + 16, (unsigned)(i + 1), 0));
        else
            CK(hipMemcpyAsync(peer_flag + 16, seq + i, 4, kNoCU, cs));
        hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, cs, flag + 16, (unsigned)(i + 1), status,
                           2000000000ull);
    }
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(cs));
    CK(hipStreamSynchronize(s));
    unsigned st = 0, b = 0;
    CK(hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&b, bad, 4, hipMemcpyDeviceToHost));
    printf("{\"test\": \"ipc\", \"side\": %d, \"mib\": %zu, \"rounds\": %d, \"flag\": \"%s\", \"split\": %d, "
           "\"us_per_round\": %.1f, \"timeouts\": %u, \"bad_words\": %u}\n",
           me, mib, rounds, wv ? "writevalue" : "nocu copy", split, ms_between(e0, e1) * 1e3 / rounds, st, b);
    fflush(stdout);
    CK(hipIpcCloseMemHandle(peer_recv));
    CK(hipIpcCloseMemHandle(peer_flag));
    return (st || b) ? 5 : 0;
}

// E: copy-engine copies on several streams at once (one engine per stream?)
static void test_multi() {
    const size_t cn = 12ull << 20;
    const int maxs = 8;
    hipStream_t st[maxs];
    char *a[maxs], *b[maxs];
    for (int i = 0; i < maxs; ++i) {
        CK(hipStreamCreate(&st[i]));
        CK(hipMalloc(&a[i], cn));
        CK(hipMalloc(&b[i], cn));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < maxs; ++i) {
        CK(hipMemset(a[i], 1, cn));
        CK(hipMemset(b[i], 2, cn));
        for (int w = 0; w < 3; ++w) CK(hipMemcpyAsync(b[i], a[i], cn, kNoCU, st[i]));
    }
    CK(hipDeviceSynchronize());
    for (int k : {1, 2, 4, 1, 2, 4, 3, 8}) {
        for (size_t chunk : {cn, cn / 2}) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            for (int i = 1; i < k; ++i) CK(hipStreamWaitEvent(st[i], e0, 0));
            const int reps = 10;
            for (int r = 0; r < reps; ++r)
                for (int i = 0; i < k; ++i) CK(hipMemcpyAsync(b[i], a[i], chunk, kNoCU, st[i]));
            for (int i = 1; i < k; ++i) {
                hipEvent_t ei;
                CK(hipEventCreateWithFlags(&ei, hipEventDisableTiming));
                CK(hipEventRecord(ei, st[i]));
                CK(hipStreamWaitEvent(st[0], ei, 0));
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipDeviceSynchronize());
            const float ms = ms_between(e0, e1);
            printf("{\"test\": \"multi\", \"streams\": %d, \"chunk_mib\": %.1f, \"us_per_round\": %.1f, "
                   "\"aggregate_GBps\": %.1f}\n",
                   k, chunk / 1048576.0, ms * 1e3 / reps, (double)k * chunk * reps / (ms * 1e-3) / 1e9);
        }
    }
    // F: hipStreamWriteValue32 as the arrival flag
    unsigned *uflag, *status;
    CK(hipExtMallocWithFlags((void **)&uflag, 256, hipDeviceMallocUncached));
    CK(hipMalloc(&status, 256));
    CK(hipMemset(uflag, 0, 256));
    CK(hipMemset(status, 0, 256));
    CK(hipDeviceSynchronize());
    const int reps = 400;
    for (int mode = 0; mode < 3; ++mode) {
        CK(hipMemset(uflag, 0, 256));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, st[0]));
        for (int r = 0; r < reps; ++r) {
            hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, st[0], (int *)status + 8);
            if (mode == 1) CK(hipStreamWriteValue32(st[0], uflag, r + 1, 0));
            if (mode == 2) {
                CK(hipStreamWriteValue32(st[1], uflag, r + 1, 0));
                hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, st[0], uflag, (unsigned)(r + 1), status,
                                   100000000ull);
            }
        }
        CK(hipEventRecord(e1, st[0]));
        CK(hipDeviceSynchronize());
        static const char *names[] = {"tiny kernel", "tiny + WriteValue32 (uncached)",
                                      "tiny + poll kernel on a WriteValue32 from stream 2"};
        printf("{\"test\": \"writevalue\", \"what\": \"%s\", \"us_per_rep\": %.2f}\n", names[mode],
               ms_between(e0, e1) * 1e3 / reps);
    }
    unsigned stv = 0;
    CK(hipMemcpy(&stv, status, 4, hipMemcpyDeviceToHost));
    printf("{\"test\": \"writevalue\", \"poll_timeouts\": %u}\n", stv);
}

int main(int argc, char **argv) {
    const char *what = argc > 1 ? argv[1] : "all";
    const bool all = !strcmp(what, "all");
    if (all || !strncmp(what, "ipc", 3)) {
        const int wv = strstr(what, "wv") != nullptr, split = strstr(what, "split") != nullptr;
        // fork before any HIP call in this process
        int p2c[2], c2p[2];
        if (pipe(p2c) || pipe(c2p)) return 2;
        fflush(stdout);
        pid_t pid = fork();
        if (pid == 0) {
            close(p2c[1]);
            close(c2p[0]);
            int rc = ipc_side(1, p2c[0], c2p[1], 12, 200, wv, split);
            _exit(rc);
        }
        close(p2c[0]);
        close(c2p[1]);
        int rc = ipc_side(0, c2p[0], p2c[1], 12, 200, wv, split);
        int status = 0;
        waitpid(pid, &status, 0);
        printf("{\"test\": \"ipc\", \"parent_rc\": %d, \"child_status\": %d}\n", rc, status);
        fflush(stdout);
        if (rc || status) return 1;
        if (!all) return 0;
    }
    CK(hipSetDevice(0));
    if (all || !strcmp(what, "copies")) test_copies();
    if (all || !strcmp(what, "overlap")) test_overlap();
    if (all || !strcmp(what, "overheads")) test_overheads();
    if (all || !strcmp(what, "multi")) test_multi();
    return 0;
}
