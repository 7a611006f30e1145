// Latency probe (not part of the library): cycles per link of a dependent
// chain in ONE wave on an idle chip -- v_add_f32, v_mul_f32, a DPP wave shift
// (v_mov_dpp wave_shr:1) followed by an add, and an LDS round trip -- to size
// the serial sweep's per-diagonal-step floor.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_chain(float *out, long long *cyc, int n, int kind) {
    float x = threadIdx.x * 1e-3f, y = 1.0000001f;
    __shared__ float sh[64];
    const long long t0 = __builtin_readcyclecounter();
    if (kind == 0) {
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x = x + y;
        }
    } else if (kind == 1) {
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) x = x * y;
        }
    } else if (kind == 2) {
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), 0x138, 0xf, 0xf, false)) + y;
        }
    } else if (kind == 3) {
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                sh[threadIdx.x] = x;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                x = sh[threadIdx.x ^ 1] + y;
            }
        }
    } else {
        // the lexicographic sweep's step: S by DPP, then ((a*(E+W) + b*(N+S)) - d) * c
        float w = x, e = 0.3f, nn = 0.2f, d = 0.1f;
        for (int i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float s = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(nn), __float_as_int(w), 0x138, 0xf, 0xf, false));
                const float a = 0.5f * (e + w);
                const float b = 0.25f * (nn + s);
                w = ((a + b) - d) * 0.7f;
            }
        }
        x = w;
    }
    const long long t1 = __builtin_readcyclecounter();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
    float *o;
    long long *c, h;
    hipMalloc(&o, 256);
    hipMalloc(&c, 8);
    const char *names[] = {"v_add chain", "v_mul chain", "dpp+add chain", "lds round trip + add", "sweep step (dpp + 5 ops)"};
    for (int kind = 0; kind < 5; ++kind) {
        const int n = 2000;
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, o, c, n, kind);
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, o, c, n, kind);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("{\"probe\": \"%s\", \"cycles_per_link\": %.2f}\n", names[kind], (double)h / (8.0 * n));
    }
    return 0;
}
