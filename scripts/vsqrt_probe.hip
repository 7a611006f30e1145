// vsqrt_probe.hip -- how often the raw v_sqrt_f32 (__builtin_amdgcn_sqrtf) and
// a v_rcp_f32-based division with one Newton step differ from the correctly
// rounded sqrtf / division on O(1) inputs (tuning aid for the predictor's
// fast paths; prints the counts).
//   hipcc -O3 --offload-arch=gfx950 scripts/vsqrt_probe.hip -o /tmp/vsqrt_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned long long *cnt, unsigned n) {
    unsigned long long a = 0, b = 0, c = 0;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        // s spread over [0.25, 16): mantissa from the index hash
        unsigned h = i * 2654435761u;
        float s = __uint_as_float(0x3e800000u + (h % (6u << 23)));
        float r0 = __builtin_amdgcn_sqrtf(s), r1 = __builtin_sqrtf(s);
        a += r0 != r1;
        float d = __uint_as_float(0x3f000000u + ((h >> 3) % (3u << 23)));
        float rc = __builtin_amdgcn_rcpf(d);
        float q0 = s * rc;
        float q1 = __builtin_fmaf(__builtin_fmaf(-q0, d, s), rc, q0);
        b += q1 != s / d;
        c += q0 != s / d;
    }
    atomicAdd(cnt, a);
    atomicAdd(cnt + 1, b);
    atomicAdd(cnt + 2, c);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 24);
    hipMemset(d, 0, 24);
    const unsigned n = 1u << 26;
    hipLaunchKernelGGL(probe, dim3(1024), dim3(256), 0, 0, d, n);
    unsigned long long h[3];
    hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    printf("of %u: v_sqrt_f32 != sqrtf: %llu (%.4f%%); rcp+newton div != IEEE div: %llu (%.5f%%); a*rcp != div: %llu (%.3f%%)\n",
           n, h[0], 100.0 * h[0] / n, h[1], 100.0 * h[1] / n, h[2], 100.0 * h[2] / n);
    return 0;
}
