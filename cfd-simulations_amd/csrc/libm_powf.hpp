// libm_powf.hpp -- device restatement of glibc's powf (2.35, x86_64), the
// function NumPy calls for a float32 scalar `**` (npy_powf -> powf).
//
// Why: compute_supg_stabilization_fast evaluates |V| as
// `(u[i,j]**2 + v[i,j]**2) ** 0.5` on float32 scalars (v5.py:155).  glibc's
// powf is not correctly rounded: powf(x, 2) differs from x*x on 1 548 806 of
// the 2^32 float inputs (its result is a double approximation with relative
// error ~1.27 * 2^-26, rounded to float), so a correctly rounded u*u cannot
// reproduce the reference bit for bit.  This is the published algorithm of
// glibc's sysdeps/ieee754/flt-32/e_powf.c (from ARM's optimized-routines):
// x = 2^k z, log2(x) = k + log2(c) + log1p(z/c - 1)/ln2 with a 16-entry table
// of (1/c, log2 c) and a degree-5 polynomial; then 2^(y log2 x) = 2^(j/32) *
// 2^r with a 32-entry table and a cubic, all in double, rounded once to float.
// The tables are glibc's __powf_log2_data / __exp2f_data constants.
//
// Verified: the same code compiled for the host (gcc, -ffp-contract=off)
// returns libm's powf bit for bit for every one of the 2^32 float x at
// y = 2 and every non-negative x at y = 0.5 (the two exponents the reference
// uses); the x86_64 FMA variant of libm agrees with the unfused form on all of
// them too.  tests/test_gpu_parity.py checks this device copy against the
// oracle's libm calls.  No multiply-add is fused here (-ffp-contract=off).
//
// Licence: this file restates an algorithm and constant tables published in
// the GNU C Library (glibc, LGPL-2.1-or-later), which took them from Arm's
// optimized-routines (MIT OR Apache-2.0 WITH LLVM-exception); see those
// projects for the upstream licence texts.
#pragma once
#ifdef CFD_LIBM_HOST
#include <cstdint>
#include <cstring>
#include <cmath>
#define CFD_HDF inline
#define CFD_LIBMF_TABLE static
#define CFD_SQRTF(x) std::sqrt(x)
#define CFD_FMAF(a, b, c) std::fma(a, b, c)
#define CFD_FABSF(x) std::fabs(x)
#else
#include "common.hpp"
#define CFD_HDF __device__ inline
#define CFD_LIBMF_TABLE __device__ __constant__
#define CFD_SQRTF(x) __builtin_sqrtf(x)
#define CFD_FMAF(a, b, c) __builtin_fmaf(a, b, c)
#define CFD_FABSF(x) __builtin_fabsf(x)
#endif
// fast-path windows: oracle/powf_window.cpp measure (1.05x the largest error + 4)
#ifndef CFD_POWF_SQ_WIN
#define CFD_POWF_SQ_WIN 952545u
#endif
#ifndef CFD_POWF_SQRT_WIN
#define CFD_POWF_SQRT_WIN 931768u
#endif

namespace cfd {
namespace libm {

CFD_HDF uint32_t asu32f(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return u;
}
CFD_HDF float asf32u(uint32_t u) {
    float x;
    memcpy(&x, &u, 4);
    return x;
}
CFD_HDF uint64_t asu64d(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
CFD_HDF double asf64d(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

// glibc's __powf_log2_data (1/c, log2 c) and __exp2f_data (tab[i] =
// bits(2^(i/32)) - (i << 47)).  A kernel whose slow path should not wait on
// global memory copies them into LDS (PowfTables in __shared__) and passes
// that copy to the *_t forms below.
struct PowfTables {
    double invc[16];
    double logc[16];
    unsigned long long exp2[32];
};
CFD_LIBMF_TABLE const PowfTables kPowfTables = {
    {0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
    0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
    0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
    0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1},
    {-0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
    -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3,  -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
    -0x1.a6f9db6475fcep-5, 0x0p+0,                0x1.338ca9f24f53dp-4,  0x1.476a9543891bap-3,
    0x1.e840b4ac4e4d2p-3,  0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2,  0x1.ce0a44eb17bccp-2},
    {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}};

CFD_HDF bool zeroinfnan(uint32_t i) { return 2u * i - 1u >= 2u * 0x7f800000u - 1u; }
// 0: not an integer, 1: odd integer, 2: even integer
CFD_HDF int checkint(uint32_t iy) {
    const int e = iy >> 23 & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}

// log2(x) for a positive normal(ised) float's bits (POWF_SCALE_BITS = 0 on x86_64)
CFD_HDF double powf_log2(uint32_t ix, const PowfTables &T = kPowfTables) {
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (tmp >> 19) % 16;
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = T.invc[i], logc = T.logc[i];
    const double z = (double)asf32u(iz);
    const double r = z * invc - 1.0;
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double yy = 0x1.27616c9496e0bp-2 * r + -0x1.71969a075c67ap-2;
    const double p = 0x1.ec70a6ca7baddp-2 * r + -0x1.7154748bef6c8p-1;
    const double r4 = r2 * r2;
    double q = 0x1.71547652ab82bp+0 * r + y0;
    q = p * r2 + q;
    yy = yy * r4 + q;
    return yy;
}

// 2^ylogx in double, before the final rounding to float (EXP2F_TABLE_BITS = 5,
// shift 0x1.8p+52 / 32)
CFD_HDF double powf_exp2(double ylogx, uint32_t sign_bias, const PowfTables &T = kPowfTables) {
    double kd = ylogx + 0x1.8p+47;
    const unsigned long long ki = asu64d(kd);
    kd -= 0x1.8p+47;
    const double rr = ylogx - kd;
    unsigned long long t = T.exp2[ki % 32];
    t += (ki + sign_bias) << 47;
    const double s = asf64d(t);
    const double zz = 0x1.c6af84b912394p-5 * rr + 0x1.ebfce50fac4f3p-3;
    const double rr2 = rr * rr;
    double e = 0x1.62e42ff0c52d6p-1 * rr + 1.0;
    e = zz * rr2 + e;
    e = e * s;
    return e;
}

CFD_HDF float powf(float x, float y, const PowfTables &T = kPowfTables) {
    uint32_t sign_bias = 0;
    uint32_t ix = asu32f(x);
    const uint32_t iy = asu32f(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || zeroinfnan(iy)) {
        // x < 0x1p-126, inf or nan; or y is 0, inf or nan
        if (zeroinfnan(iy)) {
            if (2u * iy == 0) return 1.0f;
            if (ix == 0x3f800000u) return 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;  // |x|<1 && y==inf
            return y * y;
        }
        if (zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        if (ix & 0x80000000u) {  // finite x < 0
            const int yint = checkint(iy);
            if (yint == 0) return asf32u(0x7fc00000u);
            if (yint == 1) sign_bias = 1u << 16;  // SIGN_BIAS = 1 << (EXP2F_TABLE_BITS + 11)
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {  // subnormal x: normalise
            ix = asu32f(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double ylogx = (double)y * powf_log2(ix, T);
    if ((asu64d(ylogx) >> 47 & 0xffff) >=
        (asu64d(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -asf32u(0x7f800000u) : asf32u(0x7f800000u);
        if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
    }
    return (float)powf_exp2(ylogx, sign_bias, T);
}

// ---- fast exact paths for the two exponents the reference uses ------------
// glibc's powf forms its result in double and rounds it once to float; that
// double carries an error of at most kPowfSqWin / kPowfSqrtWin units of 2^-29
// of the result's float ulp (oracle/powf_window.cpp measures the maxima over
// EVERY float input, and these windows are 1.05x those + 4).  So the float
// result equals the correctly rounded x*x (or sqrt(x)) unless the exact value
// lies within that window of a rounding midpoint.  The fast paths decide that
// in float arithmetic, with the exact residual of an fma:
//  * x*x: p = x*x rounded, e = fma(x, x, -p) = x^2 - p exactly; the square is
//    clear of the midpoints if |e| < (1/2 - w) ulp(p);
//  * sqrt(s): r = sqrtf(s), e = fma(-r, r, s) = s - r^2 exactly; sqrt(s) =
//    r + e / (2r) (+ a term below 2^-40 ulp), clear if |e| < (1 - 2w) r ulp(r)
//    -- which also proves r correctly rounded, whatever sqrtf's accuracy;
// and any other case (p or s below 2^-100, inf, NaN, s < 0) runs the full
// powf.  A call leaves the fast path with probability ~2w =
// 0.36 % on O(1) inputs.  powf_window.cpp checks powf_sq / powf_sqrt against
// libm's powf for all 2^32 float inputs, bit for bit.
#ifndef CFD_POWF_VSQRT
#define CFD_POWF_VSQRT 1  // device root candidate from v_sqrt_f32 (0: IEEE sqrtf)
#endif
constexpr uint32_t kPowfSqWin = CFD_POWF_SQ_WIN;
constexpr uint32_t kPowfSqrtWin = CFD_POWF_SQRT_WIN;
// (1/2 - w) 2^-23 and (1 - 2w) 2^-23 with w = window / 2^29
constexpr float kPowfSqT = (float)((0.5 - (double)CFD_POWF_SQ_WIN / 536870912.0) * 0x1p-23);
constexpr float kPowfSqrtT = (float)((1.0 - 2.0 * (double)CFD_POWF_SQRT_WIN / 536870912.0) * 0x1p-23);

// p = x*x rounded; true when p is glibc's powf(x, 2).  The window is taken
// in the ulp of the binade below p's last bit (exponent of bits(p) - 1): for
// p = 2^k that is the lower binade, whose midpoints are the nearer ones when
// the exact square lies below p; for every other p it is p's own ulp.
CFD_HDF bool powf_sq_fast(float x, float &p) {
    p = x * x;
    const float e = CFD_FMAF(x, x, -p);
    const float t = asf32u((asu32f(p) - 1u) & 0x7f800000u) * kPowfSqT;
    // p >= 2^-100 keeps e exact (no underflow); inf / NaN fail the compare.
    // x = +-0: glibc returns x * x = +0 (its zero branch), as p is
    // (bitwise, not short-circuit: the compiler keeps the test branch-free)
    return ((p >= 0x1p-100f) & (CFD_FABSF(e) < t)) | (x == 0.0f);
}
// r = sqrt(s) rounded; true when r is glibc's powf(s, 0.5) (the window in
// the ulp below r's last bit, as above)
CFD_HDF bool powf_sqrt_fast(float s, float &r) {
#if CFD_POWF_VSQRT && defined(__HIP_DEVICE_COMPILE__)
    // the raw v_sqrt_f32 (within an ulp; not the IEEE root on ~15 % of
    // inputs) moved to the nearest float by its residual: ~12 instructions
    // against the IEEE sqrtf expansion's ~17; the proof test below decides,
    // whatever this candidate is (r04: 0.397 against 0.41 ms per 8192^2
    // predictor launch)
    const float r0 = __builtin_amdgcn_sqrtf(s);
    const float e0 = CFD_FMAF(-r0, r0, s);
    const float h = r0 * (asf32u((asu32f(r0) - 1u) & 0x7f800000u) * 0x1p-23f);  // r0 ulp(r0)
    const uint32_t b0 = asu32f(r0);
    r = asf32u(e0 > h ? b0 + 1u : (e0 < -h ? b0 - 1u : b0));
#else
    r = CFD_SQRTF(s);
#endif
    const float e = CFD_FMAF(-r, r, s);
    const float t = r * (asf32u((asu32f(r) - 1u) & 0x7f800000u) * kPowfSqrtT);
    // s >= 2^-100 keeps e exact; s < 0, inf or NaN fail the compare.
    // s = +0: glibc returns +0 (its zero branch: x * x), as r is (not s = -0:
    // sqrtf(-0) = -0)
    return ((s >= 0x1p-100f) & (CFD_FABSF(e) < t)) | (asu32f(s) == 0u);
}

// NumPy float32 scalar x**2, bit for bit (glibc powf(x, 2.0f))
CFD_HDF float powf_sq(float x, const PowfTables &T = kPowfTables) {
    float p;
    if (powf_sq_fast(x, p)) return p;
    return powf(x, 2.0f, T);
}

// NumPy float32 scalar x**0.5, bit for bit (glibc powf(x, 0.5f))
CFD_HDF float powf_sqrt(float x, const PowfTables &T = kPowfTables) {
    float r;
    if (powf_sqrt_fast(x, r)) return r;
    return powf(x, 0.5f, T);
}

}  // namespace libm
}  // namespace cfd
