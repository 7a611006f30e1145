// stencil2d.hpp -- device helpers shared by the 2-D stencil translation units
// (poisson2d.hip, jacobi2d_tbk.hip): vector loads / stores of VEC cells and the
// 5-point Jacobi update in the reference's operation order.
#pragma once
#include <utility>

#include "internal.hpp"

namespace cfd {

template <typename T, int VEC>
struct VecOf {
    typedef T type __attribute__((ext_vector_type(VEC)));
};
template <typename T>
struct VecOf<T, 1> {
    using type = T;
};

template <typename T, int VEC>
__device__ inline void ld(const T *p, T (&r)[VEC]) {
    if constexpr (VEC == 1) {
        r[0] = p[0];
    } else {
        typename VecOf<T, VEC>::type v = *reinterpret_cast<const typename VecOf<T, VEC>::type *>(p);
#pragma unroll
        for (int k = 0; k < VEC; ++k) r[k] = v[k];
    }
}
template <typename T, int VEC>
__device__ inline void st(T *p, const T (&r)[VEC]) {
    if constexpr (VEC == 1) {
        p[0] = r[0];
    } else {
        typename VecOf<T, VEC>::type v;
#pragma unroll
        for (int k = 0; k < VEC; ++k) v[k] = r[k];
        *reinterpret_cast<typename VecOf<T, VEC>::type *>(p) = v;
    }
}

// v5.py:341-345: ((E + W + N + S) - f32(dx**2) * div / dt) * 0.25, left to
// right, no contraction; PRE: `d` is the precomputed rhs (the same bits).
template <typename T>
__device__ inline T jac5(T E, T W, T N, T S, T d, T dx2, T dtv, bool pre) {
    T s = E + W;
    s = s + N;
    s = s + S;
    const T rhs = pre ? d : (dx2 * d) / dtv;
    return T(0.25) * (s - rhs);
}

}  // namespace cfd
