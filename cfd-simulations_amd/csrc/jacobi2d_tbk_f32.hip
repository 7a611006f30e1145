// float instantiation of the temporally blocked 2-D Jacobi (jacobi2d_tbk.hpp)
#include "jacobi2d_tbk.hpp"

namespace cfd {
template int jacobi2d_tbk_pass<float, 4>(int, const float *, float *, const float *, const uint8_t *, int,
                                         int, float, float, bool, hipStream_t);
}  // namespace cfd
