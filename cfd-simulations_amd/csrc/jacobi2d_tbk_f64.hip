// double instantiation of the temporally blocked 2-D Jacobi (jacobi2d_tbk.hpp)
#include "jacobi2d_tbk.hpp"

namespace cfd {
template int jacobi2d_tbk_pass<double, 2>(int, const double *, double *, const double *, const uint8_t *,
                                          int, int, double, double, bool, hipStream_t);
}  // namespace cfd
