// internal.hpp -- launchers shared between the library's translation units.
#pragma once
#include "common.hpp"

namespace cfd {
// poisson3d.hip
int launch_fix_faces3d(const float *src, float *dst, const uint8_t *mask, int ny, int nx, int za,
                       int zb, int full_lo, int full_hi, hipStream_t s);
int jacobi3d_sweep(const float *in, float *out, const float *div, const uint8_t *mask, int nz,
                   int ny, int nx, int zb, int ze, float h2, float dt, bool pre, float *resid,
                   hipStream_t s);
int launch_rhs_f32(const float *div, float *rhs, size_t n, float h2, float dt, hipStream_t s);
int jacobi3d_tb_rows();      // configured rows per temporally blocked tile
int jacobi3d_tb_zchunk();
bool jacobi3d_tb_enabled();
int jacobi3d_tb_prefetch();  // planes of prefetch in the blocked kernel (1 or 2)
// jacobi3d_tb.hip
int jacobi3d_tb2_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                      int ze, int fixed_lo, int fixed_hi, float h2, float dt, int W, int zchunk,
                      bool pre, hipStream_t s);
}  // namespace cfd
