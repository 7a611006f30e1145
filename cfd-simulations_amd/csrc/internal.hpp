// internal.hpp -- launchers shared between the library's translation units.
#pragma once
#include "common.hpp"

namespace cfd {
// Kernel tuning knobs, set through the cfd_set_* entry points.  They are per
// host thread (thread_local): a thread's settings apply to the solves it
// launches and never to another thread's, so concurrent callers (e.g. the
// ranks of an in-process slab group) cannot change each other's kernels.
// Every thread starts from the process defaults (the CFD_* environment knobs,
// read once); cfd_reset_tuning() returns the calling thread to them.
struct Tuning {
    // 3-D single sweep: variant 0 auto / 1 LDS / 2 cache, rows, planes per tile
    int j3_variant = 0, j3_waves = 0, j3_zchunk = 0;
    // 3-D temporal blocking: sweeps per pass (0 auto, 1 off), rows, z-chunk, prefetch
    int tb_steps = 0, tb_rows = 0, tb_zchunk = 0, tb_prefetch = 0;
    // 2-D Jacobi sweeps per pass: 0 auto, 1 off, 2..6, 8, 10, 12
    int j2_blocking = 0;
    // 2-D blocked Jacobi without a mask: rows staged through a per-wave LDS
    // ring this many rows ahead (jacobi2d_tbd: 6 or 4; 0 = register prefetch
    // one row ahead, jacobi2d_tbk, the default: r03 8192^2 f64 0.337 ms per
    // pass against 0.355 (6 ahead) and 0.362 (4 ahead), same box)
    int j2_dma = 0;
    // small-grid 2-D Jacobi: sweeps per launch (1..8), rows per wave, cells per lane
    int j2s_k = 4, j2s_rw = 1, j2s_vec = 1;
    // small-grid 2-D Jacobi (f32) as one persistent launch (jacobi2d_persist)
    // when every tile fits on the chip at once, at most j2p_ni (4, 6, 8, 10)
    // sweeps per block, the levels in pairs per LDS exchange (j2p_pairs); 0 =
    // one launch per j2s_k sweeps
    int j2_persist = 1, j2p_ni = 10;
    bool j2p_pairs = true;
    // small-grid 2-D red-black GS: rows per wave, cells per lane, waves per
    // workgroup, iterations per block (1..5: the persistent solve's, at most
    // that whose tiles fit; the launch-per-block path takes at most 4)
    int gs_rw = 2, gs_vec = 1, gs_wpb = 4, gs_ni = 5;
    // small-grid GS: rows shared in a 16-wave workgroup (rbgs2d_wg) instead of
    // per-wave halo rows (rbgs2d_small).  r02 at 600 x 180, us per iteration
    // by iterations per launch 2 / 3 / 4: shared 3.04 / 2.33 / 1.97; per-wave
    // (2 rows per wave) 2.46 / 2.10 / 2.63, (1 row) 2.54 / 2.33 / 2.24
    int gs_wg = 1;
    // small-grid GS as one persistent launch (rbgs2d_persist) when the caller's
    // workspace holds its exchange rings (cfd_rbgs2d_workspace_bytes) and
    // every tile fits on the chip at once; 0 = one launch per gs_ni iterations
    int gs_persist = 1;
    // persistent GS: one LDS exchange per iteration (each wave also updates
    // the rows on either side of its two at the colour-0 level) instead of
    // one per colour level
    int gs_pairs = 1;
    // diagnostics: per-block timestamps of the persistent GS (4 per tile and
    // block, the 100 MHz clock) into this device buffer when it is big enough
    void *gs_trace = nullptr;
    size_t gs_trace_bytes = 0;
    // diagnostics: the tall-tile kernels' per-wave step timestamps (workgroup
    // 0, 64 steps, 5 marks each, 16 waves' worth: 40 KiB) into this buffer
    void *tbr_trace = nullptr;
    // fused 2-D predictor (cfd_predictor2d_f32 / _f64): 0 auto (the row march
    // whenever the arrays are below 2^31 bytes), 1 one thread per cell, 2 row
    // march; rows per chunk of the row march (0: one resident round, 2..16)
    int pred_variant = 0, pred_rows = 0;
    // row march: preferred cells per lane (0: 2; f32 1, 2, 4; f64 1, 2),
    // halved until nx and every pointer's alignment fit
    int pred_vec = 0;
    // SUPG tau: 0 exact (glibc powf / pow, bit-exact with the reference's
    // NumPy scalars), 1 fast (x*x, correctly rounded sqrt, rcp + Newton
    // divisions: the compiled reference's fastmath arithmetic, within 1e-6)
    int pred_tau = 0;
    // persistent small-grid solves (jacobi2d_persist, rbgs2d_persist): 0 = a
    // plain launch after the occupancy check (r05 default: the cooperative
    // launch cost ~30 us of queue gap per solve, 0.79 -> 0.76 ms per v5
    // cylinder step); 1 = cooperatively (the runtime guarantees every tile
    // co-resident or refuses the launch, which then takes the launch-per-pass
    // path); the bound of a neighbour poll in ticks of the 100 MHz clock
    // (0: 20 s)
    int persist_coop = 0;
    unsigned long long persist_poll = 0;
};
// The failure counter of persistent solves on the current device and stream
// s (a device int, allocated on first use when create): a solve whose poll
// expired adds 1; cfd_persistent_status_stream reads and clears it (and
// cfd_persistent_status every stream's of the device).  nullptr if allocation
// failed (or, without create, if s never had one).
int *persist_fail_word(hipStream_t s, bool create = true);
// k_energy_mean_mb's scratch for the current device and stream s (a zeroed
// counter word + kEnergyBlocks doubles, kept for the process's life); nullptr
// if allocation failed
unsigned *energy_scratch(hipStream_t s);
// Launch a persistent kernel: cooperatively when tuning().persist_coop (0 if
// the runtime refuses the size: every tile could not be co-resident -- the
// error is cleared and the caller takes its launch-per-pass path), else a
// plain launch; in either case ordered after this process's previous
// persistent launch on the device (any stream).  1 = launched; -1 = another
// launch error (set_error done).
int launch_persistent(const void *f, int nblocks, int threads, void *args, hipStream_t s);
// free the calling thread's persistent Jacobi rings (jacobi2d_persist.hip)
void release_thread_rings();
Tuning &tuning();
// the persistent solves' poll bound in effect (tuning().persist_poll, or 20 s)
inline unsigned long long persist_poll_ticks() {
    return tuning().persist_poll ? tuning().persist_poll : 2000000000ull;
}

// jacobi2d_persist.hip: 1 if it ran the solve (phi <- the result; *rc set on
// a HIP error), 0 if the persistent path does not apply
int jacobi2d_persist_solve(float *phi, const float *src, bool pre, const uint8_t *mask, int ny, int nx,
                           float dx2, float dtv, int iterations, hipStream_t s, int *rc, bool zero = false);

// poisson3d.hip
int launch_fix_faces3d(const float *src, float *dst, const uint8_t *mask, int ny, int nx, int za,
                       int zb, int full_lo, int full_hi, hipStream_t s);
int jacobi3d_sweep(const float *in, float *out, const float *div, const uint8_t *mask, int nz,
                   int ny, int nx, int zb, int ze, float h2, float dt, bool pre, float *resid,
                   hipStream_t s);
int launch_rhs_f32(const float *div, float *rhs, size_t n, float h2, float dt, hipStream_t s);
int jacobi3d_tb_zchunk();
bool jacobi3d_tb_enabled();
int jacobi3d_tb_levels();    // Jacobi sweeps per blocked pass (2..4)
// one pass of k = 1..4 sweeps, kernel and tile chosen from the blocking config
int jacobi3d_blocked_pass(int k, const float *in, float *out, const float *src, int nz, int ny,
                          int nx, int zb, int ze, int fixed_lo, int fixed_hi, float h2, float dt,
                          bool pre, hipStream_t s);
int jacobi3d_tb_prefetch();  // planes of prefetch in the blocked kernel (1 or 2)
// jacobi3d_tbr.hip: K = 2..4 sweeps per pass with several rows per wave (tall tiles)
// CUs the tall-tile launches may plan for on this host thread: all of them,
// minus those a slab solve reserved for its exchange stream (set_cu_reserve).
int tbr_cus();
void set_cu_reserve(int n);
int jacobi3d_tbr_pass(int K, int rows, const float *in, float *out, const float *div, int nz,
                      int ny, int nx, int zb, int ze, int fixed_lo, int fixed_hi, float h2,
                      float dt, int zchunk, bool pre, hipStream_t s);
// first pass of a solve: forms the rhs workspace (and starts from phi = 0 when zero)
int jacobi3d_tbr_first_pass(int K, float *out, const float *div, float *rhs_out, const float *in,
                            int nz, int ny, int nx, int zb, int ze, int fixed_lo, int fixed_hi,
                            float h2, float dt, int zchunk, bool zero, hipStream_t s);
// jacobi2d_tbk.hip: one temporally blocked 2-D pass of K sweeps (T, VEC =
// float, 4 / double, 2)
template <typename T, int VEC>
int jacobi2d_tbk_pass(int K, const T *in, T *out, const T *div, const uint8_t *mask, int ny, int nx,
                      T dx2, T dtv, bool pre, hipStream_t s);
// red-black GS workspace (declared below) passes on tall tiles
struct RbgsWs;
struct RbgsConsts;
// (levels half-sweeps from half-sweep h0; rollback = half-sweeps per pass of
// the solve, nhalf = its half-sweeps in all: see jacobi3d_tbr.hip)
int rbgs3d_tbr_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                    int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int h0,
                    int levels, RbgsWs *ws, int rollback, int nhalf, int rows, hipStream_t s,
                    int lag = 0);
// red-black GS workspace (cfd_rbgs_workspace_bytes): flags[0] = iterations,
// flags[1] = iterations done, flags[2] = tolerance (float bits), float
// maxc[iterations] at byte 16, then the small-grid 2-D kernel's 16 slot rows
// of per-iteration maxima (slot-major, folded into maxc after its loop)
struct RbgsWs {
    int flags[4];
    float maxc[1];
};
// poisson2d.hip
int launch_rbgs_init(RbgsWs *ws, int iterations, float tol, int *iters_done, hipStream_t s);
// iterations done (flags[1], *iters_done) from the per-iteration maxima
int launch_rbgs_count(RbgsWs *ws, int *iters_done, hipStream_t s);
// phi <- phi_tmp when ceil(2 done / half_per_pass) is odd, i.e. when the pass
// that completed the last iteration wrote phi_tmp (phi_tmp NULL: nothing)
int launch_rbgs_copy(const RbgsWs *ws, float *phi, const float *phi_tmp, size_t n, int half_per_pass,
                     hipStream_t s);
// after fused (out-of-place) iterations: phi <- phi_tmp when an odd number
// ran, and *iters_done <- the count (both read on device: no host sync)
int launch_rbgs_finish(RbgsWs *ws, float *phi, const float *phi_tmp, size_t n,
                       int *iters_done, hipStream_t s);  // count + copy, one iteration per pass

// rbgs2d_persist.hip: the small-grid 2-D red-black GS as one persistent
// launch.  Bytes of its exchange rings past the base workspace (0 when the
// grid is not a small grid); the solve returns 1 when it ran, 0 when it does
// not apply (too small a workspace, tiles not all resident, knob off), so the
// caller takes the launch-per-block path.
size_t rbgs2d_persist_extra_bytes(int ny, int nx);
int rbgs2d_persist_solve(float *phi, const float *div, const uint8_t *mask, int ny, int nx, float cx,
                         float cy, float cd, float dt_inv, float tol, float *phi_tmp, RbgsWs *ws,
                         size_t ws_bytes, int iterations, int *iters_done, hipStream_t s, int *rc,
                         bool zero = false);
constexpr int kGsSlotRows = 16;  // rbgs2d_small's per-iteration maxima slots
inline size_t rbgs_base_bytes(int iterations) {
    return 16 + sizeof(float) * (size_t)(1 + kGsSlotRows) * (size_t)(iterations > 0 ? iterations : 1);
}

// 3-D red-black GS (poisson3d.hip / jacobi3d_tb.hip)
struct RbgsConsts {
    float cx, cy, cz, cd, dt_inv, tol;
};
RbgsConsts rbgs3d_consts(double dx, double dy, double dz, float dt, double tolerance);
// whether the fused out-of-place pass applies (no mask, float4 layout, blocking on)
bool rbgs3d_fused_ok(const float *phi, const float *phi_tmp, const float *div, const uint8_t *mask,
                     int nx);
// in-place colour pass over planes [z0, z1); local plane 0 = global plane zoff
int rbgs3d_colour_pass(int colour, float *phi, const float *div, const uint8_t *mask, int ny,
                       int nx, int z0, int z1, int zoff, const RbgsConsts &k, RbgsWs *ws, int it,
                       hipStream_t s);
int rbgs3d_iters_per_pass();  // slab solves: 1, or 2 (blocking depth 4)
int rbgs3d_half_per_pass();   // single-GPU solves: half-sweeps per pass, 2..4 (auto 4)
int rbgs3d_fused_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                      int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int it,
                      int iters, RbgsWs *ws, hipStream_t s, int lag = 0);
int rbgs3d_half_pass(const float *in, float *out, const float *div, int nz, int ny, int nx, int zb,
                     int ze, int fixed_lo, int fixed_hi, int zoff, const RbgsConsts &k, int h0,
                     int levels, RbgsWs *ws, hipStream_t s, int lag);
}  // namespace cfd
