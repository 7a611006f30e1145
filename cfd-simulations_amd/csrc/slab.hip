// slab.hip -- multi-GPU slab decomposition of the 3-D Jacobi sweep.
//
// One process per GPU.  The (nz, ny, nx) grid is cut on z; each rank's local
// array is (nz_local + 2, ny, nx) with one ghost plane per side.  After every
// sweep the two owned boundary planes go to the z-neighbours with RCCL
// send/recv (point-to-point over xGMI: one direct link per neighbour pair).
// With overlap on, the boundary planes are swept first, their exchange runs on
// a second HIP stream, and the interior planes sweep concurrently on the main
// stream; the main stream waits on the exchange before the next sweep.  The
// decomposition is exact: every cell sees the same neighbour values as in the
// single-GPU sweep, so results are bit-identical for any rank count.
//
// The exchange plan (peers, which planes are updated) is computed on the host
// (SlabPlan in the Python package) and tested there on CPU with gloo.
#include <rccl/rccl.h>

#include "common.hpp"

namespace cfd {
int launch_fix_faces3d(const float *src, float *dst, const uint8_t *mask, int ny, int nx, int za,
                       int zb, int full_lo, int full_hi, hipStream_t s);

struct SlabComm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    hipEvent_t ev_boundary = nullptr, ev_comm = nullptr;
};

#define CFD_CHECK_NCCL(expr)                                                              \
    do {                                                                                  \
        ncclResult_t _r = (expr);                                                         \
        if (_r != ncclSuccess) {                                                          \
            ::cfd::set_error("%s failed: %s (%s:%d)", #expr, ncclGetErrorString(_r),       \
                             __FILE__, __LINE__);                                         \
            return CFD_E_COMM;                                                            \
        }                                                                                 \
    } while (0)

// ghost exchange of array `a` (local planes 0..nzl+1)
static int exchange(SlabComm *c, float *a, int nzl, size_t plane, int lo, int hi, hipStream_t s) {
    if (lo < 0 && hi < 0) return CFD_OK;
    CFD_CHECK_NCCL(ncclGroupStart());
    if (lo >= 0) {
        CFD_CHECK_NCCL(ncclSend(a + plane, plane, ncclFloat32, lo, c->comm, s));
        CFD_CHECK_NCCL(ncclRecv(a, plane, ncclFloat32, lo, c->comm, s));
    }
    if (hi >= 0) {
        CFD_CHECK_NCCL(ncclSend(a + (size_t)nzl * plane, plane, ncclFloat32, hi, c->comm, s));
        CFD_CHECK_NCCL(ncclRecv(a + (size_t)(nzl + 1) * plane, plane, ncclFloat32, hi, c->comm, s));
    }
    CFD_CHECK_NCCL(ncclGroupEnd());
    return CFD_OK;
}

}  // namespace cfd

using namespace cfd;

extern "C" {

int cfd_jacobi3d_sweep_f32(const float *in, float *out, const float *div, const uint8_t *mask,
                           int nz, int ny, int nx, int z_begin, int z_end, double h, float dt,
                           float *resid, void *stream);

int cfd_comm_unique_id(void *out, size_t bytes) {
    CFD_REQUIRE(out && bytes >= sizeof(ncclUniqueId), "comm_unique_id: need %zu bytes",
                sizeof(ncclUniqueId));
    ncclUniqueId id;
    CFD_CHECK_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof(id));
    return CFD_OK;
}

int cfd_comm_init(const void *unique_id, int nranks, int rank, void **comm) {
    CFD_REQUIRE(unique_id && comm && nranks >= 1 && rank >= 0 && rank < nranks,
                "comm_init: bad arguments");
    SlabComm *c = new SlabComm();
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank failed: %s", ncclGetErrorString(r));
        delete c;
        return CFD_E_COMM;
    }
    if (hipEventCreateWithFlags(&c->ev_boundary, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming) != hipSuccess) {
        set_error("comm_init: hipEventCreate failed");
        ncclCommDestroy(c->comm);
        delete c;
        return CFD_E_HIP;
    }
    *comm = c;
    return CFD_OK;
}

int cfd_comm_destroy(void *comm) {
    if (!comm) return CFD_OK;
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    if (c->ev_boundary) (void)hipEventDestroy(c->ev_boundary);
    if (c->ev_comm) (void)hipEventDestroy(c->ev_comm);
    ncclResult_t r = c->comm ? ncclCommDestroy(c->comm) : ncclSuccess;
    delete c;
    if (r != ncclSuccess) {
        set_error("ncclCommDestroy failed: %s", ncclGetErrorString(r));
        return CFD_E_COMM;
    }
    return CFD_OK;
}

int cfd_slab_jacobi3d_f32(void *comm, const float *div, float *phi, float *phi_tmp,
                          const uint8_t *mask, int nz_local, int ny, int nx, int lo_peer,
                          int hi_peer, int z_update_begin, int z_update_end, double h, float dt,
                          int iters, int overlap, void *stream, void *comm_stream) {
    SlabComm *c = reinterpret_cast<SlabComm *>(comm);
    CFD_REQUIRE(c && div && phi && phi_tmp, "slab_jacobi3d: null pointer");
    CFD_REQUIRE(nz_local >= 1 && ny >= 1 && nx >= 1 && iters >= 0, "slab_jacobi3d: bad shape");
    CFD_REQUIRE(z_update_begin >= 1 && z_update_end <= nz_local + 1 &&
                    z_update_begin <= z_update_end,
                "slab_jacobi3d: update range [%d,%d) outside owned planes 1..%d", z_update_begin,
                z_update_end, nz_local);
    CFD_REQUIRE(lo_peer < c->nranks && hi_peer < c->nranks, "slab_jacobi3d: bad peer");
    if (iters == 0) return CFD_OK;
    hipStream_t s = as_stream(stream);
    hipStream_t cs = comm_stream ? as_stream(comm_stream) : s;
    const int nzt = nz_local + 2;
    const size_t plane = (size_t)ny * nx;
    int rc;
    // Dirichlet faces of the owned planes: rows y=0, ny-1, and the global
    // boundary planes (owned planes outside the update range) in full.  Ghost
    // planes arrive whole from the neighbours (their face rows are never read).
    const int full_lo = z_update_begin > 1 ? 1 : -1;
    const int full_hi = z_update_end < nz_local + 1 ? nz_local : -1;
    if ((rc = launch_fix_faces3d(phi, phi_tmp, mask, ny, nx, 1, nz_local + 1, full_lo, full_hi, s)))
        return rc;
    // ghosts of the initial guess
    if ((rc = exchange(c, phi, nz_local, plane, lo_peer, hi_peer, s))) return rc;
    const float h2f = (float)(h * h);
    (void)h2f;
    const int zb = z_update_begin, ze = z_update_end;
    // planes whose values a neighbour needs next sweep
    const bool lo_b = lo_peer >= 0 && zb == 1;
    const bool hi_b = hi_peer >= 0 && ze == nz_local + 1;
    float *a = phi, *b = phi_tmp;
    const int tk = timing_begin(s);
    for (int it = 0; it < iters; ++it) {
        if (!overlap || c->nranks == 1) {
            if ((rc = cfd_jacobi3d_sweep_f32(a, b, div, mask, nzt, ny, nx, zb, ze, h, dt, nullptr, s)))
                return rc;
            if ((rc = exchange(c, b, nz_local, plane, lo_peer, hi_peer, s))) return rc;
        } else {
            int ib = zb, ie = ze;  // interior range after peeling boundary planes
            if (lo_b && ib < ie) {
                if ((rc = cfd_jacobi3d_sweep_f32(a, b, div, mask, nzt, ny, nx, 1, 2, h, dt, nullptr, s)))
                    return rc;
                ib = 2;
            }
            if (hi_b && ib < ie) {
                if ((rc = cfd_jacobi3d_sweep_f32(a, b, div, mask, nzt, ny, nx, ie - 1, ie, h, dt,
                                                 nullptr, s)))
                    return rc;
                ie -= 1;
            }
            CFD_CHECK_HIP(hipEventRecord(c->ev_boundary, s));
            CFD_CHECK_HIP(hipStreamWaitEvent(cs, c->ev_boundary, 0));
            if ((rc = exchange(c, b, nz_local, plane, lo_peer, hi_peer, cs))) return rc;
            CFD_CHECK_HIP(hipEventRecord(c->ev_comm, cs));
            if (ib < ie &&
                (rc = cfd_jacobi3d_sweep_f32(a, b, div, mask, nzt, ny, nx, ib, ie, h, dt, nullptr, s)))
                return rc;
            CFD_CHECK_HIP(hipStreamWaitEvent(s, c->ev_comm, 0));
        }
        // after sweep 1, the other buffer gets the final owned faces too
        if (it == 0 && iters > 1 &&
            (rc = launch_fix_faces3d(phi_tmp, phi, nullptr, ny, nx, 1, nz_local + 1, full_lo, full_hi, s)))
            return rc;
        float *t = a;
        a = b;
        b = t;
    }
    timing_end(tk, s, iters);
    if (a != phi)
        CFD_CHECK_HIP(hipMemcpyAsync(phi, a, sizeof(float) * plane * nzt, hipMemcpyDeviceToDevice, s));
    return CFD_OK;
}

}  // extern "C"
