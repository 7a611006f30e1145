"""Slab decomposition of the 3-D Poisson grid across GPUs (one process per GPU).

The reference runs on one node's CPU threads (SURVEY.md section 2,
"Parallelism").  Here the (nz, ny, nx) grid is cut on the slowest axis.  Each
rank holds its owned planes plus G ghost planes per side.  After every pass
the ranks swap boundary planes with their z-neighbours over xGMI -- by default
with the copy engines (SDMA writes into the neighbours' IPC-mapped ghost
planes, no CU taken from the interior), or with RCCL send/recv -- and that swap
overlaps the interior pass.
With G-deep ghosts (G = 2..4) the sweeps run temporally blocked: G sweeps per
pass and one G-plane exchange per pass, 1/G as many messages at the same bytes
per sweep.  Jacobi updates reassociate nothing across planes, so the decomposed
result is bit-identical to the single-GPU one for every rank count.

``SlabPlan`` is pure host logic: ownership, peers, update range and the
exchange list.  The C driver ``cfd_slab_jacobi3d_f32`` executes the same
exchange list: it sends the ``ghost`` owned planes next to each neighbour into
that neighbour's ghost planes (``SlabPlan.exchanges()``).  The CPU tests run
the plan on gloo with world_size 2 and 3.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ._lib import call, lib, ptr, stream_handle

UNIQUE_ID_BYTES = 128


@dataclass(frozen=True)
class SlabPlan:
    """Ownership and halo plan of one rank.  Local arrays hold the owned
    planes plus ``ghost`` planes per side (1..4; G-sweep blocked passes need G):
    local index k <-> global plane z_lo - ghost + k."""
    nz: int        # global planes
    nranks: int
    rank: int
    ghost: int = 1

    def __post_init__(self):
        if not (0 <= self.rank < self.nranks):
            raise ValueError("rank out of range")
        if self.ghost not in (1, 2, 3, 4):
            raise ValueError("ghost depth must be 1..4")
        if self.nz < self.nranks * self.ghost:
            raise ValueError(f"cannot split {self.nz} planes over {self.nranks} ranks "
                             f"with {self.ghost}-deep ghosts")

    @property
    def z_lo(self) -> int:
        """First owned global plane (near-equal split, remainder to low ranks)."""
        q, r = divmod(self.nz, self.nranks)
        return self.rank * q + min(self.rank, r)

    @property
    def z_hi(self) -> int:
        q, r = divmod(self.nz, self.nranks)
        return self.z_lo + q + (1 if self.rank < r else 0)

    @property
    def nz_local(self) -> int:
        return self.z_hi - self.z_lo

    @property
    def nz_total(self) -> int:
        """Planes of the local array, ghosts included."""
        return self.nz_local + 2 * self.ghost

    @property
    def lo_peer(self) -> int:
        return self.rank - 1 if self.rank > 0 else -1

    @property
    def hi_peer(self) -> int:
        return self.rank + 1 if self.rank < self.nranks - 1 else -1

    @property
    def z_update_begin(self) -> int:
        """Local index of the first updated plane (global plane 0 is Dirichlet)."""
        return self.ghost + (1 if self.z_lo == 0 else 0)

    @property
    def z_update_end(self) -> int:
        """Local index one past the last updated plane (global nz-1 is Dirichlet)."""
        return self.ghost + self.nz_local - (1 if self.z_hi == self.nz else 0)

    def exchanges(self):
        """[(send_first_local_plane, count, peer, peer_recv_first_local_plane)]:
        the messages the C driver sends after each pass."""
        g = self.ghost
        out = []
        if self.lo_peer >= 0:
            lo = SlabPlan(self.nz, self.nranks, self.lo_peer, g)
            out.append((g, g, self.lo_peer, lo.nz_local + g))
        if self.hi_peer >= 0:
            out.append((self.nz_local, g, self.hi_peer, 0))
        return out

    def receives(self):
        """[(first_local_ghost_plane, count, peer)]: where the ghosts come from."""
        g = self.ghost
        out = []
        if self.lo_peer >= 0:
            out.append((0, g, self.lo_peer))
        if self.hi_peer >= 0:
            out.append((self.nz_local + g, g, self.hi_peer))
        return out

    def owned(self) -> slice:
        return slice(self.ghost, self.ghost + self.nz_local)

    def scatter(self, glob: np.ndarray) -> np.ndarray:
        """Local (nz_total, ny, nx) copy of a global array; ghost planes outside
        the domain are zero."""
        loc = np.zeros((self.nz_total,) + glob.shape[1:], glob.dtype)
        base = self.z_lo - self.ghost
        for k in range(self.nz_total):
            gz = base + k
            if 0 <= gz < self.nz:
                loc[k] = glob[gz]
        return loc


def comm_unique_id() -> bytes:
    import ctypes
    cbuf = (ctypes.c_char * UNIQUE_ID_BYTES)()
    call("cfd_comm_unique_id", ctypes.addressof(cbuf), UNIQUE_ID_BYTES)
    return bytes(cbuf.raw)


class RcclComm:
    """An RCCL communicator owned by libcfdsim (ncclCommInitRank on the current
    device).  The unique id travels over the torch.distributed process group."""

    def __init__(self, rank: int, nranks: int, group=None):
        import ctypes
        import os
        import torch.distributed as dist
        # RCCL reads this once, at its first communicator: bench.py sets it
        # before the process group; see partition_streams in slab.hip
        os.environ.setdefault("NCCL_MAX_P2P_NCHANNELS", "16")
        if dist.is_available() and dist.is_initialized() and nranks > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) \
                if dist.get_backend(group) == "nccl" else torch.device("cpu")
            t = torch.zeros(UNIQUE_ID_BYTES, dtype=torch.uint8, device=dev)
            if rank == 0:
                t.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(t, src=0, group=group)
            uid = bytes(t.cpu().numpy().tobytes())
        else:
            uid = comm_unique_id()
        cbuf = (ctypes.c_char * UNIQUE_ID_BYTES).from_buffer_copy(uid)
        handle = ctypes.c_void_p()
        call("cfd_comm_init", ctypes.addressof(cbuf), int(nranks), int(rank), ctypes.byref(handle))
        self.handle = handle
        self.rank, self.nranks = rank, nranks

    def close(self):
        if self.handle:
            call("cfd_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CopyEngineComm:
    """Copy-engine slab transport (cfd_comm_init_ipc): no RCCL.  Each rank maps
    its z-neighbours' field buffers through IPC handles and the SDMA engines
    write its boundary planes straight into their ghost planes, so the halo
    exchange takes no CU from the interior launch (see slab.hip).  The handle
    blobs travel over the torch.distributed process group once per pair of
    buffers (``attach``, called by SlabJacobi3D / SlabRBGS3D)."""

    def __init__(self, rank: int, nranks: int, group=None):
        import ctypes
        handle = ctypes.c_void_p()
        call("cfd_comm_init_ipc", int(nranks), int(rank), ctypes.byref(handle))
        self.handle = handle
        self.rank, self.nranks, self.group = rank, nranks, group

    def attach(self, phi: torch.Tensor, phi_tmp: torch.Tensor, ghost_elems: int = 0):
        """Export this rank's two field buffers, gather every rank's blob (a
        collective over the process group), map the neighbours' buffers.  A
        comm holds every pair attached so far (a re-attached pair replaces its
        entry); a solve uses the pair its phi / phi_tmp belong to.
        ghost_elems = ghost planes per side x ny x nx: a pair of 2 GiB or more
        then takes its ghosts through a landing buffer (its allocation cannot
        be IPC-mapped, cfd_comm_ipc_export_ghost)."""
        import ctypes
        if phi.shape != phi_tmp.shape or phi.dtype != torch.float32 or not phi.is_cuda:
            raise ValueError("attach: two float32 device arrays of one shape")
        nb = int(lib().cfd_comm_ipc_blob_bytes())
        blob = (ctypes.c_char * nb)()
        err = None
        try:
            call("cfd_comm_ipc_export_ghost", self.handle, ptr(phi), ptr(phi_tmp), phi.numel(), int(ghost_elems),
                 ctypes.addressof(blob))
        except Exception as e:  # noqa: BLE001 -- every rank learns of it below
            err = e
        self._agree(err, "export")
        mine = bytes(blob.raw)
        if self.nranks > 1:
            import torch.distributed as dist
            blobs = [None] * self.nranks
            dist.all_gather_object(blobs, mine, group=self.group)
        else:
            blobs = [mine]
        allb = (ctypes.c_char * (nb * self.nranks)).from_buffer_copy(b"".join(blobs))
        try:
            call("cfd_comm_ipc_import", self.handle, ctypes.addressof(allb), self.nranks)
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err, "import")

    def _agree(self, err, what):
        """Collective: raise on every rank if `what` failed on any (so that no
        rank is left waiting in the next collective)."""
        ok = err is None
        if self.nranks > 1:
            import torch.distributed as dist
            dev = torch.device("cuda", torch.cuda.current_device()) \
                if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
            ok = bool(t.item())
        if not ok:
            raise RuntimeError(f"copy-engine comm: {what} failed on "
                               f"{'this rank: ' + str(err) if err else 'another rank'}")

    def status(self) -> int:
        """Synchronises the device; raises CfdError if a wait for a neighbour
        timed out (cfd_comm_status)."""
        import ctypes
        t = ctypes.c_int(0)
        call("cfd_comm_status", self.handle, ctypes.byref(t))
        return t.value

    def close(self):
        if self.handle:
            call("cfd_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_comm(rank: int, nranks: int, transport: str = "ce", group=None):
    """The slab transport: "ce" (copy engines over IPC, the default) or "rccl"."""
    if transport == "ce":
        return CopyEngineComm(rank, nranks, group)
    if transport == "rccl":
        return RcclComm(rank, nranks, group)
    raise ValueError(f"unknown slab transport {transport!r}")


class LocalComm:
    """One rank of an in-process slab group (cfd_comm_init_local): N ranks
    driven by N host threads on one GPU, for tests and rehearsals where RCCL
    cannot put several ranks on one device.  Same interface as RcclComm."""

    def __init__(self, handle, rank: int, nranks: int):
        self.handle, self.rank, self.nranks = handle, rank, nranks

    @staticmethod
    def group(nranks: int):
        import ctypes
        arr = (ctypes.c_void_p * nranks)()
        call("cfd_comm_init_local", int(nranks), arr)
        return [LocalComm(ctypes.c_void_p(arr[r]), r, nranks) for r in range(nranks)]

    def close(self):
        if self.handle:
            call("cfd_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SlabJacobi3D:
    """Distributed 7-point Jacobi on this rank's slab (device tensors).  With
    ``plan.ghost == G >= 2`` the sweeps run temporally blocked (up to G per
    pass, one G-plane halo exchange per pass)."""

    def __init__(self, plan: SlabPlan, ny: int, nx: int, h: float, dt, comm: RcclComm | None,
                 device=None, mask=None, rhs_workspace: bool = True):
        self.plan, self.ny, self.nx = plan, ny, nx
        self.h, self.dt = float(h), np.float32(dt)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        shape = (plan.nz_total, ny, nx)
        self.div = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.phi = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.tmp = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.rhs = torch.empty(shape, dtype=torch.float32, device=self.device) if rhs_workspace else None
        self.mask = None if mask is None else mask.to(torch.uint8).contiguous()
        self.comm = comm
        if hasattr(comm, "attach"):
            comm.attach(self.phi, self.tmp, plan.ghost * ny * nx)
        # high priority: its own HW queue (ROCclr pools queues per priority), so
        # the exchange is dispatched beside the interior launch, not behind it
        self.comm_stream = torch.cuda.Stream(device=self.device, priority=-1)

    def solve(self, iters: int, overlap: bool = True, zero_phi: bool = True):
        p = self.plan
        if zero_phi and self.mask is None:
            # phi = zeros (v5.py:337) inside the solve: the first pass starts
            # from the zeros and forms the RHS workspace (cfd_slab_jacobi3d_zero_f32)
            call("cfd_slab_jacobi3d_zero_f32", self.comm.handle, ptr(self.div), ptr(self.phi), ptr(self.tmp),
                 ptr(self.rhs), p.nz_local, p.ghost, self.ny, self.nx, p.lo_peer, p.hi_peer, p.z_update_begin,
                 p.z_update_end, self.h, float(self.dt), int(iters), int(bool(overlap)), stream_handle(),
                 self.comm_stream.cuda_stream)
            return self.phi
        if zero_phi:
            self.phi.zero_()
        call("cfd_slab_jacobi3d_f32", self.comm.handle, ptr(self.div), ptr(self.phi), ptr(self.tmp),
             ptr(self.rhs), ptr(self.mask), p.nz_local, p.ghost, self.ny, self.nx, p.lo_peer, p.hi_peer,
             p.z_update_begin, p.z_update_end, self.h, float(self.dt), int(iters), int(bool(overlap)),
             stream_handle(), self.comm_stream.cuda_stream)
        return self.phi

    def owned(self) -> torch.Tensor:
        return self.phi[self.plan.owned()]


class SlabRBGS3D:
    """Distributed red-black GS (config 5) on this rank's slab: the 3-D
    generalisation of solve_pressure_gauss_seidel_fast (v5.py:202-226) with
    global colours and a global stop rule.  ``plan.ghost == 2`` (and no mask)
    runs one fused pass per iteration; ghost 1 runs in-place colour passes."""

    def __init__(self, plan: SlabPlan, ny: int, nx: int, dx: float, dy: float, dz: float, dt,
                 comm: RcclComm | None, device=None, mask=None):
        self.plan, self.ny, self.nx = plan, ny, nx
        self.dx, self.dy, self.dz, self.dt = float(dx), float(dy), float(dz), np.float32(dt)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        shape = (plan.nz_total, ny, nx)
        self.div = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.phi = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.tmp = torch.zeros(shape, dtype=torch.float32, device=self.device)
        self.mask = None if mask is None else mask.to(torch.uint8).contiguous()
        self.iters_done = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.ws = None
        self.comm = comm
        if hasattr(comm, "attach"):
            comm.attach(self.phi, self.tmp, plan.ghost * ny * nx)
        # high priority: its own HW queue (ROCclr pools queues per priority), so
        # the exchange is dispatched beside the interior launch, not behind it
        self.comm_stream = torch.cuda.Stream(device=self.device, priority=-1)

    @property
    def z_global_offset(self) -> int:
        return self.plan.z_lo - self.plan.ghost

    def solve(self, iterations: int, tolerance: float = 1e-8, overlap: bool = True,
              zero_phi: bool = True):
        need = int(lib().cfd_rbgs_workspace_bytes(int(iterations)))
        if self.ws is None or self.ws.numel() < need:
            self.ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        if zero_phi:
            self.phi.zero_()
        p = self.plan
        call("cfd_slab_rbgs3d_f32", self.comm.handle, ptr(self.div), ptr(self.phi), ptr(self.tmp),
             ptr(self.mask), p.nz_local, p.ghost, self.ny, self.nx, p.lo_peer, p.hi_peer,
             p.z_update_begin, p.z_update_end, self.z_global_offset, self.dx, self.dy, self.dz,
             float(self.dt), int(iterations), float(tolerance), ptr(self.ws), ptr(self.iters_done),
             int(bool(overlap)), stream_handle(), self.comm_stream.cuda_stream)
        return self.phi

    def owned(self) -> torch.Tensor:
        return self.phi[self.plan.owned()]


def sweep_range(phi_in, phi_out, div, mask, z_begin, z_end, h, dt, resid=None):
    """One Jacobi sweep of planes [z_begin, z_end) of a local (nz, ny, nx) array
    (cfd_jacobi3d_sweep_f32, the slab driver's building block)."""
    nz, ny, nx = (int(s) for s in phi_in.shape)
    call("cfd_jacobi3d_sweep_f32", ptr(phi_in), ptr(phi_out), ptr(div),
         ptr(None if mask is None else mask), nz, ny, nx, int(z_begin), int(z_end), float(h),
         float(np.float32(dt)), ptr(resid), stream_handle())


__all__ = ["SlabPlan", "RcclComm", "CopyEngineComm", "make_comm", "LocalComm", "SlabJacobi3D", "SlabRBGS3D", "sweep_range", "comm_unique_id", "lib"]
