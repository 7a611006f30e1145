"""ctypes binding of libcfdsim.so, the C ABI declared in include/cfdsim.h.

The library is built in-tree (``make -C cfd-simulations_amd/csrc``, or
``__graft_entry__.build()``).  There is no fallback: if the shared library is
missing, importing this module raises.  ``torch`` is imported first so that
the library's ``libamdhip64.so.7`` / ``librccl.so.1`` dependencies resolve to
the HIP runtime torch already loaded.  That way one HIP runtime owns every
device pointer in the process.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_size_t, c_void_p, c_char_p
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_DIR = Path(__file__).resolve().parent
# CFDSIM_LIB selects another in-tree build of the same ABI (tuning experiments)
LIB_PATH = Path(os.environ.get("CFDSIM_LIB", PKG_DIR / "libcfdsim.so"))
ABI_VERSION = 1

P = c_void_p  # device pointer / stream / opaque handle

# name -> (restype, argtypes); mirrors include/cfdsim.h one-to-one
PROTOTYPES = {
    "cfd_abi_version": (c_int, []),
    "cfd_last_error": (c_char_p, []),
    "cfd_device_arch": (c_char_p, []),
    "cfd_jacobi2d_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_jacobi2d_f64": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_jacobi2d_zero_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_jacobi2d_zero_f64": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_jacobi3d_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_double, c_float, c_int, c_int, P,
                                 P]),
    "cfd_jacobi3d_zero_f32": (c_int, [P, P, P, P, c_int, c_int, c_int, c_double, c_float, c_int, P]),
    "cfd_rbgs_workspace_bytes": (c_size_t, [c_int]),
    "cfd_rbgs2d_workspace_bytes": (c_size_t, [c_int, c_int, c_int]),
    "cfd_rbgs2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_float, c_int, c_double,
                               P, P, P, P]),
    "cfd_rbgs2d_f32_ws": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_float, c_int, c_double,
                                  P, P, c_size_t, P, P]),
    "cfd_rbgs2d_zero_f32_ws": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_float, c_int, c_double,
                                  P, P, c_size_t, P, P]),
    "cfd_rbgs3d_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_double, c_double, c_double, c_float,
                               c_int, c_double, P, P, P, P]),
    "cfd_supg_tau2d_f32": (c_int, [P, P, P, c_float, P, c_int, c_int, c_double, c_double, c_float, P]),
    "cfd_convection_supg2d_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_convection_upwind2d_f32": (c_int, [P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_laplacian2d_f32": (c_int, [P, P, c_float, P, c_int, c_int, c_double, c_double, P]),
    "cfd_predictor2d_f32": (c_int, [P, P, P, c_float, P, P, P, c_int, c_int, c_double, c_double,
                                    c_float, c_int, P]),
    "cfd_set_predictor2d_config": (c_int, [c_int, c_int, c_int]),
    "cfd_set_predictor2d_tau_mode": (c_int, [c_int]),
    "cfd_get_predictor2d_tau_mode": (c_int, []),
    "cfd_get_last_predictor2d_path": (c_int, [ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "cfd_set_persistent_launch": (c_int, [c_int, ctypes.c_longlong]),
    "cfd_persistent_status": (c_int, [P]),
    "cfd_persistent_status_stream": (c_int, [P, P]),
    "cfd_release_thread_resources": (c_int, []),
    "cfd_divergence2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, P, P]),
    "cfd_gradient2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_project2d_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_double, c_float, P, P]),
    "cfd_clean_divergence_workspace_bytes": (c_size_t, [c_int, c_int]),
    "cfd_clean_divergence2d_f32": (c_int, [P, P, c_int, c_int, c_double, c_double, c_int, P, P]),
    "cfd_apply_bc2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_int, P]),
    "cfd_apply_lid_bc2d_f32": (c_int, [P, P, c_int, c_int, c_float, P]),
    "cfd_apply_ibm2d_f32": (c_int, [P, P, P, c_int, c_double, P]),
    "cfd_clip_f32": (c_int, [P, c_size_t, c_float, c_float, P]),
    "cfd_absmax_f32": (c_int, [P, c_size_t, P, P]),
    "cfd_absmax2_f32": (c_int, [P, P, c_size_t, P, P]),
    "cfd_energy_mean2d_f32": (c_int, [P, P, c_size_t, P, P]),
    "cfd_energy_mean_clip2d_f32": (c_int, [P, P, c_size_t, P, c_float, c_float, P]),
    "cfd_apply_bc_ibm2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_int, P, c_double, P]),
    "cfd_vorticity_absmax2d_f32": (c_int, [P, P, P, c_int, c_int, c_double, c_double, P, P]),
    "cfd_vorticity2d_f32": (c_int, [P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_nonfinite_count_f32": (c_int, [P, P, c_size_t, P, P]),
    "cfd_numpy_powf_f32": (c_int, [P, c_float, P, c_size_t, P]),
    "cfd_supg_tau2d_f64": (c_int, [P, P, P, c_double, P, c_int, c_int, c_double, c_double, c_double, P]),
    "cfd_convection_supg2d_f64": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_convection_upwind2d_f64": (c_int, [P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_laplacian2d_f64": (c_int, [P, P, c_double, P, c_int, c_int, c_double, c_double, P]),
    "cfd_predictor2d_f64": (c_int, [P, P, P, c_double, P, P, P, c_int, c_int, c_double, c_double,
                                    c_double, c_int, P]),
    "cfd_divergence2d_f64": (c_int, [P, P, P, c_int, c_int, c_double, c_double, P, P]),
    "cfd_gradient2d_f64": (c_int, [P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_project2d_f64": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_double, c_double, P, P]),
    "cfd_clean_divergence2d_f64": (c_int, [P, P, c_int, c_int, c_double, c_double, c_int, P, P]),
    "cfd_apply_bc2d_f64": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_int, P]),
    "cfd_apply_lid_bc2d_f64": (c_int, [P, P, c_int, c_int, c_double, P]),
    "cfd_apply_ibm2d_f64": (c_int, [P, P, P, c_int, c_double, P]),
    "cfd_clip_f64": (c_int, [P, c_size_t, c_double, c_double, P]),
    "cfd_numpy_pow_f64": (c_int, [P, c_double, P, c_size_t, P]),
    "cfd_absmax2_f64": (c_int, [P, P, c_size_t, P, P]),
    "cfd_energy_mean2d_f64": (c_int, [P, P, c_size_t, P, P]),
    "cfd_energy_mean_clip2d_f64": (c_int, [P, P, c_size_t, P, c_double, c_double, P]),
    "cfd_apply_bc_ibm2d_f64": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_int, P, c_double, P]),
    "cfd_vorticity2d_f64": (c_int, [P, P, P, P, P, c_int, c_int, c_double, c_double, P]),
    "cfd_nonfinite_count_f64": (c_int, [P, P, c_size_t, P, P]),
    "cfd_rbgs2d_f64": (c_int, [P, P, P, c_int, c_int, c_double, c_double, c_float, c_int, c_double, P, P, P]),
    "cfd_comm_unique_id": (c_int, [P, c_size_t]),
    "cfd_comm_init": (c_int, [P, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "cfd_comm_destroy": (c_int, [P]),
    "cfd_comm_init_local": (c_int, [c_int, ctypes.POINTER(c_void_p)]),
    "cfd_comm_init_ipc": (c_int, [c_int, c_int, ctypes.POINTER(c_void_p)]),
    "cfd_comm_ipc_blob_bytes": (c_size_t, []),
    "cfd_comm_ipc_export": (c_int, [P, P, P, c_size_t, P]),
    "cfd_comm_ipc_export_ghost": (c_int, [P, P, P, c_size_t, c_size_t, P]),
    "cfd_comm_ipc_import": (c_int, [P, P, c_int]),
    "cfd_comm_status": (c_int, [P, ctypes.POINTER(c_int)]),
    "cfd_slab_jacobi3d_f32": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_slab_jacobi3d_zero_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                           c_int, c_double, c_float, c_int, c_int, P, P]),
    "cfd_slab_cu_partition": (c_int, [c_int, c_int, P, P, c_int]),
    "cfd_jacobi3d_sweep_f32": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_double,
                                       c_float, P, P]),
    "cfd_slab_rbgs3d_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_double, c_double, c_double, c_float, c_int, c_double, P, P,
                                    c_int, P, P]),
    "cfd_rbgs3d_pass_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_double, c_double, c_double, c_float, c_double, c_int, P, P]),
    "cfd_rbgs_init": (c_int, [P, c_int, c_double, P, P]),
    "cfd_rbgs_finish": (c_int, [P, P, P, c_size_t, P, P]),
    "cfd_set_small2d_gs_iters": (c_int, [c_int, c_int]),
    "cfd_set_small2d_gs_persistent": (c_int, [c_int]),
    "cfd_set_small2d_jacobi_persistent": (c_int, [c_int, c_int]),
    "cfd_set_small2d_gs_trace": (c_int, [P, c_size_t]),
    "cfd_set_tbr_trace": (c_int, [P, c_size_t]),
    "cfd_set_jacobi3d_config": (c_int, [c_int, c_int, c_int]),
    "cfd_set_jacobi3d_blocking": (c_int, [c_int, c_int, c_int]),
    "cfd_get_jacobi3d_levels": (c_int, []),
    "cfd_get_rbgs3d_levels": (c_int, []),
    "cfd_get_jacobi2d_levels": (c_int, []),
    "cfd_set_jacobi3d_prefetch": (c_int, [c_int]),
    "cfd_set_jacobi2d_blocking": (c_int, [c_int]),
    "cfd_set_jacobi2d_staging": (c_int, [c_int]),
    "cfd_get_last_jacobi2d_path": (c_int, [ctypes.POINTER(c_int)]),
    "cfd_reset_tuning": (c_int, []),
    "cfd_get_last_tbr_shape": (c_int, [ctypes.POINTER(c_int)] * 4),
    "cfd_set_small2d_shape": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "cfd_timing_enable": (c_int, [c_int]),
    "cfd_timing_read": (c_int, [ctypes.POINTER(c_double), ctypes.POINTER(ctypes.c_longlong), c_int]),
    "cfd_timing_read_channel": (c_int, [c_int, ctypes.POINTER(c_double), ctypes.POINTER(ctypes.c_longlong), c_int]),
}


class CfdError(RuntimeError):
    """A libcfdsim entry point returned a nonzero status."""


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"{LIB_PATH} is missing: the HIP library was not built. Run "
                "`make -C cfd-simulations_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`."
                " There is no CPU fallback.")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.cfd_abi_version() != ABI_VERSION:
            raise ImportError(f"libcfdsim ABI {L.cfd_abi_version()} != expected {ABI_VERSION}")
        _lib = L
    return _lib


def call(name: str, *args) -> None:
    """Invoke an entry point and raise CfdError on a nonzero status."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().cfd_last_error().decode(errors="replace")
        raise CfdError(f"{name} returned {rc}: {msg}")


def ptr(t) -> int | None:
    """Device pointer of a CUDA/HIP tensor (None passes NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise TypeError("cfd_simulations_amd kernels take device tensors (got a CPU tensor); "
                        "there is no CPU path")
    if not t.is_contiguous():
        raise ValueError("cfd_simulations_amd kernels need C-contiguous tensors")
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream
