"""The C-ABI library loads and exports every symbol include/cfdsim.h declares
(CPU only: no compute calls without a GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

from cfd_simulations_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "cfdsim.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(cfd_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_abi():
    names = declared_functions()
    assert "cfd_jacobi3d_f32" in names and "cfd_slab_jacobi3d_f32" in names
    assert len(names) >= 30


def test_bindings_cover_header_exactly():
    assert sorted(_lib.PROTOTYPES) == declared_functions()


def test_library_exports_every_symbol():
    if not _lib.LIB_PATH.exists():
        pytest.fail(f"{_lib.LIB_PATH} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_library_identifies_itself():
    L = _lib.lib()
    assert L.cfd_abi_version() == _lib.ABI_VERSION
    assert L.cfd_device_arch() == b"gfx950"
    assert L.cfd_rbgs_workspace_bytes(1500) >= 4 * 1500
    # two row-major float64 fields, or three float32 fields (div, phi1, phi2)
    # in the skewed layout of the f32 sweep (64-row blocks x ceil((nx + 63) / 4)
    # groups of 4 diagonals x 64 rows x 4), the larger
    def skew(ny, nx):  # + 8 B of progress word per block, 256-B aligned (the multi-CU sweep)
        nb = (ny - 2 + 63) // 64
        return (3 * 4 * nb * ((nx + 63 + 3) // 4) * 256 + 255) // 256 * 256 + 8 * nb
    assert L.cfd_clean_divergence_workspace_bytes(180, 600) == 2 * 8 * 180 * 600
    assert L.cfd_clean_divergence_workspace_bytes(3, 64) == skew(3, 64) == 98304 + 8
    assert L.cfd_clean_divergence_workspace_bytes(67, 3) == skew(67, 3)
    assert L.cfd_clean_divergence_workspace_bytes(2, 5000) == 2 * 8 * 2 * 5000


def test_invalid_arguments_report_errors_without_gpu():
    """Argument validation runs before any device work."""
    with pytest.raises(_lib.CfdError, match="null"):
        _lib.call("cfd_jacobi2d_f32", None, None, None, None, None, 8, 8, 0.1, 1.0, 1, 0, None, None)
    with pytest.raises(_lib.CfdError, match="waves"):
        _lib.call("cfd_set_jacobi3d_config", 1, 3, 0)


def test_device_arch_of_code_object():
    """The fat binary carries a gfx950 code object."""
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data


@pytest.mark.parametrize("ncu,reserve", [(256, 8), (256, 16), (256, 24), (256, 32), (512, 16), (64, 8)])
def test_slab_cu_partition_spreads_reserve_over_xcds(ncu, reserve):
    """The exchange CUs of a partitioned slab solve (cfd_slab_cu_partition,
    host only): disjoint from the compute CUs, together all CUs, reserve/8 on
    each of the 8 XCDs whether mask bit b maps to XCD b // (ncu/8) or b % 8."""
    import numpy as np
    words = (ncu + 31) // 32
    cm = (ctypes.c_uint32 * words)()
    xm = (ctypes.c_uint32 * words)()
    _lib.call("cfd_slab_cu_partition", ncu, reserve, ctypes.addressof(cm), ctypes.addressof(xm), words)

    def bits(m):
        return np.array([(m[b // 32] >> (b % 32)) & 1 for b in range(ncu)], dtype=bool)

    c, x = bits(cm), bits(xm)
    assert x.sum() == reserve and c.sum() == ncu - reserve
    assert not (c & x).any() and (c | x).all()
    b = np.nonzero(x)[0]
    for xcd in (b // (ncu // 8), b % 8):
        assert np.bincount(xcd, minlength=8).tolist() == [reserve // 8] * 8


@pytest.mark.parametrize("ncu,reserve", [(256, 0), (256, 12), (256, 40), (100, 8)])
def test_slab_cu_partition_rejects_unbalanced_requests(ncu, reserve):
    words = (ncu + 31) // 32
    cm = (ctypes.c_uint32 * words)()
    xm = (ctypes.c_uint32 * words)()
    with pytest.raises(_lib.CfdError, match="slab_cu_partition"):
        _lib.call("cfd_slab_cu_partition", ncu, reserve, ctypes.addressof(cm), ctypes.addressof(xm), words)


def test_tuning_knobs_are_per_thread():
    """cfd_set_* changes only the calling thread's kernels (thread_local
    tuning): another thread keeps the defaults, and cfd_reset_tuning restores
    them (host-only calls, no GPU)."""
    import threading
    L = _lib.lib()
    _lib.call("cfd_reset_tuning")
    base3, base2 = L.cfd_get_jacobi3d_levels(), L.cfd_get_jacobi2d_levels()
    _lib.call("cfd_set_jacobi3d_blocking", 4, 0, 0)
    _lib.call("cfd_set_jacobi2d_blocking", 5)
    seen = {}

    def other():
        seen["j3"], seen["j2"] = L.cfd_get_jacobi3d_levels(), L.cfd_get_jacobi2d_levels()
        _lib.call("cfd_set_jacobi3d_blocking", 2, 0, 0)  # must not leak back

    t = threading.Thread(target=other)
    t.start()
    t.join()
    try:
        assert seen == {"j3": base3, "j2": base2}
        assert L.cfd_get_jacobi3d_levels() == 4 and L.cfd_get_jacobi2d_levels() == 5
    finally:
        _lib.call("cfd_reset_tuning")
    assert (L.cfd_get_jacobi3d_levels(), L.cfd_get_jacobi2d_levels()) == (base3, base2)


@pytest.mark.parametrize("args", [(9, 0, 0, 0, 0, 0), (-1, 0, 0, 0, 0, 0), (0, 3, 0, 0, 0, 0), (0, 0, 2, 0, 0, 0),
                                  (0, 0, 0, 0, 3, 0), (0, 0, 0, 0, 0, 8)])
def test_small2d_shape_validated(args):
    """Out-of-range small-grid shapes are rejected (the r01 env knob took any
    K and could count sweeps it never ran)."""
    with pytest.raises(_lib.CfdError, match="small-grid"):
        _lib.call("cfd_set_small2d_shape", *args)
