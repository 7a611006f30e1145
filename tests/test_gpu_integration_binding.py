"""INTEGRATION.md §B, the binding a reference maintainer pastes into v5.py,
run as written in a fresh interpreter that never imports torch (device
memory from hipMalloc through ctypes), bit-exact against the v5.py fixtures
(tests/integration_binding_check.py).  Reference: v5.py:336-346 (Jacobi
branch of solve_pressure_fast) and v5.py:202-226 (red-black GS)."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.gpu
def test_integration_b_binding_without_torch():
    r = subprocess.run([sys.executable, "-u", str(ROOT / "tests" / "integration_binding_check.py")],
                       capture_output=True, text=True, timeout=110, cwd=str(ROOT))
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "BINDING OK" in r.stdout, out[-4000:]


def test_integration_b_blocks_parse():
    """CPU: §B holds the two blocks the GPU test executes, and they compile."""
    sys.path.insert(0, str(ROOT / "tests"))
    import integration_binding_check as ibc
    jac, gs = ibc.blocks()
    compile(jac, "jacobi", "exec")
    compile(gs, "gs", "exec")
    assert "def solve_pressure_jacobi" in jac and "cfd_jacobi2d_f32" in jac
    assert "def solve_pressure_gauss_seidel" in gs and "cfd_rbgs2d_f32_ws" in gs
