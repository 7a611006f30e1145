#!/usr/bin/env python3
"""Runs INTEGRATION.md §B's reference-side binding AS WRITTEN, with no torch.

The two ```python blocks of §B (the hipMalloc-via-ctypes Jacobi drop-in for
v5.py:336-346 and the red-black GS one for v5.py:202-226) are read from
INTEGRATION.md and executed, "/path/to/repo" replaced by this checkout.  The
`self` they are written against is a stand-in carrying the attributes the
reference solver has (config.ny/nx/dx/dy/dt/pressure_iterations/
pressure_tolerance, cylinder_mask, phi).  Results are compared bit for bit
with reference-generated fixtures (tests/golden, made by make_golden.py from
v5.py).  Exits 0 and prints BINDING OK, or raises.  Started by
tests/test_gpu_integration_binding.py in a fresh interpreter."""
import re
import sys
import types
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"


def blocks():
    text = (ROOT / "INTEGRATION.md").read_text()
    sec = text[text.index("## B."):text.index("## C.")]
    b = re.findall(r"```python\n(.*?)```", sec, re.S)
    assert len(b) == 2, f"expected the Jacobi and the GS block in §B, found {len(b)}"
    return [x.replace("/path/to/repo", str(ROOT)) for x in b]


def main():
    jac, gs = blocks()
    g = {"__name__": "integration_b"}
    exec(compile(jac, "INTEGRATION.md §B (Jacobi)", "exec"), g)

    d = np.load(GOLD / "jacobi2d_f32_40x72_it60_cyl.npz", allow_pickle=False)
    ny, nx = d["div"].shape
    cfg = types.SimpleNamespace(ny=ny, nx=nx, dx=float(d["dx"]), dt=d["dt"], pressure_iterations=int(d["iters"]))
    solver = types.SimpleNamespace(config=cfg, cylinder_mask=d["mask"], phi=np.full((ny, nx), 7.0, np.float32))
    phi = g["solve_pressure_jacobi"](solver, d["div"])
    assert phi is solver.phi and np.array_equal(phi, d["phi"]), "Jacobi binding differs from the v5.py fixture"
    print("jacobi2d_f32_40x72_it60_cyl: bit-exact", flush=True)

    for name in ("rbgs2d_f32_64x64_it20_seed7_mask", "rbgs2d_f32_48x80_it15_aniso"):
        f = np.load(GOLD / f"{name}.npz", allow_pickle=False)
        ny, nx = f["div"].shape
        cfg = types.SimpleNamespace(ny=ny, nx=nx, dx=float(f["dx"]), dy=float(f["dy"]), dt=f["dt"],
                                    pressure_iterations=int(f["iters"]), pressure_tolerance=float(f["tol"]))
        # the GS block is module-level code written after the Jacobi block:
        # it sizes its buffers from `cfg` and `n` (bytes of one field)
        g["cfg"], g["n"] = cfg, f["div"].nbytes
        exec(compile(gs, "INTEGRATION.md §B (GS)", "exec"), g)
        dmalloc, h2d, d2h, hip = g["dmalloc"], g["h2d"], g["d2h"], g["hip"]
        phi = np.zeros((ny, nx), np.float32)                     # v5.py:331
        d_phi, d_div, d_mask = dmalloc(phi.nbytes), dmalloc(phi.nbytes), dmalloc(phi.size)
        h2d(d_phi, phi)
        h2d(d_div, f["div"])
        h2d(d_mask, f["mask"].astype(np.uint8))
        g["solve_pressure_gauss_seidel"](types.SimpleNamespace(config=cfg), d_phi, d_div, d_mask)
        d2h(phi, d_phi)
        done = np.zeros(1, np.int32)
        d2h(done, g["d_done"])
        assert np.array_equal(phi, f["phi"]), f"GS binding differs from the v5.py fixture {name}"
        assert 1 <= int(done[0]) <= cfg.pressure_iterations
        for p in (d_phi, d_div, d_mask, g["d_ws"], g["d_tmp"], g["d_done"]):
            hip.hipFree(p)
        print(f"{name}: bit-exact, {int(done[0])} iterations", flush=True)

    assert "torch" not in sys.modules, "the reference-side binding must not need torch"
    print("BINDING OK", flush=True)


if __name__ == "__main__":
    main()
