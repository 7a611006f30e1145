"""Shared test setup.

* registers the ``gpu`` marker (tests that need an MI355X and libcfdsim.so);
* makes the repo root importable (``oracle``, ``_pkgpath``) and registers the
  product package ``cfd-simulations_amd`` as ``cfd_simulations_amd``.
"""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import _pkgpath  # noqa: E402

_pkgpath.load()

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU and the built HIP library")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load


def rel_linf(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    return float(np.abs(a - b).max() / scale)
