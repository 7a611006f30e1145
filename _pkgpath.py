"""Import helper for the product package.

The package directory is named ``cfd-simulations_amd`` (after the reference
repository), which is not a valid Python identifier; this registers it as the
importable package ``cfd_simulations_amd``.  Used by bench.py,
__graft_entry__.py and tests/conftest.py.
"""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "cfd-simulations_amd"
NAME = "cfd_simulations_amd"


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(NAME, PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(NAME, None)
        raise
    return mod
