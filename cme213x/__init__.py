"""Importable alias for the ``2012-04_stanford_cme213_amd`` package.

The package directory name is not a Python identifier, so it is imported by
path once and every one of its modules is registered under ``cme213x.*`` too
(one module object per file, no duplicates).
"""
import importlib
import sys
from pathlib import Path

_REAL = "2012-04_stanford_cme213_amd"
_root = str(Path(__file__).resolve().parent.parent)
if _root not in sys.path:
    sys.path.insert(0, _root)

_pkg = importlib.import_module(_REAL)


def _alias_all() -> None:
    for name, mod in list(sys.modules.items()):
        if name == _REAL or name.startswith(_REAL + "."):
            sys.modules["cme213x" + name[len(_REAL):]] = mod


_alias_all()
_pkg._alias_all = _alias_all  # drivers call this after lazy imports
