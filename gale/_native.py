"""Loader for the in-tree native library ``gale/_C.so`` (built by ``make``).

torch is imported first so that the process has exactly one HIP runtime: torch ships its own
``libamdhip64.so.7`` and ``_C.so`` resolves to the already-loaded copy by SONAME.
"""

from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


def native():
    """Return the ``gale._C`` extension module, raising a clear error if it is not built."""
    global _mod, _err
    if _mod is not None:
        return _mod
    try:
        import torch  # noqa: F401  (single HIP runtime, see module docstring)

        _mod = importlib.import_module("gale._C")
        return _mod
    except ImportError as e:  # pragma: no cover - exercised only when unbuilt
        _err = e
        here = os.path.dirname(os.path.abspath(__file__))
        raise ImportError(
            f"gale native library not built ({e}); run `make -C {os.path.dirname(here)}`"
        ) from e


def native_available() -> bool:
    try:
        native()
        return True
    except ImportError:
        return False
