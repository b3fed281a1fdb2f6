"""Loader for the in-tree native extension (``pytorch_distributed_tutorials_amd/_C*.so``).

The extension is built by ``build_native.py`` (or ``__graft_entry__.build()``)
with hipcc for gfx950 and lives next to this package, so it travels with the
repo snapshot to the GPU box.  On a GPU, every op in ``ops/`` dispatches to it
and FAILS LOUDLY when it is missing -- there is no silent eager fallback for
device tensors.  CPU tensors use the PyTorch reference implementations (tests).
"""
from __future__ import annotations

import importlib
import importlib.util as importlib_util
import os
from typing import Any, Optional

_C: Optional[Any] = None
_ERR: Optional[BaseException] = None
_LOADED = False


def _load() -> None:
    global _C, _ERR, _LOADED
    if _LOADED:
        return
    _LOADED = True
    if os.environ.get("PDT_DISABLE_NATIVE", "0") == "1":
        _ERR = RuntimeError("native extension disabled by PDT_DISABLE_NATIVE=1")
        return
    try:
        import torch  # noqa: F401  (libtorch must be loaded before _C)
        so = os.environ.get("PDT_NATIVE_SO")
        if so:  # an alternative build of the same module (build_native.py --sanitize)
            import sys
            spec = importlib_util.spec_from_file_location("pytorch_distributed_tutorials_amd._C", so)
            _C = importlib_util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["pytorch_distributed_tutorials_amd._C"] = _C
            return
        _C = importlib.import_module("pytorch_distributed_tutorials_amd._C")
    except BaseException as e:  # ImportError, OSError (missing .so deps) ...
        _C = None
        _ERR = e


def native_available() -> bool:
    _load()
    return _C is not None


def native() -> Any:
    """Return the extension module or raise with the reason it failed to load."""
    _load()
    if _C is None:
        raise RuntimeError(
            "pytorch_distributed_tutorials_amd native extension (_C) is not available: "
            f"{_ERR!r}.  Build it with `python build_native.py` (hipcc, gfx950)."
        )
    return _C
