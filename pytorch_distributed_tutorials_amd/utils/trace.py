"""Tracing: roctx ranges for rocprofv3 timelines, zero-cost when off.

The reference has no tracing code; its only implicit hook is the
``record_function("DistributedDataParallel.forward")`` torch DDP wraps around
forward.  Here the trainer brackets forward / backward / optimizer / eval in
named ranges that show up in ``rocprofv3 --marker-trace`` (ROCTx from
``/opt/rocm/lib/libroctx64.so``, loaded with ctypes so nothing is linked) and,
when a ``torch.profiler`` session is active, in its trace too.

Enable with ``PDT_TRACE=1`` or :func:`enable`.  Disabled ranges are a single
attribute check.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

import torch

_enabled = os.environ.get("PDT_TRACE", "0") == "1"
_lib: Optional[ctypes.CDLL] = None
_lib_tried = False


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib, _lib_tried
    if not _lib_tried:
        _lib_tried = True
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled


def available() -> bool:
    """True when ROCTx could be loaded (ranges then reach rocprofv3)."""
    return _roctx() is not None


@contextlib.contextmanager
def trace_range(name: str):
    if not _enabled:
        yield
        return
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _roctx() is not None:
        _lib.roctxMarkA(name.encode())
