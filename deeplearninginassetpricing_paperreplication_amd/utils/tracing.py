"""roctx ranges around the training schedule (an addition: the reference only prints wall-clock
times, `/root/reference/src/train.py:227,239,276`).

Ranges are pushed through ROCm's ``libroctx64`` (loaded with ctypes, nothing to build) so
``rocprofv3 --marker-trace`` shows phase / print-interval / evaluation regions around the HIP
kernels. The library is optional: without it (CPU-only machines) every call is a no-op.
``DLAP_ROCTX=0`` disables the ranges.

    with trace_range("phase3"):
        ...
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, Optional

_LIB = None
_TRIED = False
_CANDIDATES = ("libroctx64.so", "/opt/rocm/lib/libroctx64.so", "libroctx64.so.4")


def _lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("DLAP_ROCTX", "1") == "0":
        return None
    for name in _CANDIDATES:
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _LIB = lib
            break
        except (OSError, AttributeError):
            continue
    return _LIB


def available() -> bool:
    return _lib() is not None


def push(name: str):
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop():
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str):
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class Timers:
    """Accumulated host wall time per range name (printed by the trainer's summary)."""

    def __init__(self):
        self.total: Dict[str, float] = {}
        self.count: Dict[str, int] = {}

    def add(self, name: str, dt: float):
        self.total[name] = self.total.get(name, 0.0) + dt
        self.count[name] = self.count.get(name, 0) + 1

    def summary(self) -> str:
        return "\n".join(f"  {k:<24s} {v:9.3f} s  ({self.count[k]} calls)" for k, v in self.total.items())


@contextlib.contextmanager
def trace_range(name: str, timers: Optional[Timers] = None):
    push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        pop()
        if timers is not None:
            timers.add(name, time.perf_counter() - t0)
