"""roctx ranges for the PS phases (the reference has no tracer at all).

``PSX_ROCTX=1`` turns every ``PhaseTimer.span`` (fetch / compute_issue / push / apply ...) and
explicit ``trace.range(...)`` into a roctx range, so ``rocprofv3 --marker-trace
--kernel-trace`` shows the parameter-server protocol phases on the same timeline as the HIP
kernels and RCCL collectives. The ranges come from librocprofiler-sdk-roctx (what rocprofv3
records), falling back to the legacy libroctx64; with the variable unset nothing is loaded.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_tried = False


def enabled() -> bool:
    return os.environ.get("PSX_ROCTX", "0") == "1"


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        for path in (name, os.path.join("/opt/rocm/lib", name)):
            try:
                lib = ctypes.CDLL(path)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return _lib
    return None


def push(name: str):
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop():
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str):
    lib = _load() if enabled() else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001  (mirrors roctx naming)
    push(name)
    try:
        yield
    finally:
        pop()
