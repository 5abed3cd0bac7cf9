"""roctx ranges around step phases.

``with trace("fwd"):`` pushes a roctx range (visible in
``rocprofv3 --marker-trace`` timelines) when ``PTDT_TRACE=1``; otherwise it is
a no-op costing one attribute lookup. Uses torch's bundled ``libroctx64``
through ctypes, so no extra dependency.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from pathlib import Path

_lib = None
_enabled = os.environ.get("PTDT_TRACE", "0") == "1"


def _load():
    global _lib
    if _lib is not None:
        return _lib
    import torch

    cands = [Path(torch.__file__).parent / "lib" / "libroctx64.so", Path("/opt/rocm/lib/libroctx64.so")]
    for c in cands:
        if c.exists():
            try:
                lib = ctypes.CDLL(str(c))
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return lib
            except OSError:
                continue
    _lib = False
    return _lib


def enable(flag: bool = True) -> None:
    global _enabled
    _enabled = flag


def enabled() -> bool:
    return _enabled and bool(_load())


@contextlib.contextmanager
def trace(name: str):
    if not _enabled or not _load():
        yield
        return
    _lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled and _load():
        _lib.roctxMarkA(name.encode())
