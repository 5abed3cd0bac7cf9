"""Loader for the in-tree native extension (``_C``: gfx950 kernels, RCCL
communicator, DDP reducer).

The extension is built by :mod:`._build` (``__graft_entry__.build()``) into
this package directory. Rules:

* torch is always imported first, so the extension binds to the HIP and RCCL
  runtimes torch already mapped (same sonames) -- never a second copy;
* on a machine with a GPU the native path is mandatory: :func:`native` raises
  if the extension is missing instead of silently falling back to eager ATen;
* on a CPU-only machine the pure-PyTorch reference implementations in
  ``ops`` are used (plumbing tests), and the reducer still runs natively on
  CPU tensors when the extension is importable.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

import torch  # noqa: F401  -- must precede the extension import

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            override = os.environ.get("PTDT_EXT_PATH")  # e.g. the ASan/UBSan host build (tools/sanitize_host.py)
            if override:
                spec = importlib.util.spec_from_file_location(__package__ + "._C", override)
                _mod = importlib.util.module_from_spec(spec)
                sys.modules[__package__ + "._C"] = _mod
                spec.loader.exec_module(_mod)
                return
            _mod = importlib.import_module(__package__ + "._C")
        except Exception as e:  # pragma: no cover - depends on build state
            if os.environ.get("PTDT_AUTOBUILD", "1") == "1":
                try:
                    from . import _build

                    _build.build()
                    _mod = importlib.import_module(__package__ + "._C")
                    return
                except Exception as e2:  # noqa: BLE001
                    _err = e2
                    return
            _err = e


def has_native() -> bool:
    _load()
    return _mod is not None


def native():
    """The native module; raises if it is unavailable."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "pytorch_distributed_training_tutorials_amd native extension (_C) is not available: "
            f"{_err!r}. Build it with `python -m pytorch_distributed_training_tutorials_amd._build`."
        )
    return _mod


def gpu_available() -> bool:
    return torch.cuda.is_available()


def use_native(*tensors) -> bool:
    """True when the tensors live on the GPU (native kernels are then REQUIRED)."""
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors)


def hip_runtime_copies() -> list[str]:
    """Paths of libamdhip64 mapped in this process (must be exactly one)."""
    out = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    out.add(line.split()[-1])
    except OSError:
        pass
    return sorted(out)
