"""Native build driver: compiles csrc/ for gfx950 with hipcc into the in-tree
extension ``pytorch_distributed_training_tutorials_amd/_C*.so``.

No hipify, no torch JIT cache: every ``.hip`` kernel file is compiled with
``hipcc --offload-arch=gfx950`` without torch headers (fast, ABI independent),
the C++ runtime (RCCL communicator, reducer, bindings) with torch headers, and
the objects are linked against the HIP/RCCL libraries torch itself ships (same
sonames, so one copy of each runtime is loaded per process).

Usage: ``python -m pytorch_distributed_training_tutorials_amd._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ARCH = "gfx950"
PKG_DIR = Path(__file__).resolve().parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
TARGET = PKG_DIR / f"_C{EXT_SUFFIX}"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the native extension)")


def _torch_paths():
    import torch  # noqa: F401  (import only for paths / ABI flag)
    from torch.utils import cpp_extension as ce

    tdir = Path(torch.__file__).resolve().parent
    incs = [str(tdir / "include"), str(tdir / "include" / "torch" / "csrc" / "api" / "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, str(tdir / "lib"), abi, ce


def _sources():
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    hosts = [CSRC / "comm" / "rccl_comm.cpp", CSRC / "comm" / "xgmi_comm.cpp", CSRC / "reducer" / "reducer.cpp",
             CSRC / "bindings.cpp"]
    return kernels, hosts


def _headers():
    return sorted(list(CSRC.rglob("*.h")))


_INC = None


def _deps(src: Path):
    """The csrc headers ``src`` includes, transitively (quoted includes resolved next to the including
    file, then under csrc/): a header edit rebuilds only the units that see it."""
    import re

    global _INC
    if _INC is None:
        _INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)
    seen, todo = set(), [src]
    while todo:
        f = todo.pop()
        try:
            text = f.read_text(errors="replace")
        except OSError:
            continue
        for name in _INC.findall(text):
            for cand in (f.parent / name, CSRC / name):
                cand = cand.resolve()
                if cand.exists() and cand.suffix == ".h" and cand not in seen:
                    seen.add(cand)
                    todo.append(cand)
                    break
    return sorted(seen)


def _newer(src: Path, obj: Path, deps) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{p.stdout}")
    return p.stdout


def build(force: bool = False, jobs: int | None = None, verbose: bool = False, stamps: bool = False) -> Path:
    """Build the extension. ``stamps=True`` builds a DIAGNOSTIC copy instead: the single-wave
    engine with its per-phase timers compiled in (-DPTDT_WAVE_STAMPS=1, objects in
    build/native_stamps, every other object shared), linked to tools/bin/_C_stamps.so; load it
    with ``PTDT_EXT_PATH=tools/bin/_C_stamps.so`` for ``bench.py --stamps`` phase splits."""
    hipcc = _hipcc()
    incs, tlib, abi, _ = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    BUILD.mkdir(parents=True, exist_ok=True)
    kernels, hosts = _sources()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", f"-I{CSRC}", "-Wno-unused-result"]
    host_flags = common + [
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1", "-DHIPBLAS_V2",
        f"-I{py_inc}", *[f"-I{i}" for i in incs], "-I/opt/rocm/include",
        "-Wno-deprecated-declarations", "-Wno-unused-parameter",
    ]
    jobs = jobs or min(8, (os.cpu_count() or 2))
    todo = []
    objs = []
    stamp_dir = REPO / "build" / "native_stamps"
    if stamps:
        stamp_dir.mkdir(parents=True, exist_ok=True)
    for src in kernels:
        wave = src.stem.startswith("linear_wave")
        obj = (stamp_dir if (stamps and wave) else BUILD) / (src.stem + ".o")
        objs.append(obj)
        if force or _newer(src, obj, _deps(src)):
            # single-wave engine: no SLP vectorisation -- it splits DPP adds into
            # v_mov_dpp + v_pk_add pairs (plus zero-inits), ~50 extra VALU per step
            extra = ["-fno-slp-vectorize"] if wave else []
            if stamps and wave:
                extra.append("-DPTDT_WAVE_STAMPS=1")
            todo.append([hipcc, *common, *extra, "-c", str(src), "-o", str(obj)])
    for src in hosts:
        obj = BUILD / (src.stem + ".host.o")
        objs.append(obj)
        if force or _newer(src, obj, _deps(src)):
            # host-only translation units: -x hip keeps hipcc's HIP headers/macros, no device code is emitted
            todo.append([hipcc, *host_flags, "-x", "hip", "-c", str(src), "-o", str(obj)])
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, todo):
                if verbose and out.strip():
                    print(out)
    target = (REPO / "tools" / "bin" / "_C_stamps.so") if stamps else TARGET
    target.parent.mkdir(parents=True, exist_ok=True)
    relink = force or bool(todo) or not target.exists() or any(o.stat().st_mtime > target.stat().st_mtime for o in objs)
    if relink:
        tmp = target.with_suffix(".tmp.so")
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs),
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
              "-lrccl", "-lamdhip64", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"])
        os.replace(tmp, target)
    return target


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--stamps", action="store_true", help="diagnostic build with the wave engine's phase timers")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose, stamps=a.stamps)
    print(f"built {out}")


if __name__ == "__main__":
    main(sys.argv[1:])
