#!/usr/bin/env python3
"""Build an A/B variant of the extension: the named kernel units recompiled with extra -D defines,
every other object shared with the in-tree build, linked to tools/bin/_C_<tag>.so. Load it with
``PTDT_EXT_PATH=tools/bin/_C_<tag>.so`` (same process layout as the in-tree _C).

    python tools/build_variant.py --tag c1 --units mlp_tp,mlp_tp_bf16 -D PTDT_TP_PRODUCE_C=1
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pytorch_distributed_training_tutorials_amd import _build as B  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--tag", required=True)
    ap.add_argument("--units", required=True, help="comma-separated csrc/kernels/<unit>.hip stems")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args(argv)
    B.build()  # the shared objects are current
    hipcc = B._hipcc()
    _, tlib, _, _ = B._torch_paths()
    out_dir = B.REPO / "build" / f"variant_{a.tag}"
    out_dir.mkdir(parents=True, exist_ok=True)
    units = set(a.units.split(","))
    kernels, hosts = B._sources()
    objs, todo = [], []
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={B.ARCH}", f"-I{B.CSRC}", "-Wno-unused-result"]
    for src in kernels:
        if src.stem in units:
            obj = out_dir / (src.stem + ".o")
            extra = ["-fno-slp-vectorize"] if src.stem.startswith("linear_wave") else []
            todo.append([hipcc, *common, *extra, *[f"-D{d}" for d in a.defines], "-c", str(src), "-o", str(obj)])
        else:
            obj = B.BUILD / (src.stem + ".o")
        objs.append(obj)
    objs += [B.BUILD / (src.stem + ".host.o") for src in hosts]
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(B._run, todo))
    target = B.REPO / "tools" / "bin" / f"_C_{a.tag}.so"
    target.parent.mkdir(parents=True, exist_ok=True)
    B._run([hipcc, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", str(target), *map(str, objs),
            f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-lrccl", "-lamdhip64", f"-Wl,-rpath,{tlib}", "-Wl,--no-as-needed"])
    print(f"built {target}")


if __name__ == "__main__":
    main(sys.argv[1:])
