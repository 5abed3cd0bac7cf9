#!/bin/bash
# BN kernels in isolation (ResNet-50 shapes): per-kernel time from a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bnprof -o bn -- python3 benchmarks/bn_bench.py --iters 20 > gpurun_out/bnprof.log 2>&1
