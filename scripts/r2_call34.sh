#!/bin/bash
# BN reductions with more rows in flight (packed loads): numerics, per-kernel trace, fwd+bwd totals.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm.py > gpurun_out/bn34_tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnprof34 -o bn -- python3 benchmarks/bn_bench.py --iters 20 --native_only > gpurun_out/bnprof34.log 2>&1 &&
timeout -k 10 120 python3 benchmarks/bn_bench.py --iters 30 > gpurun_out/bn34.jsonl 2>/dev/null
