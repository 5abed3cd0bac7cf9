#!/bin/bash
# BN: vectorised one-round partial combine -- numerics tests, then a per-kernel trace and a block-count sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm.py > gpurun_out/bn33_tests.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnprof33 -o bn -- python3 benchmarks/bn_bench.py --iters 20 --native_only > gpurun_out/bnprof33.log 2>&1 &&
for round in 1 2; do
for rb in 384 512 768; do
  PTDT_BN_RED_BLOCKS=$rb timeout -k 10 120 python3 benchmarks/bn_bench.py --iters 30 --native_only >> gpurun_out/bn_sweep33.jsonl 2>/dev/null || exit 1
done; done
