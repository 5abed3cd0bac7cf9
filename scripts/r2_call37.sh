#!/bin/bash
# BN reductions: interleaved row chunks (grid sweeps the tensor together) vs one slab per block.
# numerics, isolated per-kernel traces of both orders, then the ResNet-50 DDP step A/B (2 rounds).
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm.py > gpurun_out/bn37_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnprof37 -o il -- python3 benchmarks/bn_bench.py --iters 20 --native_only > gpurun_out/bnprof37.log 2>&1 &&
PTDT_BN_INTERLEAVE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnprof37 -o slab -- python3 benchmarks/bn_bench.py --iters 20 --native_only >> gpurun_out/bnprof37.log 2>&1 &&
o=gpurun_out/r2_resnet37.jsonl && : > $o &&
for round in 1 2; do
  for il in 1 0; do
    PTDT_BN_INTERLEAVE=$il timeout -k 10 300 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5 | sed "s/^{/{\"bn_interleave\": $il, /" >> $o 2>> gpurun_out/r2_resnet37.err || exit 1
  done
done
