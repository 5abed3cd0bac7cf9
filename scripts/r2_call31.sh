#!/bin/bash
# BN reduction geometry / row-pipelining sweep (interleaved variants, one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for round in 1 2; do
for pipe in 0 1; do
for rb in 384 512 768 1024; do
  PTDT_BN_PIPE=$pipe PTDT_BN_RED_BLOCKS=$rb timeout -k 10 120 python3 benchmarks/bn_bench.py --iters 30 --native_only >> gpurun_out/bn_sweep.jsonl 2>/dev/null || exit 1
done; done; done
