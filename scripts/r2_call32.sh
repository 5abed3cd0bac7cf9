#!/bin/bash
# GEMM: ring-slab schedule (sched 2) vs the ping-pong kernel vs hipBLASLt, interleaved in one process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 benchmarks/gemm_bench.py --extra_sched 2 --splits "" --rounds 5 \
  --shapes 1000x3000x4096,256x256x64,300x520x128,4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x11008x4096,4096x4096x1024,3072x3072x3072 \
  > gpurun_out/gemm_ring.jsonl 2> gpurun_out/gemm_ring.err
