#!/bin/bash
# GEMM: 10-piece LDS ring + coalesced epilogue -- numerics (GEMM/Linear tests), then the interleaved bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or linear" > gpurun_out/gemm36_tests.log 2>&1 &&
timeout -k 10 400 python3 benchmarks/gemm_bench.py --extra_sched 1 --splits "" --rounds 5 \
  --shapes 4096x4096x4096,8192x8192x8192,8192x8192x1024,4096x11008x4096,4096x4096x1024,3072x3072x3072,2048x2048x2048,1000x3000x4096,256x256x64,300x520x128 \
  > gpurun_out/gemm36.jsonl 2> gpurun_out/gemm36.err
