#!/bin/bash
# Final tree (rebuilt after the early-start revert): full GPU suite, smoke, driver bench.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r46_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r46_smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/r46_bench_default.json 2>> gpurun_out/r46.err &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r46_bench.json 2>> gpurun_out/r46.err
