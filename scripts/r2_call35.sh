#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke, the driver's bench command (3 fresh processes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gpu35.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke35.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/r2_bench35.jsonl 2>> gpurun_out/r2_bench35.err || exit 1; done
