#!/bin/bash
# Re-created container: validate the freshly rebuilt tree on the GPU -- full GPU suite, smoke,
# the driver's bench command (3 fresh processes), the mlp side metric, and a kernel trace of the
# driver command.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r38_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r38_smoke.log 2>&1 &&
o=gpurun_out/r38_bench.jsonl && : > $o &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $o 2>> gpurun_out/r38_bench.err || exit 1; done &&
timeout -k 10 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --stamps >> $o 2>> gpurun_out/r38_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof38 -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r38_prof.log 2>&1
