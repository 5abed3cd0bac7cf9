#!/bin/bash
# TP MLP engine: lists produced before the batch loads, 32-bit label loads (no vmcnt(0) stall in the
# forward). TP numerics first, then A/B vs the build before this session's TP changes
# (abtest/_C_old.so) on bench --model mlp (20000 steps), interleaved, 3 rounds; stamps last.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abtest/_C_new.so &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py > gpurun_out/r43_tests.log 2>&1 &&
o=gpurun_out/r43_ab.jsonl && : > $o &&
for round in 1 2 3; do
  for v in old new; do
    cp abtest/_C_$v.so $SO &&
    timeout -k 10 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 2>> gpurun_out/r42.err | grep '^{' | sed "s/^{/{\"build\": \"$v\", /" >> $o || exit 1
  done
done &&
cp abtest/_C_new.so $SO &&
timeout -k 10 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --stamps 2>> gpurun_out/r42.err | grep '^{' > gpurun_out/r43_stamps.json
