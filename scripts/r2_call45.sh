#!/bin/bash
# Wave engine early start: the trainer computes its prologue positions' indices itself and issues
# their row loads while the helpers copy the epoch list (barrier 0 after the prologue fetches).
# Engine/plan/trainer tests, then A/B vs the previous build (abtest/_C_old.so) on the driver
# command, interleaved, 4 rounds; prologue stamps last.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abtest/_C_new.so &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py tests/test_kernels_gpu.py tests/test_trainer_gpu.py > gpurun_out/r45_tests.log 2>&1 &&
o=gpurun_out/r45_ab.jsonl && : > $o &&
for round in 1 2 3 4; do
  for v in old new; do
    cp abtest/_C_$v.so $SO &&
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side 2>> gpurun_out/r45.err | grep '^{' | sed "s/^{/{\"build\": \"$v\", /" >> $o || exit 1
  done
done &&
cp abtest/_C_new.so $SO &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side --stamps 2>> gpurun_out/r45.err | grep '^{' > gpurun_out/r45_stamps.json
