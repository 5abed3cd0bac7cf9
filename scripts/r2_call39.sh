#!/bin/bash
# Persistent-launch prologue: epoch list copied with every load in flight (one round trip with
# the cache tag) and the trainer's parameters read before it. A/B against the previous build
# (abtest/_C_old.so) on the driver command, interleaved, 3 rounds; numerics of the engines first.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abtest/_C_new.so &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py tests/test_kernels_gpu.py tests/test_trainer_gpu.py tests/test_mlp_tp_gpu.py > gpurun_out/r39_tests.log 2>&1 &&
o=gpurun_out/r39_ab.jsonl && : > $o &&
for round in 1 2 3; do
  for v in old new; do
    cp abtest/_C_$v.so $SO &&
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side | sed "s/^{/{\"build\": \"$v\", /" >> $o 2>> gpurun_out/r39_ab.err || exit 1
  done
done &&
cp abtest/_C_new.so $SO &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side --stamps > gpurun_out/r39_stamps.json 2>> gpurun_out/r39_ab.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof39 -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side > gpurun_out/r39_prof.log 2>&1
