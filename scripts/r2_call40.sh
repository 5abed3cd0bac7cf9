#!/bin/bash
# Persistent-launch prologue, 3-way A/B on the driver command (interleaved, 4 rounds):
#   old  = previous build (abtest/_C_old.so), device cursor;
#   cur  = new build (list copy in one round trip, parameters read first), device cursor;
#   at   = new build, PersistentPlan.launch_at (start position from the bench's step count).
# Numerics first (launch_at vs device cursor bitwise, plan tests), then prologue split stamps.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
cp $SO abtest/_C_new.so &&
true &&
o=gpurun_out/r40_ab.jsonl && : > $o &&
for round in 1 2 3 4; do
  for v in old cur at; do
    so=new; dc=1
    [ $v = old ] && so=old
    [ $v = at ] && dc=0
    cp abtest/_C_$so.so $SO &&
    PTDT_BENCH_DEVICE_CURSOR=$dc timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side 2>> gpurun_out/r40_ab.err | sed "s/^{/{\"build\": \"$v\", /" >> $o 2>> gpurun_out/r40_ab.err || exit 1
  done
done &&
cp abtest/_C_new.so $SO &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side --stamps > gpurun_out/r40_stamps.json 2>> gpurun_out/r40_ab.err &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r40_full.json 2>> gpurun_out/r40_ab.err
