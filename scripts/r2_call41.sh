#!/bin/bash
# Prologue split of the timed path (plan with a warm list cache, launch_at), 3 processes;
# then launch_at vs device cursor on the new build, interleaved, 4 rounds.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r41.jsonl && : > $o &&
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side --stamps 2>> gpurun_out/r41.err | grep '^{' >> $o || exit 1
done &&
for round in 1 2 3 4; do
  for dc in 1 0; do
    PTDT_BENCH_DEVICE_CURSOR=$dc timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side 2>> gpurun_out/r41.err | grep '^{' | sed "s/^{/{\"device_cursor\": $dc, /" >> $o || exit 1
  done
done
