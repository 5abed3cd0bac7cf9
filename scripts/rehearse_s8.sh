#!/bin/bash
# Rehearse the per-rank shape of the N=8 run (256 samples per rank -> 8 steps per epoch) with
# 4 ranks sharing cuda:0 and a 1024-sample dataset; plus an odd world size. Not a scaling number.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, N, extra args...
  local name=$1 n=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus "$n" --share_gpu "$@" > "gpurun_out/$name.log" 2>&1
  local c=$?
  echo "=== $name exit $c"; grep '^{' "gpurun_out/$name.log" || tail -20 "gpurun_out/$name.log"
  [ $c -eq 0 ] || exit $c
}
run rehearse_n4_s8 4 --dataset_size 1024 --steps 20000 --warmup 2000
run rehearse_n3 3 --steps 20000 --warmup 2000
run rehearse_n4_s8_mlp 4 --model mlp --dataset_size 1024 --steps 5000 --warmup 500
echo "=== done"
