#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: N ranks share cuda:0 (gloo control plane,
# in-kernel xGMI all-reduce through IPC buffers, replica-sync check). Not a scaling number.
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
run rehearse_n2 2 --steps 20000 --warmup 2000
run rehearse_n4 4 --steps 20000 --warmup 2000
run rehearse_n2_mlp 2 --model mlp --steps 5000 --warmup 500
run rehearse_n4_mlp 4 --model mlp --steps 5000 --warmup 500
run rehearse_n2_fused 2 --engine fused --steps 2000 --warmup 200
run rehearse_n4_fused_mlp 4 --engine fused --model mlp --steps 2000 --warmup 200
echo "=== done"
