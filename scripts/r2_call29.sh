set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --share_gpu --steps 200 --warmup 20 > gpurun_out/r2_share29.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --share_gpu --steps 200 --warmup 20 --model mlp > gpurun_out/r2_share29_mlp.log 2>&1
rc=$?; for f in gpurun_out/r2_share29.log gpurun_out/r2_share29_mlp.log; do grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in ('value','ms_per_step','n_gpus','allreduce','persistent_engine','replicas_in_sync','mlp_us_per_step','mlp_replicas_in_sync')})"; done; tail -3 gpurun_out/r2_share29.log
exit $rc
