cd $GRAFT_REPO_ROOT
S="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $S --nproc-per-node 2 --master-port 29621 bench.py --gpus 2 --share_gpu --steps 20 --warmup 5 --out gpurun_out/r4_share_final.jsonl > /dev/null 2> gpurun_out/r4_share_final.err || exit 1
timeout -k 10 400 $S --nproc-per-node 8 --master-port 29622 bench.py --gpus 8 --share_gpu --steps 20 --warmup 5 --out gpurun_out/r4_share_final.jsonl > /dev/null 2>> gpurun_out/r4_share_final.err || exit 2
timeout -k 10 400 $S --nproc-per-node 4 --master-port 29623 bench.py --gpus 4 --share_gpu --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_final.jsonl > /dev/null 2>> gpurun_out/r4_share_final.err || exit 3
