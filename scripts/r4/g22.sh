cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_tp22.log 2>&1 || exit 1
S="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
for i in 1 2; do
timeout -k 10 400 $S --nproc-per-node 4 --master-port 2964$i bench.py --gpus 4 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_mlp2.jsonl > /dev/null 2>> gpurun_out/r4_share_mlp2.err || exit 2
timeout -k 10 400 $S --nproc-per-node 2 --master-port 2965$i bench.py --gpus 2 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_mlp2.jsonl > /dev/null 2>> gpurun_out/r4_share_mlp2.err || exit 3
done
timeout -k 10 400 $S --nproc-per-node 8 --master-port 29661 bench.py --gpus 8 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_mlp2.jsonl > /dev/null 2>> gpurun_out/r4_share_mlp2.err || exit 4
