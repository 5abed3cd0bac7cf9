cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_tp27.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model mlp --steps 2000 --warmup 200 --no_ref --stamps --out gpurun_out/r4_tp_ahead.jsonl > /dev/null 2>> gpurun_out/r4_tp_ahead.err || exit 2
timeout -k 10 200 python -u bench.py --model mlp --steps 20 --warmup 5 --no_ref --out gpurun_out/r4_tp_ahead.jsonl > /dev/null 2>> gpurun_out/r4_tp_ahead.err || exit 3
S="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $S --nproc-per-node 4 --master-port 29681 bench.py --gpus 4 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_tp_ahead_share.jsonl > /dev/null 2>> gpurun_out/r4_tp_ahead.err || exit 4
timeout -k 10 400 $S --nproc-per-node 2 --master-port 29682 bench.py --gpus 2 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_tp_ahead_share.jsonl > /dev/null 2>> gpurun_out/r4_tp_ahead.err || exit 5
