cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_llm_int8.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_int8_21.log 2>&1 || exit 9
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_tp20.log 2>&1 || exit 1
for n in 1 20 2000; do
  timeout -k 10 200 python -u bench.py --model mlp --steps $n --warmup 5 --no_ref --out gpurun_out/r4_mlp_steps2.jsonl > /dev/null 2>> gpurun_out/r4_mlp_steps2.err || exit 2
done
S="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 400 $S --nproc-per-node 4 --master-port 29631 bench.py --gpus 4 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_mlp.jsonl > /dev/null 2> gpurun_out/r4_share_mlp.err || exit 3
timeout -k 10 400 $S --nproc-per-node 8 --master-port 29632 bench.py --gpus 8 --share_gpu --model mlp --steps 2000 --warmup 200 --no_ref --out gpurun_out/r4_share_mlp.jsonl > /dev/null 2>> gpurun_out/r4_share_mlp.err || exit 4
