set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py tests/test_trainer_gpu.py tests/test_grad_sink.py tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests9.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench9.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side > gpurun_out/r2_bench9_mlp.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side --persist mfma > gpurun_out/r2_bench9_mlp_old.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 50 --share_gpu --model mlp --no_mlp_side > gpurun_out/r2_bench9_share2.log 2>&1
rc=$?; tail -2 gpurun_out/r2_gputests9.log
for f in r2_bench9 r2_bench9_mlp r2_bench9_mlp_old r2_bench9_share2; do grep '^{' gpurun_out/$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', {k:d.get(k) for k in ('value','ms_per_step','mlp_us_per_step','mlp_engine','persistent_engine','final_loss','replicas_in_sync')})"; done
exit $rc
