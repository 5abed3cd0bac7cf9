set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_trainer_gpu.py tests/test_multi_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests7.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench7.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 200 --warmup 20 --share_gpu > gpurun_out/r2_bench7_share2.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests7.log; grep '^{' gpurun_out/r2_bench7.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','ms_per_step','mlp_us_per_step','mlp_engine','mlp_final_loss','persistent_engine')})"; grep '^{' gpurun_out/r2_bench7_share2.log | cut -c1-400; grep -v '^{' gpurun_out/r2_bench7_share2.log | tail -5; exit $rc
