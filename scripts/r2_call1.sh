set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench20.log 2>&1 && \
timeout -k 10 120 python benchmarks/overhead_probe.py > gpurun_out/r2_probe.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests.log; tail -1 gpurun_out/r2_bench20.log; cat gpurun_out/r2_probe.log | tail -12; exit $rc
