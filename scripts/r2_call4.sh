set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent or wave or sampler or fused or xgmi" > gpurun_out/r2_gputests4.log 2>&1 && \
timeout -k 10 120 python benchmarks/overhead_probe.py > gpurun_out/r2_probe4.log 2>&1 && \
for i in 1 2 3 4 5; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>&1 | grep '^{' >> gpurun_out/r2_bench20_4.jsonl || exit 1; done
rc=$?; tail -3 gpurun_out/r2_gputests4.log; grep '^{' gpurun_out/r2_probe4.log | head -9; cut -c100-220 gpurun_out/r2_bench20_4.jsonl; exit $rc
