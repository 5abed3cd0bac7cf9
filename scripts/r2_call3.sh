set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent or wave or sampler or fused" > gpurun_out/r2_gputests3.log 2>&1 && \
timeout -k 10 100 python benchmarks/wave_fixed_cost.py > gpurun_out/r2_wave_fixed3.log 2>&1 && \
timeout -k 10 120 python benchmarks/overhead_probe.py > gpurun_out/r2_probe3.log 2>&1 && \
for i in 1 2 3; do timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>&1 | grep '^{' >> gpurun_out/r2_bench20_3.jsonl || exit 1; done
rc=$?; tail -3 gpurun_out/r2_gputests3.log; grep '^{' gpurun_out/r2_wave_fixed3.log; grep '^{' gpurun_out/r2_probe3.log | head -9; cut -c1-330 gpurun_out/r2_bench20_3.jsonl; exit $rc
