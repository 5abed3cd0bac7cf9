set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python benchmarks/pipeline_stream_probe.py > gpurun_out/r2_pp26a.log 2>&1 && \
PYTORCH_NO_HIP_MEMORY_CACHING=1 timeout -k 10 300 python benchmarks/pipeline_stream_probe.py > gpurun_out/r2_pp26b.log 2>&1 && \
MIOPEN_FIND_MODE=1 timeout -k 10 300 python benchmarks/pipeline_stream_probe.py > gpurun_out/r2_pp26c.log 2>&1
rc=$?; grep -h "caching" gpurun_out/r2_pp26*.log; exit $rc
