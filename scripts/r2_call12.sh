set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_dp_mp_gpu.py tests/test_parallel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests12.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench12_prof.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests12.log; grep '^{' gpurun_out/r2_bench12_prof.log
exit $rc
