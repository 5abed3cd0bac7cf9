set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_dp_mp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests11.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench11_prof.log 2>&1
rc=$?; tail -2 gpurun_out/r2_gputests11.log; grep '^{' gpurun_out/r2_bench11_prof.log
exit $rc
