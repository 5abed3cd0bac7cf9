set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_llm_int8.py tests/test_dp_mp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests27.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests27.log; grep -E "^E " gpurun_out/r2_gputests27.log | head -8; exit $rc
