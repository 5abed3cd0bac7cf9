set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests23.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests23.log; exit $rc
