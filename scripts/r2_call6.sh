set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_trainer_gpu.py tests/test_parallel_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_gputests6.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r2_gputests6.log | tail -40; exit $rc
