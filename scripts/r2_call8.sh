set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_mlp_tp_gpu.py tests/test_xgmi_gpu.py tests/test_trainer_gpu.py tests/test_grad_sink.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_gputests8.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert|passed|failed" gpurun_out/r2_gputests8.log | tail -40; exit $rc
