set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/r2_counters.txt 2>&1
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/r2_counters.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
timeout -k 10 300 python -u -m pytest tests/test_norm.py -x -q --timeout 120 --timeout-method thread -k residual_link > gpurun_out/r2_gputests18.log 2>&1; tail -2 gpurun_out/r2_gputests18.log
