set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests28.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke28.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench28.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side --stamps > gpurun_out/r2_bench28_mlp.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests28.log; grep -E "^(FAILED|ERROR)" gpurun_out/r2_gputests28.log | head; tail -1 gpurun_out/r2_smoke28.log; grep '^{' gpurun_out/r2_bench28.log | cut -c1-400
exit $rc
grep "^{" gpurun_out/r2_bench28_mlp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in (\"value\",\"ms_per_step\",\"phase_timers\")})"
