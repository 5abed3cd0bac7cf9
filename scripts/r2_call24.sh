set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_mlp_tp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests24.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side --stamps > gpurun_out/r2_bench24_mlp.log 2>&1 && \
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side > gpurun_out/r2_bench24_mlp_nostamp.log 2>&1
rc=$?; tail -3 gpurun_out/r2_gputests24.log
for f in gpurun_out/r2_bench24_mlp.log gpurun_out/r2_bench24_mlp_nostamp.log; do grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in ('value','ms_per_step','persistent_engine','phase_timers')})"; done
exit $rc
