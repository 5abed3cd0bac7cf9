set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python bench.py --gpus 1 --steps 2000 --warmup 200 --model mlp --no_mlp_side --stamps > gpurun_out/r2_bench22_mlp.log 2>&1
rc=$?; grep '^{' gpurun_out/r2_bench22_mlp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:d.get(k) for k in ('value','ms_per_step','persistent_engine','phase_timers')})"
exit $rc
