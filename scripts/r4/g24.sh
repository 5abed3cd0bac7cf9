cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mlp_tp_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_tp24.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --model mlp --steps 20 --warmup 5 --no_ref --stamps --out gpurun_out/r4_tp_prologue.jsonl > /dev/null 2>> gpurun_out/r4_tp_prologue.err || exit 2
timeout -k 10 200 python -u bench.py --model mlp --steps 1 --warmup 5 --no_ref --stamps --out gpurun_out/r4_tp_prologue.jsonl > /dev/null 2>> gpurun_out/r4_tp_prologue.err || exit 3
