cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --no-header --tb=short > gpurun_out/t_all25.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke25.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/bench25.json 2> gpurun_out/bench25.err || exit 3
timeout -k 10 200 python -u bench.py --model mlp --steps 20 --warmup 5 --no_ref --stamps --out gpurun_out/r4_tp_prologue2.jsonl > /dev/null 2>> gpurun_out/r4_tp_prologue2.err || exit 4
