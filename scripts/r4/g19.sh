cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_llm_int8.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_int8_19.log 2>&1 || exit 1
timeout -k 10 200 python -u benchmarks/int8_bench.py --shapes 16x11008x4096,1x11008x4096,32x4096x4096,16x4096x11008 > gpurun_out/int8_decode_bench5.jsonl 2> gpurun_out/int8_decode_bench5.err || exit 2
