cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" -p no:cacheprovider --no-header --tb=short > gpurun_out/t_gemm15.log 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/gemm_bench.py --shapes 4096x4096x4096,8192x8192x8192,4096x11008x4096 --extra_sched 7 --splits 2 > gpurun_out/gemm_w4.jsonl 2> gpurun_out/gemm_w4.err || exit 2
