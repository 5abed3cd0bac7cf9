cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_llm_int8.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_int8_12.log 2>&1 || exit 1
timeout -k 10 200 python -u benchmarks/int8_bench.py --shapes 16x11008x4096,1x11008x4096,32x4096x4096,16x4096x11008 > gpurun_out/int8_decode_bench3.jsonl 2> gpurun_out/int8_decode_bench3.err || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8b -o run -- python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x4096x4096,16x4096x11008 --rounds 2 > gpurun_out/prof_int8b.log 2>&1 || exit 3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" -p no:cacheprovider --no-header --tb=short > gpurun_out/t_gemm12.log 2>&1 || exit 4
timeout -k 10 300 python -u benchmarks/gemm_bench.py --shapes 4096x4096x4096,8192x8192x8192,4096x11008x4096 --extra_sched 3 5 6 --splits 2 > gpurun_out/gemm_grp2.jsonl 2> gpurun_out/gemm_grp2.err || exit 5
