# int8 decode: one-launch statistics + quantisation kernel -- tests, then fused vs three-launch A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_fused_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x11008x4096,16x4096x11008 > gpurun_out/r4_i8_fused_bench.jsonl 2>&1 || exit 2
PTDT_I8_FUSED_PREP=0 timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x11008x4096,16x4096x11008 > gpurun_out/r4_i8_unfused_bench.jsonl 2>&1 || exit 3
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x11008x4096,16x4096x11008 > gpurun_out/r4_i8_fused_bench2.jsonl 2>&1 || exit 4
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/i8p -o run -- python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x11008x4096,16x4096x11008 > gpurun_out/r4_i8_prof.log 2>&1 || exit 5
cp $(find /tmp/i8p -name '*kernel_stats.csv' | head -1) gpurun_out/r4_i8_kernel_stats.csv
