# int8 decode: one-launch prep (every workgroup computes all column maxima) vs stats + quant (PTDT_I8_PREP=2)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SH=16x11008x4096,32x11008x4096,16x4096x11008,16x4096x4096,1x4096x4096
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_p1_tests.log 2>&1 || exit 1
PTDT_I8_PREP=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_p2_tests.log 2>&1 || exit 2
for r in 1 2; do
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_p1_$r.jsonl 2>&1 || exit 3
PTDT_I8_PREP=2 timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_p2_$r.jsonl 2>&1 || exit 4
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/i8p -o run -- python3 -u benchmarks/int8_bench.py --shapes $SH --rounds 2 > gpurun_out/r4_i8_prof.log 2>&1 || exit 5
cp $(find /tmp/i8p -name '*kernel_stats.csv' | head -1) gpurun_out/r4_i8_p1_kernel_stats.csv
