# int8 decode GEMV on pre-shuffled weights (PTDT_I8_PACKED=1 default) vs row-major -- tests, A/B, kernel stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SH=16x11008x4096,32x11008x4096,16x4096x11008,16x4096x4096
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_pk_tests.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_pk$r.jsonl 2>&1 || exit 2
PTDT_I8_PACKED=0 timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_rm$r.jsonl 2>&1 || exit 3
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/i8p -o run -- python3 -u benchmarks/int8_bench.py --shapes $SH --rounds 2 > gpurun_out/r4_i8_prof.log 2>&1 || exit 4
cp $(find /tmp/i8p -name '*kernel_stats.csv' | head -1) gpurun_out/r4_i8_pk_kernel_stats.csv
