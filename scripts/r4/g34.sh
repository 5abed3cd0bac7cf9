# int8 decode GEMV: 8 waves per workgroup everywhere (PTDT_I8_WIDE=1) vs the default split
cd $GRAFT_REPO_ROOT
SH=16x11008x4096,32x11008x4096,16x4096x11008,16x4096x4096
for r in 1 2; do
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_def$r.jsonl 2>&1 || exit 1
PTDT_I8_WIDE=1 timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_wide$r.jsonl 2>&1 || exit 2
PTDT_I8_WIDE=0 timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_narrow$r.jsonl 2>&1 || exit 3
done
PTDT_I8_WIDE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_wide_tests.log 2>&1 || exit 4
