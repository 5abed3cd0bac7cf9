# int8 decode: statistics kernel with 8 row groups of 4 rows vs the previous build (same box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
SH=16x11008x4096,32x11008x4096,16x4096x11008,16x4096x4096,1x4096x4096
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_llm_int8.py > gpurun_out/r4_i8_s_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_snew1.jsonl 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/i8p -o run -- python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096 --rounds 2 > gpurun_out/r4_i8_prof.log 2>&1 || exit 3
cp $(find /tmp/i8p -name '*kernel_stats.csv' | head -1) gpurun_out/r4_i8_s_kernel_stats.csv
cp $SO /tmp/new.so && cp _ab/old_C.so $SO || exit 4
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_sold1.jsonl 2>&1 || exit 5
cp /tmp/new.so $SO || exit 6
timeout -k 10 200 python3 -u benchmarks/int8_bench.py --shapes $SH > gpurun_out/r4_i8_snew2.jsonl 2>&1 || exit 7
