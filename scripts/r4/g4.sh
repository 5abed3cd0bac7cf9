# int8 decode rework + ResNet A/B of the fused conv1x1 backward + kernel-trace profile of the step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_llm_int8.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_int8.log 2>&1 || exit 1
timeout -k 10 200 python -u benchmarks/int8_bench.py --shapes 16x11008x4096,1x11008x4096,32x4096x4096,16x4096x11008 > gpurun_out/int8_decode_bench2.jsonl 2> gpurun_out/int8_decode_bench2.err || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_int8 -o run -- python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096,32x4096x4096,16x4096x11008 --rounds 2 > gpurun_out/prof_int8.log 2>&1 || exit 3
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py"
for i in 1 2; do
  PTDT_CONVBN_BWD=0 $R --tag bwd0_$i >> gpurun_out/r4_convbwd_ab.jsonl 2>> gpurun_out/r4_convbwd_ab.err || exit 4
  $R --tag bwd1_$i >> gpurun_out/r4_convbwd_ab.jsonl 2>> gpurun_out/r4_convbwd_ab.err || exit 5
done
timeout -k 10 200 python -u benchmarks/resnet_ddp.py --impl torch --tag torch >> gpurun_out/r4_convbwd_ab.jsonl 2>> gpurun_out/r4_convbwd_ab.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run -- python3 -u benchmarks/resnet_ddp.py --graph off --steps 10 --warmup 3 > gpurun_out/prof_resnet.log 2>&1 || exit 7
