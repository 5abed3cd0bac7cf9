# ResNet A/B of the fused conv1x1 backward, kernel-trace profile of the default step, full GPU suite, bench.py
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py"
for i in 1 2; do
  PTDT_CONVBN_BWD=0 $R --tag bwd0_$i >> gpurun_out/r4_convbwd_ab.jsonl 2>> gpurun_out/r4_convbwd_ab.err || exit 1
  $R --tag bwd1_$i >> gpurun_out/r4_convbwd_ab.jsonl 2>> gpurun_out/r4_convbwd_ab.err || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run -- python3 -u benchmarks/resnet_ddp.py --graph off --steps 10 --warmup 3 > gpurun_out/prof_resnet.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --no-header --tb=short > gpurun_out/t_all.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 5
