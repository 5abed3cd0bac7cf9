cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convbn_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_convbn16.log 2>&1 || exit 1
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve"
for i in 1 2; do
  $R --tag c256_128_$i >> gpurun_out/r4_convbwd_256_128.jsonl 2>> gpurun_out/r4_convbwd_256_128.err || exit 2
done
