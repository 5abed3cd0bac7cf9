cd $GRAFT_REPO_ROOT
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py"
O=gpurun_out/r4_convbwd_256_128_ab.jsonl
for i in 1 2 3; do
  PTDT_CONVBN_BWD_SKIP=256x128 $R --tag skip_$i >> $O 2>> gpurun_out/r4_ab17.err || exit 1
  $R --tag with_$i >> $O 2>> gpurun_out/r4_ab17.err || exit 2
done
