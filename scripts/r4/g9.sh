cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convbn_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_convbn9.log 2>&1 || exit 1
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve"
O=gpurun_out/r4_convbwd_ab2.jsonl
E=gpurun_out/r4_convbwd_ab2.err
for i in 1 2; do
  PTDT_CONVBN_BWD=0 $R --tag bwd0_$i >> $O 2>> $E || exit 2
  PTDT_CONVBN_BWD=1 $R --tag bwd1_$i >> $O 2>> $E || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet2 -o run -- python3 -u benchmarks/resnet_ddp.py --graph off --steps 10 --warmup 3 > gpurun_out/prof_resnet2.log 2>&1 || exit 4
