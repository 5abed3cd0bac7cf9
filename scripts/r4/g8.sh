cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_graphs_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_graphs8.log 2>&1 || exit 1
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve --steps 10 --warmup 5"
O=gpurun_out/r4_loss_diag3.jsonl
E=gpurun_out/r4_loss_diag3.err
$R --graph on --tag on_fix >> $O 2>> $E || exit 2
$R --tag auto_fix >> $O 2>> $E || exit 3
PTDT_GRAPH_MEMSET_FIX=0 $R --tag auto_nofix >> $O 2>> $E || exit 4
$R --tag auto_fix2 >> $O 2>> $E || exit 5
