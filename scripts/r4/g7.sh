cd $GRAFT_REPO_ROOT
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve --steps 10 --warmup 5"
O=gpurun_out/r4_loss_diag2.jsonl
E=gpurun_out/r4_loss_diag2.err
$R --graph on --tag on >> $O 2>> $E || exit 1
$R --tag auto_a >> $O 2>> $E || exit 2
$R --tag auto_b >> $O 2>> $E || exit 3
$R --deterministic --tag auto_det >> $O 2>> $E || exit 4
$R --deterministic --graph off --pre_steps 24 --tag off_det >> $O 2>> $E || exit 5
