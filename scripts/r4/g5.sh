# ResNet training-trajectory diagnostic: native (graph off / auto / no shadow / no deferred casts) vs torch
cd $GRAFT_REPO_ROOT
R="timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve --steps 10 --warmup 5"
O=gpurun_out/r4_loss_diag.jsonl
$R --impl torch --pre_steps 24 --tag torch >> $O 2>> gpurun_out/r4_loss_diag.err || exit 1
$R --graph off --pre_steps 24 --tag native_off >> $O 2>> gpurun_out/r4_loss_diag.err || exit 2
$R --tag native_auto >> $O 2>> gpurun_out/r4_loss_diag.err || exit 3
$R --graph off --pre_steps 24 --no_shadow --tag native_noshadow >> $O 2>> gpurun_out/r4_loss_diag.err || exit 4
PTDT_DEFER_GRAD_CAST=0 $R --graph off --pre_steps 24 --tag native_nodefer >> $O 2>> gpurun_out/r4_loss_diag.err || exit 5
