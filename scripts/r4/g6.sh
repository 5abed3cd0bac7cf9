# replay-first state diff: K replays right after capture vs K eager steps from the same snapshot
cd $GRAFT_REPO_ROOT
R="timeout -k 10 200 python -u benchmarks/graph_state_diff.py --replays 4"
O=gpurun_out/r4_replay_diff.jsonl
E=gpurun_out/r4_replay_diff.err
$R --batch 128 --image 224 --nondet >> $O 2>> $E || exit 1
PTDT_DEFER_GRAD_CAST=0 $R --batch 128 --image 224 --nondet >> $O 2>> $E || exit 2
$R --batch 128 --image 224 >> $O 2>> $E || exit 3
$R --batch 32 --image 128 --nondet >> $O 2>> $E || exit 4
PTDT_CONVBN=off PTDT_BN_POOL=0 PTDT_PAD_RGB=0 $R --batch 128 --image 224 --nondet >> $O 2>> $E || exit 5
