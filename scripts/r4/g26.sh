cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no_ref --no_mlp_side --stamps --out gpurun_out/r4_lin_prologue.jsonl > /dev/null 2>> gpurun_out/r4_lin_prologue.err || exit 1
done
