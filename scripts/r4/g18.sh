cd $GRAFT_REPO_ROOT
for n in 1 20 200 2000; do
  timeout -k 10 200 python -u bench.py --model mlp --steps $n --warmup 5 --no_ref --out gpurun_out/r4_mlp_steps.jsonl > /dev/null 2>> gpurun_out/r4_mlp_steps.err || exit 1
done
for n in 1 20; do
  timeout -k 10 200 python -u bench.py --steps $n --warmup 5 --no_ref --no_mlp_side --out gpurun_out/r4_lin_steps.jsonl > /dev/null 2>> gpurun_out/r4_mlp_steps.err || exit 2
done
