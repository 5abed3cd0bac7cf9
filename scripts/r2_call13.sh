set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2_sched13.log; : > $out
for kv in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "PTDT_DEVICE_SCHED=1" "PTDT_DEVICE_SCHED=2" "PTDT_DEVICE_SCHED=1 HIP_FORCE_DEV_KERNARG=1"; do
  echo "== $kv" >> $out
  env $kv timeout -k 10 120 python benchmarks/overhead_probe.py > gpurun_out/_p.log 2>&1 || { echo "probe failed: $kv"; cat gpurun_out/_p.log | tail -5; exit 1; }
  tail -1 gpurun_out/_p.log >> $out
  for r in 1 2 3; do
    env $kv timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no_mlp_side > gpurun_out/_b.log 2>&1 || { echo "bench failed: $kv"; tail -5 gpurun_out/_b.log; exit 1; }
    grep '^{' gpurun_out/_b.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench us/step', round(d['ms_per_step']*1e3,3))" >> $out
  done
done
cat $out
