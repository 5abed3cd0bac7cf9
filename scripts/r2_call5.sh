set -o pipefail
export PYTHONUNBUFFERED=1
for v in "" "ROC_ACTIVE_WAIT_TIMEOUT=20" "ROC_ACTIVE_WAIT_TIMEOUT=100" "AMD_DIRECT_DISPATCH=0"; do
  echo "== $v" >> gpurun_out/r2_probe5.log
  env $v timeout -k 10 120 python benchmarks/overhead_probe.py 2>&1 | grep '^{"linear": \(1\|20\),\|sync_us' | cut -c1-200 >> gpurun_out/r2_probe5.log || exit 1
  env $v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>&1 | grep '^{' | cut -c100-200 >> gpurun_out/r2_probe5.log || exit 1
done
cat gpurun_out/r2_probe5.log
