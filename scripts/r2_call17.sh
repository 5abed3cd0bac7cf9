set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python benchmarks/tp_shape_sweep.py > gpurun_out/r2_tpsweep17.log 2>&1
rc=$?; grep -v "^$" gpurun_out/r2_tpsweep17.log | tail -20; exit $rc
