set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof_probe -o probe -- python3 benchmarks/overhead_probe.py > gpurun_out/r2_probe2.log 2>&1
rc=$?; tail -12 gpurun_out/r2_probe2.log; find gpurun_out/r2_prof_probe -name '*.csv' | head; exit $rc
