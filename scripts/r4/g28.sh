cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_resnet3 -o run -- python3 -u benchmarks/resnet_ddp.py --graph off --steps 10 --warmup 3 > gpurun_out/prof_resnet3.log 2>&1 || exit 1
python3 tools/step_breakdown.py $(ls /tmp/prof_resnet3/*/run_results.db /tmp/prof_resnet3/run_results.db 2>/dev/null | head -1) > gpurun_out/r4_resnet_step_breakdown.md || exit 2
