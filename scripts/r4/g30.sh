# Per-shape durations of the native BN kernels (bn_kernel_bench, B = 128); geometry knob A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d /tmp/bnk -o run -- python3 -u benchmarks/bn_kernel_bench.py --iters 10 > gpurun_out/r4_bnk.log 2>&1 || exit 1
python3 tools/kernel_grid_stats.py /tmp/bnk --match "bn_" > gpurun_out/r4_bn_grid.md || exit 2
