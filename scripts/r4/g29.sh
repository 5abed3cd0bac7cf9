# HBM bandwidth of the native ResNet-50 kernels (FETCH_SIZE / WRITE_SIZE passes, summarised on the box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python3 -u benchmarks/resnet_ddp.py --graph off --steps 3 --warmup 2 --pre_steps 0"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_f -o run -- $R > gpurun_out/pmc_bw_f.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pmc_w -o run -- $R > gpurun_out/pmc_bw_w.log 2>&1 || exit 2
python3 tools/pmc_bandwidth.py /tmp/pmc_f /tmp/pmc_w --match "ptdt::" > gpurun_out/r4_pmc_bandwidth.md || exit 3
