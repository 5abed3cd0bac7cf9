# driver-command kernel trace + PMC bandwidth of the fused conv1x1 backward and the int8 decode GEMV
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver -o run -- python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/prof_driver.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_convbwd_fetch -o run -- python3 -u -m pytest -x -q tests/test_convbn_gpu.py -k "conv1x1_bwd_matches" -p no:cacheprovider > gpurun_out/pmc_convbwd_fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_convbwd_write -o run -- python3 -u -m pytest -x -q tests/test_convbn_gpu.py -k "conv1x1_bwd_matches" -p no:cacheprovider > gpurun_out/pmc_convbwd_write.log 2>&1 || exit 3
