# HBM bandwidth of the int8 decode kernels: packed vs row-major GEMV weights (FETCH_SIZE / WRITE_SIZE passes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R="python3 -u benchmarks/int8_bench.py --shapes 16x11008x4096 --rounds 1"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pf -o run -- $R > gpurun_out/pmc_i8_1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pw -o run -- $R > gpurun_out/pmc_i8_2.log 2>&1 || exit 2
export PTDT_I8_PACKED=0
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/rf -o run -- $R > gpurun_out/pmc_i8_3.log 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/rw -o run -- $R > gpurun_out/pmc_i8_4.log 2>&1 || exit 4
{ echo "## packed weights"; python3 tools/pmc_bandwidth.py /tmp/pf /tmp/pw --match "i8_decode|Cijk_Alik_Bljk_HHS"; echo; echo "## row-major weights (PTDT_I8_PACKED=0)"; python3 tools/pmc_bandwidth.py /tmp/rf /tmp/rw --match "i8_decode|Cijk_Alik_Bljk_HHS"; } > gpurun_out/r4_pmc_int8_decode.md || exit 5
