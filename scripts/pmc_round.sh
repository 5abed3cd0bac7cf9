#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per counter group, kernel-trace only).
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
pass() {  # name, counters, cmd...
  local name=$1 ctr=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc_$name -o run -- "$@" \
    > gpurun_out/pmc_$name.log 2>&1
  local c=$?
  echo "=== $name exit $c"; tail -3 gpurun_out/pmc_$name.log
  [ $c -eq 0 ] || exit $c
}
[ -n "$LIST" ] && { timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1; echo "list exit $?"; }
GEMM="python3 benchmarks/gemm_bench.py --shapes 4096x4096x4096 --rounds 1"
for p in ${PASSES:-gemm}; do
  case $p in
    gemm) pass gemm_sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" $GEMM
          pass gemm_lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT" $GEMM
          pass gemm_mem "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" $GEMM ;;
    wave) W="python3 bench.py --steps 20000 --warmup 2000"
          pass wave_sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" $W
          pass wave_mem "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT" $W ;;
    mlp)  M="python3 bench.py --model mlp --steps 5000 --warmup 500"
          pass mlp_sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" $M
          pass mlp_lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_BRANCH" $M ;;
    bn)   N="python3 benchmarks/bn_bench.py --iters 5"
          pass bn_fetch "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" $N
          pass bn_write "WRITE_SIZE" $N
          pass bn_sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" $N ;;
  esac
done
echo "=== done"
