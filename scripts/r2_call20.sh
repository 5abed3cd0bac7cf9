set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"
for v in tp mfma; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc20_${v}_$p -o run -- python3 bench.py --model mlp --persist $v --steps 20000 --warmup 1 --no_mlp_side > gpurun_out/pmc20_${v}_$p.log 2>&1 || { echo "pmc $v $p failed"; tail -5 gpurun_out/pmc20_${v}_$p.log; exit 1; }
  done
done
ls -R gpurun_out/pmc20_tp_1 | head
