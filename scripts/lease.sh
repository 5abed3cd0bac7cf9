#!/bin/bash
# One parameterised GPU-lease script (replaces the per-call scripts of earlier rounds).
#
#   gpurun --timeout 1200 -- bash scripts/lease.sh STAGE [STAGE ...]
#
# Every GPU step runs under its own `timeout -k 10`, output goes to gpurun_out/<tag>_<step>.*,
# and the first failing step ends the script (no retries, nothing more on the GPU after a
# fault / abort / time limit). TAG (env, default "l") prefixes every output file.
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
T=${TAG:-l}
O=gpurun_out
PORT=$((29500 + RANDOM % 1000))
PF=0

step() {  # name secs cmd...   (stdout+stderr -> $O/$T_name.log)
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/${T}_$name.log" 2>&1
  local c=$?
  echo "=== $name exit $c"; tail -4 "$O/${T}_$name.log"
  [ $c -eq 0 ] || { echo "STOP after $name (exit $c)"; exit $c; }
}
tstep() {  # like step, but test failures (exit 1) do not end the script; crashes/timeouts do
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/${T}_$name.log" 2>&1
  local c=$?
  echo "=== $name exit $c"; tail -4 "$O/${T}_$name.log"
  [ $c -eq 0 ] || [ $c -eq 1 ] || { echo "STOP after $name (exit $c)"; exit $c; }
}
jstep() {  # name secs cmd...   (JSON lines appended to $O/$T_name.jsonl, the rest to .err)
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" 2>> "$O/${T}_$name.err" | grep '^{' >> "$O/${T}_$name.jsonl"
  local c=$?
  echo "=== $name exit $c"; tail -c 600 "$O/${T}_$name.jsonl"; echo
  [ $c -eq 0 ] || { echo "STOP after $name (exit $c)"; tail -20 "$O/${T}_$name.err"; exit $c; }
}
share() {  # name N bench-args...   (N ranks share cuda:0: protocol rehearsal, not a scaling number)
  local name=$1 n=$2; shift 2
  PORT=$((PORT + 1))
  jstep "$name" 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $PORT bench.py --gpus "$n" --share_gpu "$@"
}
prof() {  # name secs cmd...   (kernel trace + stats under $O/prof_$T_name)
  local name=$1 secs=$2; shift 2
  step "prof_$name" "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_${T}_$name" -o run -- "$@"
}
pmc() {  # name "counters" cmd...   (one counter pass; kill hard on a hang)
  local name=$1 ctr=$2; shift 2
  echo "=== pmc_$name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$O/pmc_${T}_$name" -o run -- "$@" \
    > "$O/${T}_pmc_$name.log" 2>&1
  local c=$?
  echo "=== pmc_$name exit $c"; tail -3 "$O/${T}_pmc_$name.log"
  [ $c -eq 0 ] || exit $c
}
PYTEST="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"

for s in "$@"; do
  case $s in
    tests)     tstep pytest_gpu 1000 python3 -u -m pytest -q -rf --timeout 120 --timeout-method thread tests -m gpu ;;
    tests:*)   tstep pytest_sel 600 python3 -u -m pytest -q -rf --timeout 120 --timeout-method thread ${s#tests:} ;;
    smoke)     step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    driver)    for i in 1 2 3; do jstep bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5; done ;;
    rehab)     # A/B of the warm-up split (PTDT_BENCH_REHEARSALS), interleaved, headline only
               for i in 1 2 3; do for r in 1 2 3; do
                 jstep rehab 120 env PTDT_BENCH_REHEARSALS=$r python3 bench.py --steps 20 --warmup 5 --no_ref --no_mlp_side
               done; done ;;
    rehab2)    # A/B of 3 vs 5 rehearsal launches, interleaved, headline only
               for i in 1 2 3 4 5 6; do for r in 3 5; do
                 jstep rehab2 120 env PTDT_BENCH_REHEARSALS=$r python3 bench.py --steps 20 --warmup 5 --no_ref --no_mlp_side
               done; done ;;
    pinab)     # A/B: default vs the persistent launches pinned to one CU (PTDT_BENCH_PIN_CU), interleaved
               for i in 1 2 3 4; do
                 jstep pinab 120 python3 bench.py --steps 20 --warmup 5 --no_ref --no_mlp_side
                 jstep pinab 120 env PTDT_BENCH_PIN_CU=0 python3 bench.py --steps 20 --warmup 5 --no_ref --no_mlp_side
               done ;;
    default)   jstep bench_default 300 python3 bench.py ;;
    tp20k)     # toy-MLP TP engine, bf16 and fp32, long launch
               for dt in bf16 fp32; do jstep tp20k 300 python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 2000 --no_ref; done ;;
    hl20k)     # headline engine alone, long launch: per-step cost without the fixed part
               for r in 1 2; do jstep hl20k 300 python3 bench.py --steps 20000 --warmup 2000 --no_ref --no_mlp_side; done ;;
    stamps)    jstep stamps 300 python3 bench.py --steps 20000 --warmup 2000 --stamps --no_mlp_side
               jstep stamps 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --stamps ;;
    share)     share share 2 --steps 20000 --warmup 2000 --stamps --no_mlp_side
               share share 4 --steps 20000 --warmup 2000 --stamps --no_mlp_side
               share share 2 --model mlp --steps 20000 --warmup 2000 --stamps
               share share 4 --model mlp --steps 5000 --warmup 500 --stamps ;;
    wstamps)   # single-wave engine phase split (diagnostic build, tools/bin/_C_stamps.so) at W = 1, 2, 4
               export PTDT_EXT_PATH=$PWD/tools/bin/_C_stamps.so
               jstep wstamps 300 python3 bench.py --steps 20000 --warmup 2000 --stamps --no_mlp_side --no_ref
               share wstamps 2 --steps 20000 --warmup 2000 --stamps --no_mlp_side
               share wstamps 4 --steps 20000 --warmup 2000 --stamps --no_mlp_side
               unset PTDT_EXT_PATH ;;
    tpab)      # A/B of this tree vs tools/bin/_C_base.so (an earlier commit's build), shared-GPU rehearsals, interleaved
               for r in 1 2; do for W in 2 4 8; do
                 share tpab_cur $W --model mlp --steps 2000 --warmup 200 --no_ref
                 export PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so
                 share tpab_base $W --model mlp --steps 2000 --warmup 200 --no_ref
                 unset PTDT_EXT_PATH
               done; done ;;
    bnab)      # BN kernels + ResNet-50 step: this tree vs tools/bin/_C_base.so, interleaved
               for r in 1 2; do
                 jstep bnab_cur 180 python3 benchmarks/bn_kernel_bench.py
                 jstep bnab_base 180 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 benchmarks/bn_kernel_bench.py
               done ;;
    resab)     for r in 1 2; do
                 jstep resab_cur 600 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5
                 jstep resab_base 600 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5
               done ;;
    linab)     # single-wave engine exchange: this tree vs tools/bin/_C_base.so, shared-GPU rehearsals, interleaved
               for r in 1 2; do for W in 2 4 8; do
                 share linab_cur $W --steps 2000 --warmup 200 --no_ref --no_mlp_side
                 export PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so
                 share linab_base $W --steps 2000 --warmup 200 --no_ref --no_mlp_side
                 unset PTDT_EXT_PATH
               done; done ;;
    pfab)      # wave-engine prefetch depth: this tree (3) vs tools/bin/_C_pf2.so (2), driver command + 20k steps
               for r in 1 2 3 4; do
                 jstep pfab_3 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
                 jstep pfab_2 120 env PTDT_EXT_PATH=$PWD/tools/bin/_C_pf2.so python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
               done
               for r in 1 2; do
                 jstep pfab20k_3 300 python3 bench.py --steps 20000 --warmup 2000 --no_ref --no_mlp_side
                 jstep pfab20k_2 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_pf2.so python3 bench.py --steps 20000 --warmup 2000 --no_ref --no_mlp_side
               done ;;
    llab)      # single-wave chunked exchange poll loop: this tree vs tools/bin/_C_{nosleep,llpipe}.so, W = 4, 8
               for r in 1 2; do for W in 4 8; do
                 share llab_base $W --steps 2000 --warmup 200 --no_ref --no_mlp_side
                 for v in nosleep llpipe; do
                   export PTDT_EXT_PATH=$PWD/tools/bin/_C_$v.so
                   share llab_$v $W --steps 2000 --warmup 200 --no_ref --no_mlp_side
                   unset PTDT_EXT_PATH
                 done
               done; done ;;
    wsab)      # single-wave engine phase split (stamps builds): this tree vs tools/bin/_C_stamps_base.so, W = 2, 4
               for W in 2 4; do
                 export PTDT_EXT_PATH=$PWD/tools/bin/_C_stamps.so
                 share wsab_cur $W --steps 2000 --warmup 200 --stamps --no_mlp_side
                 export PTDT_EXT_PATH=$PWD/tools/bin/_C_stamps_base.so
                 share wsab_base $W --steps 2000 --warmup 200 --stamps --no_mlp_side
                 unset PTDT_EXT_PATH
               done ;;
    firstab)   # driver command with / without the host-planned first rows (PTDT_NO_FIRST_ROWS), interleaved
               for r in 1 2 3; do
                 jstep first_on 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
                 jstep first_off 300 env PTDT_NO_FIRST_ROWS=1 python3 bench.py --gpus 1 --steps 20 --warmup 5
               done ;;
    sprep)     step sprep 300 python3 tools/stream_pipeline_repeat.py 25 ;;
    sprep_r4)  step sprep_r4 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_r4.so python3 tools/stream_pipeline_repeat.py 25 ;;
    sprep_nl)  step sprep_nl 300 env PTDT_BN_FENCE=1 python3 tools/stream_pipeline_repeat.py 10 ;;
    linshare)  for W in 2 4 8; do share linshare $W --steps 2000 --warmup 200 --no_ref; done ;;
    share_fused) share share_fused 2 --engine fused --steps 2000 --warmup 200
               share share_fused 4 --engine fused --model mlp --steps 2000 --warmup 200 ;;
    engines)   jstep engines 300 python3 bench.py --engine fused --steps 2000 --warmup 200
               jstep engines 300 python3 bench.py --engine fused --steps 2000 --warmup 200 --allreduce rccl
               jstep engines 300 python3 bench.py --engine autograd --steps 300 --warmup 50
               jstep engines 300 python3 bench.py --engine reference --steps 300 --warmup 50 ;;
    apps)      step mp_toy 300 python3 model_parallel.py toy
               step mp_resnet 600 python3 model_parallel.py resnet --repeat 5 --json $O/${T}_mp_resnet.json --fig $O/${T}_mp_vs_single.png
               step dp_toy 300 python3 data_parallel.py --quiet ;;
    int8)      jstep int8 300 python3 benchmarks/int8_bench.py ;;
    probe)     jstep probe 300 python3 benchmarks/pipeline_stream_probe.py ;;
    exch)      step exch 120 bash -c "tools/bin/exchange_bench > $O/${T}_exchange.jsonl" ;;
    resnet)    jstep resnet_ddp 600 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5
               jstep resnet_ddp 600 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5 --impl torch ;;
    prof_resnet) prof resnet 600 python3 benchmarks/resnet_ddp.py --steps 3 --warmup 2 ;;
    tl0)       # round-5 fixed-cost baseline: prologue split + kernel/HIP-API trace of the driver command
               jstep tl0_stamps 300 python3 bench.py --steps 20 --warmup 5 --stamps --no_mlp_side --no_ref
               step prof_tl0 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d "$O/prof_${T}_tl0" -o run -- python3 bench.py --steps 20 --warmup 5 --no_mlp_side --no_ref ;;
    tl)        jstep timeline 300 python3 tools/driver_timeline.py ;;
    tlpin)     jstep tlpin 300 python3 tools/driver_timeline.py --variants bench,pinned,bench,pinned,nostamp ;;
    memset)    jstep memset_probe 600 python3 benchmarks/graph_memset_probe.py ;;
    memsyn)    jstep memset_syn 300 python3 benchmarks/graph_memset_probe.py --synthetic ;;
    memtrace)  step prof_memtrace 600 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_${T}_memtrace" -o run -- python3 benchmarks/graph_memset_probe.py --trace_only
               timeout -k 5 120 python3 tools/graph_replay_order.py "$O/prof_${T}_memtrace/run_kernel_trace.csv" \
                 > "$O/${T}_replay_order.txt" 2>&1; echo "replay_order exit $?"; tail -5 "$O/${T}_replay_order.txt"
               rm -rf "$O/prof_${T}_memtrace" ;;  # ~200k dispatches (MIOpen find): too big to copy back
    mlpstamps) jstep mlpstamps 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --stamps --no_ref ;;
    profdrv)   prof drvonly 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side ;;
    prof)      prof driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
               prof reference 300 python3 bench.py --engine reference --steps 200 --warmup 20 ;;
    tppmcab)   # TP engine PMC per step: this tree vs tools/bin/_C_r4.so (round-4 build), two passes each
               for side in cur r4; do
                 [ $side = r4 ] && export PTDT_EXT_PATH=$PWD/tools/bin/_C_r4.so
                 pmc tp_${side}_1 "$P1" python3 bench.py --model mlp --steps 20000 --warmup 1 --no_mlp_side --no_ref
                 pmc tp_${side}_2 "$P2" python3 bench.py --model mlp --steps 20000 --warmup 1 --no_mlp_side --no_ref
                 unset PTDT_EXT_PATH
               done
               python3 tools/pmc_table.py --steps 20000 cur=$O/pmc_${T}_tp_cur_1,$O/pmc_${T}_tp_cur_2 \
                 r4=$O/pmc_${T}_tp_r4_1,$O/pmc_${T}_tp_r4_2 > $O/${T}_tppmc.txt 2>&1
               cat $O/${T}_tppmc.txt
               rm -rf $O/pmc_${T}_tp_* ;;
    tpbfpmc)   # TP engine PMC per step: bf16 operands vs exact fp32 (same tree), two passes each
               for dt in bf16 fp32; do
                 pmc tp_${dt}_1 "$P1" python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 1 --no_ref
                 pmc tp_${dt}_2 "$P2" python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 1 --no_ref
               done
               python3 tools/pmc_table.py --steps 20000 bf16=$O/pmc_${T}_tp_bf16_1,$O/pmc_${T}_tp_bf16_2 \
                 fp32=$O/pmc_${T}_tp_fp32_1,$O/pmc_${T}_tp_fp32_2 > $O/${T}_tpbfpmc.txt 2>&1
               cat $O/${T}_tpbfpmc.txt
               rm -rf $O/pmc_${T}_tp_* ;;
    tpbfab)    # TP engine at W = 1: bf16 vs fp32 operands, interleaved, plus one phase-timer run each
               for r in 1 2 3; do
                 jstep tpbf_bf16 300 python3 bench.py --model mlp --dtype bf16 --steps 20000 --warmup 2000 --no_ref
                 jstep tpbf_fp32 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref
               done
               jstep tpbf_stamps 300 python3 bench.py --model mlp --dtype bf16 --steps 20000 --warmup 2000 --no_ref --stamps
               jstep tpbf_stamps 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref --stamps ;;
    intab)     # driver command: ROCr interrupt-signalled completion (default) vs polled (HSA_ENABLE_INTERRUPT=0)
               for r in 1 2 3; do
                 jstep intab_default 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
                 jstep intab_polled 300 env HSA_ENABLE_INTERRUPT=0 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
               done ;;
    tpvar)     # TP engine at W = 1: this tree vs tools/bin/_C_$VAR.so (build_variant.py), bf16 + fp32,
               # interleaved, then one phase-timer run of each
               for r in 1 2; do
                 for dt in bf16 fp32; do
                   jstep tpvar_base 300 python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 2000 --no_ref
                   jstep tpvar_$VAR 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_$VAR.so python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 2000 --no_ref
                 done
               done
               for dt in bf16 fp32; do
                 jstep tpvar_base_st 300 python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 2000 --no_ref --stamps
                 jstep tpvar_${VAR}_st 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_$VAR.so python3 bench.py --model mlp --dtype $dt --steps 20000 --warmup 2000 --no_ref --stamps
               done ;;
    tpshare)   # TP engine exchange rehearsal: W ranks sharing cuda:0, fp32 and bf16 (TPW: world sizes)
               for w in ${TPW:-2 4 8}; do
                 for dt in ${TPDT:-fp32 bf16}; do
                   share tpshare_$dt $w --model mlp --dtype $dt --steps 2000 --warmup 200 --no_mlp_side
                 done
               done ;;
    tpw1ab)    # TP engine at W = 1, this tree vs the round-4 build, interleaved
               for r in 1 2; do
                 jstep tpw1_cur 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref
                 jstep tpw1_r4 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_r4.so python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref
               done ;;
    tpw1base)  # TP engine at W = 1, this tree vs tools/bin/_C_base.so, interleaved
               for r in 1 2 3; do
                 jstep tpw1_cur 300 python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref
                 jstep tpw1_base 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 bench.py --model mlp --steps 20000 --warmup 2000 --no_ref
               done ;;
    drvab)     # driver command + 20,000-step headline: this tree vs tools/bin/_C_base.so, interleaved
               for r in 1 2 3; do
                 jstep drvab_cur 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
                 jstep drvab_base 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref --no_mlp_side
               done
               for r in 1 2; do
                 jstep drvab_cur 300 python3 bench.py --steps 20000 --warmup 2000 --no_ref --no_mlp_side
                 jstep drvab_base 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 bench.py --steps 20000 --warmup 2000 --no_ref --no_mlp_side
               done ;;
    sideab)    # driver command incl. the toy-MLP side measurement: this tree vs tools/bin/_C_base.so
               for r in 1 2 3 4; do
                 jstep sideab_cur 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref
                 jstep sideab_base 300 env PTDT_EXT_PATH=$PWD/tools/bin/_C_base.so python3 bench.py --gpus 1 --steps 20 --warmup 5 --no_ref
               done ;;
    pmc_tp)    pmc tp1 "$P1" python3 bench.py --model mlp --persist tp --steps 20000 --warmup 1 --no_mlp_side
               pmc tp2 "$P2" python3 bench.py --model mlp --persist tp --steps 20000 --warmup 1 --no_mlp_side ;;
    wavepmc)   # single-wave engine PMC per step (two passes) + table, then the pass directories removed
               pmc wave_1 "$P1" python3 bench.py --steps 20000 --warmup 1 --no_mlp_side --no_ref
               pmc wave_2 "$P2" python3 bench.py --steps 20000 --warmup 1 --no_mlp_side --no_ref
               python3 tools/pmc_table.py --steps 20000 wave=$O/pmc_${T}_wave_1,$O/pmc_${T}_wave_2 > $O/${T}_wavepmc.txt 2>&1
               cat $O/${T}_wavepmc.txt
               rm -rf $O/pmc_${T}_wave_* ;;
    pmc_wave)  pmc wave1 "$P1" python3 bench.py --steps 20000 --warmup 1 --no_mlp_side
               pmc wave2 "$P2" python3 bench.py --steps 20000 --warmup 1 --no_mlp_side ;;
    bnsweep)   # BN kernel geometry / sweep-direction sweep (benchmarks/bn_kernel_bench.py), one process per setting
               for cfg in ${BNCFGS:-"PTDT_BN_DIR=0" "PTDT_BN_DIR=10" "PTDT_BN_DIR=5" "PTDT_BN_DIR=2" "PTDT_BN_DIR=8" "PTDT_BN_TC=8"}; do
                 jstep bnk 120 env ${cfg//,/ } python3 benchmarks/bn_kernel_bench.py
               done ;;
    resdir)    # ResNet-50 DDP step under each BN sweep-direction setting
               for d in ${BNDIRS:-0 10 5}; do
                 jstep resnet_dir 600 env PTDT_BN_DIR=$d python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5
               done ;;
    resgraph)  # ResNet-50 DDP: whole-step hipGraph (default) vs eager launches, same box
               jstep resnet_graph 600 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5 --graph on
               jstep resnet_graph 600 python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5 --graph off ;;
    resenv)    # ResNet-50 DDP under MIOpen solver switches (RESENVS: space-separated VAR=V[,VAR=V] sets)
               for cfg in ${RESENVS:-"X=0"}; do
                 jstep resnet_env 600 env ${cfg//,/ } python3 benchmarks/resnet_ddp.py --steps 20 --warmup 5 --tag "$cfg"
               done ;;
    bntest)    # BN numerics under non-default geometry
               tstep pytest_bn 300 env PTDT_BN_DIR=15 PTDT_BN_AU=4 PTDT_BN_APPLY_BLOCKS=0 $PYTEST tests/test_norm.py ;;
    run:*)     step "run" 600 bash -c "${s#run:}" ;;
    pyfail:*)  # one pytest selection whose failure report is printed to stdout (gpurun's tail)
               PF=$((PF + 1)); L="$O/${T}_pyfail$PF.log"
               timeout -k 10 600 python3 -u -m pytest -q -rf --timeout 120 --timeout-method thread ${s#pyfail:} \
                 > "$L" 2>&1; c=$?; grep -E "^E  |^FAILED|passed|failed" "$L" | head -30
               echo "pyfail$PF exit $c"; [ $c -le 1 ] || [ $c -eq 5 ] || exit $c ;;  # ad-hoc: run:'python3 benchmarks/x.py'
    *)         echo "unknown stage $s"; exit 2 ;;
  esac
done
echo "=== done"
