#!/bin/bash
# GPU validation: tests, smoke, short bench runs, rocprofv3 stats.
# Each GPU step has its own time limit; a crash/timeout (exit >= 124 or signal)
# stops the script, plain test failures (exit 1) do not.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { local c=$1; [ "$c" -eq 0 ] || [ "$c" -eq 1 ]; }
step() {  # name, seconds, cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local c=$?
  echo "=== $name exit $c"; tail -5 "gpurun_out/$name.log"
  if ! ok $c; then echo "STOP after $name (exit $c)"; exit $c; fi
}
STAGES=${STAGES:-"tests smoke bench prof"}
for s in $STAGES; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -rf ;;
    micro) step microbench 120 tools/bin/microbench_launch
           step microbench_isa 120 tools/bin/microbench_isa ;;
    xgmi)  step xgmi_latency 300 python benchmarks/xgmi_step_latency.py --steps 20000 ;;
    quick) step bench_persistent 300 python bench.py --steps 20000 --warmup 2000 --stamps
           step bench_persistent_wg 300 python bench.py --steps 20000 --warmup 2000 --stamps --persist workgroup
           step bench_mlp 300 python bench.py --model mlp --steps 20000 --warmup 2000 --stamps
           step bench_fused 300 python bench.py --engine fused --steps 2000 --warmup 200 ;;
    apps)  step mp_toy 300 python model_parallel.py toy
           step mp_resnet 600 python model_parallel.py resnet --repeat 5 --json gpurun_out/mp_resnet.json --fig gpurun_out/mp_vs_single.png
           step dp_toy 300 python data_parallel.py --quiet
           step resnet_ddp_native 600 python benchmarks/resnet_ddp.py --steps 20 --warmup 5
           step resnet_ddp_torch 600 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 --impl torch ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_persistent 300 python bench.py --steps 20000 --warmup 2000
           step bench_fused 300 python bench.py --engine fused --steps 2000 --warmup 200
           step bench_fused_rccl 300 python bench.py --engine fused --steps 2000 --warmup 200 --allreduce rccl
           step bench_autograd 300 python bench.py --engine autograd --steps 300 --warmup 50
           step bench_reference 300 python bench.py --engine reference --steps 300 --warmup 50
           step bench_mlp 300 python bench.py --model mlp --steps 20000 --warmup 2000
           step bench_mlp_fused 300 python bench.py --engine fused --model mlp --steps 2000 --warmup 200 ;;
    prof)  step prof_persistent 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_persistent -o run -- python3 bench.py --steps 20000 --warmup 2000
           step prof_fused 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused -o run -- python3 bench.py --engine fused --steps 500 --warmup 64
           step prof_fused_rccl 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fused_rccl -o run -- python3 bench.py --engine fused --steps 500 --warmup 64 --allreduce rccl
           step prof_mlp 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python3 bench.py --model mlp --steps 500 --warmup 64
           step prof_reference 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_reference -o run -- python3 bench.py --engine reference --steps 200 --warmup 20 ;;
    pmc)   step pmc_list 120 rocprofv3 -L
           step pmc_wave 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --stats --output-format csv -d gpurun_out/pmc_wave -o run -- python3 bench.py --steps 8192 --warmup 64 ;;
  esac
done
echo "=== done"
