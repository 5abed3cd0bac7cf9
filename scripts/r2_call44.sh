#!/bin/bash
# End-of-session validation of the committed tree: full GPU suite, smoke, driver bench (3 fresh
# processes), 2-rank shared-GPU rehearsal of the N>1 path, kernel trace of the driver command, and
# two PMC passes on the TP MLP engine (tools/pmc_table.py).
set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r44_pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r44_smoke.log 2>&1 &&
o=gpurun_out/r44_bench.jsonl && : > $o &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 2>> gpurun_out/r44.err | grep '^{' >> $o || exit 1; done &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --share_gpu --steps 20 --warmup 5 > gpurun_out/r44_share2.log 2>&1 &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --share_gpu --model mlp --steps 5000 --warmup 500 > gpurun_out/r44_share2_mlp.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof44 -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r44_prof.log 2>&1 &&
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_BRANCH" &&
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" &&
timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc44_tp_1 -o run -- python3 bench.py --model mlp --persist tp --steps 20000 --warmup 1 --no_mlp_side > gpurun_out/pmc44_1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc44_tp_2 -o run -- python3 bench.py --model mlp --persist tp --steps 20000 --warmup 1 --no_mlp_side > gpurun_out/pmc44_2.log 2>&1
