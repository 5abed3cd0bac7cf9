cd $GRAFT_REPO_ROOT
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_graphs_gpu.py -p no:cacheprovider --no-header --tb=short > gpurun_out/tg_after.log 2>&1 || exit 1
PTDT_CONVBN=on timeout -k 10 200 python -u benchmarks/resnet_interleave.py --batch 32 --image 128 --deterministic --variants eager,interleave,graph --tail 10 > gpurun_out/il_det2.jsonl 2> gpurun_out/il_det2.err || exit 2
timeout -k 10 300 python -u benchmarks/resnet_interleave.py --variants eager,interleave,graph --tail 10 > gpurun_out/il_nondet2.jsonl 2> gpurun_out/il_nondet2.err || exit 3
for i in 1 2 3; do timeout -k 10 200 python -u benchmarks/resnet_ddp.py --tag fix$i >> gpurun_out/r4_resnet_fix.jsonl 2>> gpurun_out/r4_resnet_fix.err || exit 4; done
for n in 2 8; do timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) bench.py --gpus $n --steps 20 --warmup 5 --share_gpu --no_mlp_side >> gpurun_out/r4_share_skew.jsonl 2>> gpurun_out/r4_share_skew.err || exit 5; done
