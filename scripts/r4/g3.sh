cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/bin/graph_memset_repro > gpurun_out/memset_repro.txt 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/resnet_interleave.py --variants eager,interleave,interleave_raw,graph --tail 10 > gpurun_out/il_nondet3.jsonl 2> gpurun_out/il_nondet3.err || exit 2
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_convbn_gpu.py tests/test_graphs_gpu.py tests/test_llm_int8.py tests/test_grad_sink.py tests/test_norm.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_g3.log 2>&1 || exit 3
for i in 1 2 3; do timeout -k 10 200 python -u benchmarks/resnet_ddp.py --tag fix$i >> gpurun_out/r4_resnet_fix2.jsonl 2>> gpurun_out/r4_resnet_fix2.err || exit 4; done
timeout -k 10 200 python -u benchmarks/int8_bench.py --shapes 16x11008x4096,1x11008x4096,32x4096x4096,16x4096x11008 > gpurun_out/int8_decode_bench.jsonl 2> gpurun_out/int8_decode_bench.err || exit 5
timeout -k 10 300 python -u benchmarks/capture_free_audit.py > gpurun_out/cfa.json 2> gpurun_out/cfa.err || exit 6
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_big" -p no:cacheprovider --no-header --tb=short > gpurun_out/t_gemm3.log 2>&1 || exit 7
timeout -k 10 200 python -u benchmarks/gemm_bench.py --shapes 4096x4096x4096,8192x8192x8192,4096x11008x4096 --extra_sched 2 3 --splits 2 > gpurun_out/gemm_p8.jsonl 2> gpurun_out/gemm_p8.err || exit 8
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_xgmi_gpu.py -k "two_ranks or pair" -p no:cacheprovider --no-header --tb=short > gpurun_out/t_pair.log 2>&1 || exit 9
S="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --share_gpu --steps 20000 --warmup 2000 --no_ref --no_mlp_side"
for i in 1 2; do
  PTDT_XGMI_PAIR=0 timeout -k 10 200 $S --out gpurun_out/share2_pair_ab.jsonl > /dev/null 2>> gpurun_out/share2_pair_ab.err || exit 10
  PTDT_XGMI_PAIR=1 timeout -k 10 200 $S --out gpurun_out/share2_pair_ab.jsonl > /dev/null 2>> gpurun_out/share2_pair_ab.err || exit 11
done
