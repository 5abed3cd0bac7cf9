cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u benchmarks/capture_free_audit.py > gpurun_out/cfa.json 2> gpurun_out/cfa.err
R="timeout -k 10 200 python -u benchmarks/graph_state_diff.py --batch 128 --image 224 --nondet"
PTDT_BN_FENCE=1 $R --eager 4 > gpurun_out/gsd_fence.jsonl 2> gpurun_out/gsd_fence.err || exit 1
PTDT_CONVBN=off PTDT_BN_POOL=0 PTDT_PAD_RGB=0 $R --eager 4 > gpurun_out/gsd_alloff.jsonl 2> gpurun_out/gsd_alloff.err || exit 2
$R --eager 1 > gpurun_out/gsd_e1.jsonl 2> gpurun_out/gsd_e1.err || exit 3
AMD_SERIALIZE_KERNEL=3 $R --eager 4 > gpurun_out/gsd_serial.jsonl 2> gpurun_out/gsd_serial.err || exit 4
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_llm_int8.py tests/test_grad_sink.py -p no:cacheprovider --no-header --tb=short > gpurun_out/t_int8_sink.log 2>&1 || exit 6
timeout -k 10 200 python -u benchmarks/int8_bench.py --shapes 16x11008x4096,1x11008x4096,32x4096x4096,16x4096x11008 > gpurun_out/int8_decode_bench.jsonl 2> gpurun_out/int8_decode_bench.err || exit 7
