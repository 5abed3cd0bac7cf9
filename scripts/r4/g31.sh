# BN reductions: guarded last batch (no serial tail loop) -- tests, BN kernel bench and ResNet A/B vs old .so
cd $GRAFT_REPO_ROOT
SO=pytorch_distributed_training_tutorials_amd/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_norm.py tests/test_convbn_gpu.py tests/test_graphs_gpu.py > gpurun_out/r4_bn_tail_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -u benchmarks/bn_kernel_bench.py --iters 20 > gpurun_out/r4_bn_tail_new.jsonl 2>&1 || exit 2
timeout -k 10 200 python3 -u benchmarks/resnet_ddp.py --loss_curve > gpurun_out/r4_bn_tail_resnet_new.log 2>&1 || exit 3
cp $SO /tmp/new.so && cp _ab/old_C.so $SO || exit 4
timeout -k 10 120 python3 -u benchmarks/bn_kernel_bench.py --iters 20 > gpurun_out/r4_bn_tail_old.jsonl 2>&1 || exit 5
timeout -k 10 200 python3 -u benchmarks/resnet_ddp.py --loss_curve > gpurun_out/r4_bn_tail_resnet_old.log 2>&1 || exit 6
cp /tmp/new.so $SO || exit 7
timeout -k 10 200 python3 -u benchmarks/resnet_ddp.py --loss_curve > gpurun_out/r4_bn_tail_resnet_new2.log 2>&1 || exit 8
