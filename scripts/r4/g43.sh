# End-of-session validation: full GPU suite, smoke, default bench, ResNet loss-curve run
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --no-header --tb=short > gpurun_out/t_all43.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke43.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/bench43.json 2> gpurun_out/bench43.err || exit 3
timeout -k 10 200 python -u benchmarks/resnet_ddp.py --loss_curve > gpurun_out/resnet43.log 2>&1 || exit 4
