set -o pipefail
export PYTHONUNBUFFERED=1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_dp_mp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests25.log 2>&1 && \
timeout -k 10 400 python model_parallel.py resnet --repeat 5 --split_sizes 20 --json gpurun_out/r2_mp25.json > gpurun_out/r2_mp25.log 2>&1 && \
timeout -k 10 400 python model_parallel.py resnet --repeat 5 --split_sizes 20 --channels_last --json gpurun_out/r2_mp25_cl.json > gpurun_out/r2_mp25_cl.log 2>&1
rc=$?; tail -2 gpurun_out/r2_gputests25.log
for f in gpurun_out/r2_mp25.json gpurun_out/r2_mp25_cl.json; do [ -f $f ] && python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'); [print(' ', k, round(v['mean_s'],4), round(v['img_per_s'],1)) for k,v in d.items()]"; done
exit $rc
