set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2_resnet16.jsonl; : > $o
timeout -k 10 300 python -u -m pytest tests/test_grad_sink.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gputests16.log 2>&1 && \
timeout -k 10 420 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 >> $o 2> gpurun_out/r2_resnet16_a.err && \
timeout -k 10 300 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 --no_shadow >> $o 2> gpurun_out/r2_resnet16_b.err && \
PTDT_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof16a -o resnet -- python3 benchmarks/resnet_ddp.py --steps 4 --warmup 3 >> $o 2> gpurun_out/r2_resnet16_c.err && \
PTDT_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof16b -o resnet -- python3 benchmarks/resnet_ddp.py --steps 4 --warmup 3 --bucket_cap_mb 25 >> $o 2> gpurun_out/r2_resnet16_d.err
rc=$?; tail -2 gpurun_out/r2_gputests16.log; cat $o | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['ms_per_step'], d['value'], d.get('buckets_MB'))"
exit $rc
