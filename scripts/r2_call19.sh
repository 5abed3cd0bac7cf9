set -o pipefail
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2_resnet19.jsonl; : > $o
timeout -k 10 300 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 >> $o 2> gpurun_out/r2_resnet19_a.err && \
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 >> $o 2> gpurun_out/r2_resnet19_b.err && \
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python benchmarks/resnet_ddp.py --steps 20 --warmup 5 >> $o 2> gpurun_out/r2_resnet19_c.err
rc=$?; cat $o | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['ms_per_step'], d['value'])"
exit $rc
