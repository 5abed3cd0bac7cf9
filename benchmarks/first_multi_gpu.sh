#!/bin/bash
# First run on a multi-GPU node: for N = 1, 2, 4, 8 visible GPUs, one JSON line per N
# with what is needed to trust (or diagnose) the scaling numbers:
#   RCCL rank count, peer-access matrix, xGMI one-shot self-test result (and why not),
#   the bench's engine / all-reduce / any fallback taken and why, per-rank start skew, the
#   driver-command throughput and E(N) = S(N) / (N * S(1)).
# Usage: benchmarks/first_multi_gpu.sh [steps] [warmup]   (defaults: the driver's 20 / 5)
# Every GPU step has its own time limit. A step that fails with an ordinary error (a test / bench error
# line, exit 1-4) is recorded and the script goes on to the next N; a crash, abort or time limit
# (exit >= 124: 124 timeout, 134 abort, 137 kill, 139 segfault) ends it -- nothing more runs on a GPU
# that may be in a bad state.
cd "$(dirname "$0")/.." || exit 2
STEPS=${1:-20}; WARM=${2:-5}
export PYTHONUNBUFFERED=1
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
OUT=$(mktemp -d)
run() {  # log secs cmd...: run one GPU step; echo its exit code; stop the script on a crash / time limit
  local log=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local c=$?
  echo "$c" > "$log.rc"
  if [ "$c" -ne 0 ]; then
    tail -5 "$log"
    if [ "$c" -ge 124 ]; then echo "stopping: exit $c (crash / abort / time limit)"; STOP=1; fi
  fi
  return 0
}
STOP=0
for N in 1 2 4 8; do
  [ "$STOP" -eq 1 ] && break
  [ "$N" -gt "$NGPU" ] && break
  PORT=$((29600 + N))
  if [ "$N" -eq 1 ]; then
    run "$OUT/probe_$N.log" 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $PORT benchmarks/multi_gpu_probe.py
    [ "$STOP" -eq 1 ] && break
    run "$OUT/bench_$N.log" 600 python3 bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM"
  else
    run "$OUT/probe_$N.log" 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $PORT benchmarks/multi_gpu_probe.py
    [ "$STOP" -eq 1 ] && break
    run "$OUT/bench_$N.log" 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
      --master-addr 127.0.0.1 --master-port $((PORT + 10)) bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM"
  fi
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
out = sys.argv[1]
def last_json(path):
    if not os.path.exists(path):
        return {}
    rows = []
    for l in open(path, errors="replace"):
        if '{"' in l:
            try:
                rows.append(json.loads(l[l.index('{"'):]))
            except ValueError:
                pass
    return rows[-1] if rows else {}
def rc(path):
    try:
        return int(open(path + ".rc").read())
    except (OSError, ValueError):
        return None
def tail(path, n=3):
    try:
        return [l.rstrip()[:300] for l in open(path, errors="replace").readlines()[-n:]]
    except OSError:
        return None
res = {}
for p in sorted(glob.glob(os.path.join(out, "bench_*.log"))):
    n = int(p.rsplit("_", 1)[1].split(".")[0])
    b, pr = last_json(p), last_json(os.path.join(out, f"probe_{n}.log"))
    res[n] = {"n_gpus": n, "rccl_ranks": pr.get("rccl_ranks"), "peer_access": pr.get("peer_access"),
              "xgmi_ok": pr.get("xgmi_ok"), "xgmi_why": pr.get("xgmi_why"),
              "barrier_skew_us": pr.get("barrier_skew_us"), "allreduce_84B_us": pr.get("allreduce_84B_us"),
              "samples_per_s": b.get("value"), "us_per_step": (b.get("ms_per_step") or 0) * 1e3,
              "engine": b.get("persistent_engine") or b.get("config", {}).get("engine"),
              "allreduce": b.get("allreduce"), "fallback": b.get("fallback"),
              "replicas_in_sync": b.get("replicas_in_sync"),
              "start_skew_us": b.get("timing", {}).get("headline", {}).get("start_skew_us"),
              "window_us": b.get("timing", {}).get("headline", {}).get("window_us"),
              "engine_path": b.get("engine_path"), "error": b.get("error") or b.get("incomplete"),
              "probe_rc": rc(os.path.join(out, f"probe_{n}.log")), "bench_rc": rc(p),
              "bench_tail": tail(p) if rc(p) else None}
s1 = res.get(1, {}).get("samples_per_s")
for n in sorted(res):
    r = res[n]
    r["efficiency"] = round(r["samples_per_s"] / (n * s1), 3) if (s1 and r["samples_per_s"]) else None
    print(json.dumps({"what": "first_multi_gpu", **r}))
PY
