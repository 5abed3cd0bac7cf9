#!/bin/bash
# First run on a multi-GPU node: for N = 1, 2, 4, 8 visible GPUs, one JSON line per N
# with what is needed to trust (or diagnose) the scaling numbers:
#   RCCL rank count, peer-access matrix, xGMI one-shot self-test result (and why not),
#   the bench's engine / all-reduce / any fallback taken and why, per-rank start skew, the
#   driver-command throughput and E(N) = S(N) / (N * S(1)).
# Usage: benchmarks/first_multi_gpu.sh [steps] [warmup]   (defaults: the driver's 20 / 5)
# Every GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.." || exit 2
STEPS=${1:-20}; WARM=${2:-5}
export PYTHONUNBUFFERED=1
NGPU=$(python3 -c "import torch; print(torch.cuda.device_count())")
OUT=$(mktemp -d)
for N in 1 2 4 8; do
  [ "$N" -gt "$NGPU" ] && break
  PORT=$((29600 + N))
  if [ "$N" -eq 1 ]; then
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $PORT benchmarks/multi_gpu_probe.py > "$OUT/probe_$N.log" 2>&1 || { tail -20 "$OUT/probe_$N.log"; exit 1; }
    timeout -k 10 600 python3 bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM" > "$OUT/bench_$N.log" 2>&1 \
      || { tail -20 "$OUT/bench_$N.log"; exit 1; }
  else
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $PORT benchmarks/multi_gpu_probe.py > "$OUT/probe_$N.log" 2>&1 || { tail -20 "$OUT/probe_$N.log"; exit 1; }
    timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((PORT + 10)) bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM" > "$OUT/bench_$N.log" 2>&1 \
      || { tail -20 "$OUT/bench_$N.log"; exit 1; }
  fi
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
out = sys.argv[1]
def last_json(path):
    rows = [json.loads(l) for l in open(path) if l.startswith("{")]
    return rows[-1] if rows else {}
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
              "error": b.get("error")}
s1 = res.get(1, {}).get("samples_per_s")
for n in sorted(res):
    r = res[n]
    r["efficiency"] = round(r["samples_per_s"] / (n * s1), 3) if (s1 and r["samples_per_s"]) else None
    print(json.dumps({"what": "first_multi_gpu", **r}))
PY
