#!/bin/bash
# Weak-scaling sweep of the flagship benchmark on one node (N = 1, 2, 4, 8 GPUs).
# Prints one JSON line per N and the scaling efficiency E(N) = S(N) / (N * S(1)).
# Usage: benchmarks/scaling_sweep.sh [steps] [warmup] [extra bench.py args...]
cd "$(dirname "$0")/.." || exit 2
STEPS=${1:-20000}; WARM=${2:-2000}; shift 2 2>/dev/null
NGPU=$(python -c "import torch; print(torch.cuda.device_count())")
OUT=$(mktemp)
for N in 1 2 4 8; do
  [ "$N" -gt "$NGPU" ] && break
  if [ "$N" -eq 1 ]; then
    timeout -k 10 600 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM" "$@" | tee -a "$OUT" || exit $?
  else
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port $((29500 + N)) bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM" "$@" | tee -a "$OUT" || exit $?
  fi
done
python - "$OUT" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
s1 = next((r["value"] for r in rows if r["n_gpus"] == 1), None)
for r in rows:
    eff = r["value"] / (r["n_gpus"] * s1) if s1 else float("nan")
    print(f"N={r['n_gpus']}: {r['value']:.0f} samples/s, {r['ms_per_step']*1e3:.2f} us/step, efficiency {eff:.3f}")
PY
