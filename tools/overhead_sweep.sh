#!/bin/bash
# Per-round overhead study on one GPU: a small problem (compute ~0.1 ms) run with 1, 2 and 4
# ranks sharing the GPU over the IPC mailbox, so the step time exposes host + transport latency.
# Usage (via gpurun): bash tools/overhead_sweep.sh OUTDIR [n_rows]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-overhead}"
mkdir -p "$OUT"
N=${2:-80000}
: > "$OUT/overhead.jsonl"
for NP in 1 2 4; do
  timeout -k 10 300 python bench.py --gpus "$NP" --n-rows "$N" --steps 200 --warmup 20 --no-floor --device-loop off --json-out "$OUT/ov_$NP.json" > "$OUT/ov_$NP.log" 2>&1 || { tail -20 "$OUT/ov_$NP.log"; exit 1; }
  cat "$OUT/ov_$NP.json" >> "$OUT/overhead.jsonl"
  python -c "
import json; d=json.load(open('$OUT/ov_$NP.json'))
print($NP, d['config']['transport'], 'ms/step', round(d['ms_per_step'], 4), 'host-driven', round(d['host_driven_ms_per_step'], 4))
for r in d['ranks']: print('   ', {k: r[k] for k in r if k.endswith('_us')})"
done
