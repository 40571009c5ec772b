#!/bin/bash
# Per-round overhead study on one GPU: a small problem (compute ~0.1-0.3 ms) run with 1, 2 and 4
# ranks sharing the GPU over the IPC mailbox, so the step time exposes host + transport latency.
# Usage (via gpurun): bash tools/overhead_sweep.sh [n_rows]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
N=${1:-80000}
: > "$OUT/overhead.jsonl"
for NP in 1 2 4; do
  if [ "$NP" = 1 ]; then
    timeout -k 10 300 python bench.py --n-rows "$N" --steps 100 --warmup 10 --no-floor --json-out "$OUT/ov_$NP.json" > "$OUT/ov_$NP.log" 2>&1 || { tail -20 "$OUT/ov_$NP.log"; exit 1; }
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NP" --master-addr 127.0.0.1 --master-port $((29600 + NP)) bench.py --gpus "$NP" --n-rows "$N" --steps 100 --warmup 10 --no-floor --json-out "$OUT/ov_$NP.json" > "$OUT/ov_$NP.log" 2>&1 || { tail -20 "$OUT/ov_$NP.log"; exit 1; }
  fi
  cat "$OUT/ov_$NP.json" >> "$OUT/overhead.jsonl"
  python -c "import json;d=json.load(open('$OUT/ov_$NP.json'));print($NP, d['config']['transport'], round(d['ms_per_step'],4), d['phases_us'])"
done
