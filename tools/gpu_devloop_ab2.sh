#!/bin/bash
# Device-driven (stream / graph) vs host-driven rounds at the headline, alternated 3x.
# Usage (via gpurun):  bash tools/gpu_devloop_ab2.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-devloop_ab2}"
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for rep in 1 2 3; do
  for m in off stream graph; do
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --device-loop $m --json-out "$OUT/$m$rep.json" > "$OUT/$m$rep.log" 2>&1 || { tail -20 "$OUT/$m$rep.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$m$rep.json')); print(json.dumps({'mode':'$m','rep':$rep,'ms':d['ms_per_step'],'phases':d['phases_us']}))" | tee -a "$OUT/ab.jsonl"
  done
done
