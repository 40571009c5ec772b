#!/bin/bash
# Bundle rows sized to fill the chip's workgroup slots in whole waves at the sharded per-rank shapes
# (one partition = 125k rows: 123 rows -> 1017 bundles for 1024 slots; 128 -> 977).
# Usage (via gpurun): bash tools/sweep_bundle_fill.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-bundle_fill}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for rep in 1 2; do
for n in 8 4 2; do
  for br in 116 120 122 123 124 126 128; do
    ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/one.json')); d.update(bundle_rows_env=$br, rep=$rep); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
    python -c "import json; d=json.load(open('$OUT/one.json')); print('rep $rep N=$n bundle $br: ntasks', d['ntasks'], round(d['kernel_ms'], 4))"
  done
done
done
