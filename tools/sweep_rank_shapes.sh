#!/bin/bash
# Staged-bundle geometry sweep for the per-rank shapes of the N-GPU headline (fp64).
# Usage (via gpurun): bash tools/sweep_rank_shapes.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-rank_sweep}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for n in 8 4 2; do
  for cfg in "1 2 1" "1 2 pair" "2 4 1" "2 4 pair" "1 4 1" "2 8 1"; do
    set -- $cfg
    for br in 64 128 256; do
      ERASUREHEAD_STAGED_WPR=$1 ERASUREHEAD_STAGE_ROWS=$2 ERASUREHEAD_STAGED=$3 ERASUREHEAD_BUNDLE_ROWS=$br \
        timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(wpr=$1, stage_rows=$2, staged='$3', bundle_rows_env=$br); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('N=$n wpr $1 rows $2 mode $3 bundle $br:', round(d['kernel_ms'], 4))"
    done
  done
done
