#!/bin/bash
# fp32 staged-bundle geometry sweep at the headline shape (rows per stage x ring depth x waves per replica).
# Usage (via gpurun): bash tools/sweep_fp32_staged.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-fp32_sweep}"
mkdir -p "$OUT"
: > "$OUT/sweep.txt"
for wpr in 1 2; do
for rows in 2 4 8; do
  for st in 2 3 4; do
    ERASUREHEAD_STAGED_WPR=$wpr ERASUREHEAD_STAGE_ROWS=$rows ERASUREHEAD_STAGES=$st timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown --precision fp32 --json-out "$OUT/w${wpr}_r${rows}_s${st}.json" > "$OUT/w${wpr}_r${rows}_s${st}.log" 2>&1 || { tail -5 "$OUT/w${wpr}_r${rows}_s${st}.log"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/w${wpr}_r${rows}_s${st}.json')); print('wpr $wpr rows $rows stages $st:', round(d['ms_per_step'], 4), 'ms')" | tee -a "$OUT/sweep.txt"
  done
done
done
