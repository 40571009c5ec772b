#!/bin/bash
# Second staged-geometry sweep at the N=8 / N=4 per-rank shapes (pair form, one wave per replica):
# rows per stage x ring depth x bundle rows.   Usage (via gpurun): bash tools/sweep_rank_shapes2.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-rank_sweep2}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for n in 8 4; do
  for cfg in "2 2" "4 2" "2 3" "4 3" "6 2"; do
    set -- $cfg
    for br in 96 128 192; do
      ERASUREHEAD_STAGED_WPR=1 ERASUREHEAD_STAGED=pair ERASUREHEAD_STAGE_ROWS=$1 ERASUREHEAD_STAGES=$2 ERASUREHEAD_BUNDLE_ROWS=$br \
        timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(stage_rows=$1, stages=$2, bundle_rows_env=$br); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('N=$n rows $1 stages $2 bundle $br:', round(d['kernel_ms'], 4))"
    done
  done
done
echo "== one-GPU headline, one wave per replica for every bundle (R=2 bundles default to two)"
for p in fp64 fp32; do
  for w in 0 1; do
    if [ "$w" = 1 ]; then export ERASUREHEAD_STAGED_WPR=1; else unset ERASUREHEAD_STAGED_WPR; fi
    unset ERASUREHEAD_STAGED ERASUREHEAD_STAGE_ROWS ERASUREHEAD_STAGES ERASUREHEAD_BUNDLE_ROWS
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown --precision $p --json-out "$OUT/n1_${p}_w$w.json" > "$OUT/n1_${p}_w$w.log" 2>&1 || { tail -5 "$OUT/n1_${p}_w$w.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/n1_${p}_w$w.json')); print('N=1 $p wpr_forced=$w:', round(d['ms_per_step'], 4))"
  done
done
