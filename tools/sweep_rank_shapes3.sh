#!/bin/bash
# Staged-kernel forms x bundle rows at the N=2 / N=4 per-rank shapes (500k / 250k distinct rows):
# pair + one wave per replica (the sharded default) vs the one-GPU form (one row per step, default
# waves per replica).   Usage (via gpurun): bash tools/sweep_rank_shapes3.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-rank_sweep3}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for n in 2 4; do
  for form in pair1 single0 pair0; do
    for br in 128 192 256 384 512; do
      case $form in
        pair1) E="ERASUREHEAD_STAGED=pair ERASUREHEAD_STAGED_WPR=1";;
        pair0) E="ERASUREHEAD_STAGED=pair";;
        single0) E="ERASUREHEAD_STAGED=1";;
      esac
      env $E ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(form='$form', bundle_rows_env=$br); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('N=$n $form bundle $br:', round(d['kernel_ms'], 4), 'variant', d['variant'])"
    done
  done
done
