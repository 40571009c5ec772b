#!/bin/bash
# Bundle length of the one-wave replica bundles (ERASUREHEAD_STAGED=multi) at each N-GPU rank shape
# (tools/bench_rank_shapes.py --one N), against the default kernel at that shape.  Two repetitions.
# Usage: bash tools/sweep_multi_rows.sh OUTDIR "N:ROWS,ROWS N:ROWS ..."   (PREC=fp32 for fp32 rows)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-multi_rows}"
SPEC=${2:-"1:512,768,1024 2:256,384 4:128,192,256 8:32,48,64"}
PREC=${PREC:-fp64}
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for rep in 1 2; do
  for item in $SPEC; do
    n=${item%%:*}
    for r in default ${item#*:}; do
      r=${r//,/ }
      for rr in $r; do
        if [ "$rr" = default ]; then E="ERASUREHEAD_AB=0"; else E="ERASUREHEAD_STAGED=multi ERASUREHEAD_BUNDLE_ROWS=$rr"; fi
        env $E timeout -k 10 120 python tools/bench_rank_shapes.py --one $n --precision $PREC > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
        python -c "import json; d=json.load(open('$OUT/one.json')); d.update(label='$rr', rep=$rep, prec='$PREC'); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
        python -c "import json; d=json.load(open('$OUT/one.json')); print('rep $rep $PREC N=$n rows $rr:', round(d['kernel_ms'], 4))"
      done
    done
  done
done
