#!/bin/bash
# Replica-bundle kernel per dense scheme over a long timed window: the default choice vs the
# LDS-staged bundles (ERASUREHEAD_STAGED=1) and one-wave bundles (ERASUREHEAD_STAGED=multi) for
# AGC s=2 k=6, cyclic s=2 and FRC s=1 at the headline shape, 95 timed rounds after 5 warm-up
# rounds (the suite's window), alternating, two repetitions.  Usage: bash tools/gpu_scheme_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-scheme_ab}"
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for rep in 1 2; do
  for sch in "agc:--coded-ver 3 --stragglers 2 --num-collect 6" "cyclic:--coded-ver 0 --stragglers 2" "frc:--coded-ver 1 --stragglers 1"; do
    name=${sch%%:*}; args=${sch#*:}
    for k in default 1 multi; do
      if [ $k = default ]; then E="ERASUREHEAD_AB=0"; else E="ERASUREHEAD_STAGED=$k"; fi
      env $E timeout -k 10 300 python bench.py $args --steps 95 --warmup 5 --no-floor --no-breakdown --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 2; }
      python -c "import json; d=json.load(open('$OUT/b.json')); print(json.dumps(dict(scheme='$name', kernel='$k', rep=$rep, ms=round(d['ms_per_step'],4))))" | tee -a "$OUT/ab.jsonl"
    done
  done
done
