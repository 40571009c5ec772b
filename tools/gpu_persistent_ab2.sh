#!/bin/bash
# Persistent staged grid, second look: what the occupancy query gives, a forced 4 workgroups per CU,
# and finer bundles at the sharded rank shapes.   Usage (via gpurun): bash tools/gpu_persistent_ab2.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-persistent2}"
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python tools/bench_rank_shapes.py --one $N > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
  grep -h "persistent staged grid" "$OUT/one.err" | head -1
  python -c "import json; d=json.load(open('$OUT/one.json')); d.update(tag='$tag'); print(json.dumps(d))" >> "$OUT/ab.jsonl"
  python -c "import json; d=json.load(open('$OUT/one.json')); print('N=$N $tag:', round(d['kernel_ms'], 4))"
}
for N in 1 2 4 8; do
  run static
  run pers_api ERASUREHEAD_PERSISTENT=1 ERASUREHEAD_PERSISTENT_VERBOSE=1
  run pers_4cu ERASUREHEAD_PERSISTENT=1 ERASUREHEAD_PERSISTENT_PER_CU=4
  if [ $N -gt 1 ]; then
    for br in 64 96; do
      run "static_b$br" ERASUREHEAD_BUNDLE_ROWS=$br
      run "pers_4cu_b$br" ERASUREHEAD_PERSISTENT=1 ERASUREHEAD_PERSISTENT_PER_CU=4 ERASUREHEAD_BUNDLE_ROWS=$br
    done
  fi
done
