#!/bin/bash
# Stage-walk rotation (ERASUREHEAD_STAGE_ROTATE=k: bundle b starts at stage (b*k) mod stages) vs none:
# kernel tests with it on, then the 1-GPU headline and the per-rank shapes.  Usage: bash tools/gpu_rotate_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-rotate}"
mkdir -p "$OUT"
ERASUREHEAD_STAGE_ROTATE=37 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
: > "$OUT/ab.jsonl"
for rep in 1 2; do
  for k in 0 37; do
    ERASUREHEAD_STAGE_ROTATE=$k timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/n1_k$k.json" > "$OUT/n1.log" 2>&1 || { tail -20 "$OUT/n1.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/n1_k$k.json')); print('rep $rep N=1 fp64 rotate=$k', round(d['ms_per_step'],4))"
    for cfg in "2 128" "2 512" "4 128" "8 128"; do
      set -- $cfg
      ERASUREHEAD_STAGE_ROTATE=$k ERASUREHEAD_BUNDLE_ROWS=$2 timeout -k 10 120 python tools/bench_rank_shapes.py --one $1 > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(rotate=$k, bundle_rows_env=$2, rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('   N=$1 bundle $2 rotate=$k:', round(d['kernel_ms'], 4))"
    done
  done
done
