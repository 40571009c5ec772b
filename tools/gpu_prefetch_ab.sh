#!/bin/bash
# L2 prefetch ahead of the staged LDS ring (ERASUREHEAD_STAGE_PREFETCH=k: issue(t) also touches every
# line of stage t+k) vs none: kernel tests with it on, then the 1-GPU headline and the per-rank shapes.
# Usage: bash tools/gpu_prefetch_ab.sh OUTDIR "K1 K2 ..."
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-prefetch}"
KS=${2:-"0 1 2"}
mkdir -p "$OUT"
ERASUREHEAD_STAGE_PREFETCH=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
: > "$OUT/ab.jsonl"
for rep in 1 2; do
  for k in $KS; do
    ERASUREHEAD_STAGE_PREFETCH=$k timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/n1_k$k.json" > "$OUT/n1.log" 2>&1 || { tail -20 "$OUT/n1.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/n1_k$k.json')); print('rep $rep N=1 fp64 prefetch=$k', round(d['ms_per_step'],4))"
    python -c "import json; d=json.load(open('$OUT/n1_k$k.json')); print(json.dumps(dict(shape='N1_bench', prefetch=$k, rep=$rep, ms=d['ms_per_step'])))" >> "$OUT/ab.jsonl"
    for n in 2 4 8; do
      ERASUREHEAD_STAGE_PREFETCH=$k timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(prefetch=$k, rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('   N=$n prefetch=$k:', round(d['kernel_ms'], 4))"
    done
  done
done
