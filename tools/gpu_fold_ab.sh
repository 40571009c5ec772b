#!/bin/bash
# One-wave bundles with and without the workgroup fold (ERASUREHEAD_MULTI_FOLD): kernel tests, the
# rank shapes (kernel + slab reduction per round) at N = 1/2/4/8 fp64 and fp32 N=1 bundle rows.
# Usage: bash tools/gpu_fold_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-fold_ab}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "one_wave or staged or bundle" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
echo "kernel tests: $(tail -1 "$OUT/pytest.log")"
: > "$OUT/ab.jsonl"
for rep in 1 2; do
  for n in 1 2 4 8; do
    for f in 0 1; do
      ERASUREHEAD_MULTI_FOLD=$f timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(fold=$f, rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('rep $rep fp64 N=$n fold=$f:', round(d['kernel_ms'], 4), 'rows', d['bundle_rows'])"
    done
  done
  for r in 256 384 512; do
    ERASUREHEAD_BUNDLE_ROWS=$r timeout -k 10 120 python tools/bench_rank_shapes.py --one 1 --precision fp32 > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
    python -c "import json; d=json.load(open('$OUT/one.json')); d.update(fold=1, rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
    python -c "import json; d=json.load(open('$OUT/one.json')); print('rep $rep fp32 N=1 fold rows $r:', round(d['kernel_ms'], 4), 'variant', d['variant'])"
  done
done
