#!/bin/bash
# One-wave replica bundles (ERASUREHEAD_STAGED=multi, grad_dense_multi) vs the default LDS-staged
# bundles: kernel tests, then the fp64/fp32 headline (50 steps) and the 2/4/8-GPU rank shapes for
# a few bundle lengths.  Usage: bash tools/gpu_multi_ab.sh OUTDIR "ROWS1 ROWS2 ..."
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-multi}"
ROWS=${2:-"128 256 512"}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "one_wave or staged or bundle" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
echo "kernel tests: $(tail -1 "$OUT/pytest.log")"
: > "$OUT/ab.jsonl"
one() {  # label, env...
  local label=$1; shift
  for p in fp64 fp32; do
    env "$@" timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --precision $p --json-out "$OUT/n1.json" > "$OUT/n1.log" 2>&1 || { tail -20 "$OUT/n1.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/n1.json')); print(json.dumps(dict(shape='N1_$p', label='$label', rep=$rep, ms=round(d['ms_per_step'],4))))" | tee -a "$OUT/ab.jsonl"
  done
  for n in 2 8; do
    env "$@" timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
    python -c "import json; d=json.load(open('$OUT/one.json')); d.update(label='$label', rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
    python -c "import json; d=json.load(open('$OUT/one.json')); print('   N=$n $label:', round(d['kernel_ms'], 4))"
  done
}
for rep in 1 2; do
  one default ERASUREHEAD_AB=0
  for r in $ROWS; do
    one multi$r ERASUREHEAD_STAGED=multi ERASUREHEAD_BUNDLE_ROWS=$r
  done
done
