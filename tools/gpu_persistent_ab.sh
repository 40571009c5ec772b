#!/bin/bash
# Persistent staged workgroups (ERASUREHEAD_PERSISTENT=1, default) vs one bundle per workgroup:
# kernel/engine GPU tests, the 1-GPU headline (fp64, fp32) and the per-rank shapes at N=2/4/8 with
# a few bundle sizes.   Usage (via gpurun):  bash tools/gpu_persistent_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-persistent}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
: > "$OUT/shapes.jsonl"
for rep in 1 2; do
  for P in 0 1; do
    for p in fp64 fp32; do
      ERASUREHEAD_PERSISTENT=$P timeout -k 10 300 python bench.py --precision $p --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/n1_${p}_p$P.json" > "$OUT/n1.log" 2>&1 || { tail -20 "$OUT/n1.log"; exit 2; }
      python -c "import json; d=json.load(open('$OUT/n1_${p}_p$P.json')); print('rep $rep N=1 $p persistent=$P', round(d['ms_per_step'],4))"
    done
  done
done
for n in 2 4 8; do
  for br in 128 256 512; do
    for P in 0 1; do
      ERASUREHEAD_PERSISTENT=$P ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(persistent=$P, bundle_rows_env=$br); print(json.dumps(d))" >> "$OUT/shapes.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('N=$n bundle $br persistent=$P:', round(d['kernel_ms'], 4))"
    done
  done
done
