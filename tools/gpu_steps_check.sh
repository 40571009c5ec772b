#!/bin/bash
# Headline step time at the default 20 timed steps vs 50 (fixed per-run costs inside the timed
# region show up as a gap), plus the engine GPU tests.  Usage: bash tools/gpu_steps_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-steps}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for K in 20 50 20 50; do
  for m in stream off; do
    timeout -k 10 300 python bench.py --steps $K --warmup 5 --no-floor --no-breakdown --device-loop $m --json-out "$OUT/k$K$m.json" > "$OUT/k$K$m.log" 2>&1 || { tail -20 "$OUT/k$K$m.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/k$K$m.json')); print('steps $K $m', round(d['ms_per_step'],4), d['phases_us'])"
  done
done
