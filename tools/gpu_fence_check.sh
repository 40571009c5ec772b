#!/bin/bash
# Headline bench (1 GPU and 2 ranks) + engine GPU tests.  Usage: bash tools/gpu_fence_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-fence}"
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-floor --json-out "$OUT/bench2.json" > "$OUT/bench2.log" 2>&1 || { tail -20 "$OUT/bench2.log"; exit 2; }
for f in bench bench2; do
  python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'],4), d.get('host_driven_ms_per_step'), d['phases_us'])"
done
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; exit $rc
