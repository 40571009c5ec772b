#!/bin/bash
# fp32-compute sigmoid on the hardware exp2 / reciprocal: kernel + engine GPU tests, then the
# fp32 and bf16 headline.   Usage (via gpurun):  bash tools/gpu_fastsig_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-fastsig}"
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for p in fp32 bf16 fp32; do
  timeout -k 10 300 python bench.py --precision $p --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/$p.json" > "$OUT/$p.log" 2>&1 || { tail -20 "$OUT/$p.log"; exit 2; }
  python -c "import json; d=json.load(open('$OUT/$p.json')); print('$p', round(d['ms_per_step'],4), 'ms', round(d['hbm_distinct_TBps'],2), 'TB/s')"
done
