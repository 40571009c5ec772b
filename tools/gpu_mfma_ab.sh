#!/bin/bash
# bf16 MFMA stage geometry A/B (16-row stages / 4-deep ring vs 32-row / 2-deep) after the tests.
# Usage (via gpurun): bash tools/gpu_mfma_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-mfma_ab}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "mfma or transpose or bf16" > "$OUT/pytest.log" 2>&1 || { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
ERASUREHEAD_MFMA_ROWS=32 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "mfma_bf16_replica or bundle_kernel" > "$OUT/pytest32.log" 2>&1 || { grep -E "FAIL|Error" "$OUT/pytest32.log" | head -20; exit 1; }
tail -1 "$OUT/pytest32.log"
B="python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown --precision bf16"
for rows in 32; do
  for br in 512 1024 2048 4096; do
    ERASUREHEAD_MFMA_ROWS=$rows ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 300 $B --json-out "$OUT/r${rows}_b${br}.json" > "$OUT/r${rows}_b${br}.log" 2>&1 || { tail -20 "$OUT/r${rows}_b${br}.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/r${rows}_b${br}.json')); print('stage rows $rows bundle rows $br:', round(d['ms_per_step'], 4), 'ms', round(d['hbm_distinct_TBps'], 2), 'TB/s')"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "fp32" > "$OUT/pytest_fp32.log" 2>&1 || { grep -E "FAIL|Error" "$OUT/pytest_fp32.log" | head -20; exit 3; }
tail -1 "$OUT/pytest_fp32.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown --precision fp32 --json-out "$OUT/fp32.json" > "$OUT/fp32.log" 2>&1 || { tail -20 "$OUT/fp32.log"; exit 4; }
python -c "import json; d=json.load(open('$OUT/fp32.json')); print('fp32 packed:', round(d['ms_per_step'], 4), 'ms', round(d['hbm_distinct_TBps'], 2), 'TB/s')"
