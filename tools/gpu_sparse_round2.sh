#!/bin/bash
# Sparse evaluation kernel + amazon-scale checks on one GPU.
# Usage (via gpurun): bash tools/gpu_sparse_round2.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-sparse2}"
mkdir -p "$OUT"
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sparse or amazon" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
echo "== sparse eval bench"
timeout -k 10 300 python tools/bench_sparse_eval.py --out "$OUT/sparse_eval.jsonl" > "$OUT/sparse_eval.log" 2>&1 || { tail -30 "$OUT/sparse_eval.log"; exit 2; }
cat "$OUT/sparse_eval.jsonl"
echo "== suite rows (sparse stand-ins)"
timeout -k 10 600 python tools/bench_suite.py --only agc_amazon,agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k6 --out "$OUT/suite" > "$OUT/suite.log" 2>&1 || { tail -30 "$OUT/suite.log"; exit 3; }
cat "$OUT/suite/suite.md"
echo "== amazon over 2 ranks (IPC, time-sharing the GPU)"
timeout -k 10 300 python tools/rank_breakdown.py --gpus 2 --data amazon --json-out "$OUT/amazon_2rank.json" > "$OUT/amazon_2rank.log" 2>&1 || { tail -30 "$OUT/amazon_2rank.log"; exit 4; }
cat "$OUT/amazon_2rank.json"
