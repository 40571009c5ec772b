#!/bin/bash
# Headline bench (1 GPU) + 2-rank IPC rehearsal through the one-command launcher.
# Usage (via gpurun):  bash tools/gpu_bench_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-bench}"
mkdir -p "$OUT"
echo "== bench (1 GPU)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 3; }
tail -c 1500 "$OUT/bench.json"
echo "== bench --gpus 2 (two ranks time-sharing the GPU, IPC mailbox)"
timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 --no-floor --json-out "$OUT/bench_2rank.json" > "$OUT/bench_2rank.log" 2>&1 || { tail -30 "$OUT/bench_2rank.log"; exit 5; }
tail -c 1500 "$OUT/bench_2rank.json"
