#!/bin/bash
# One-launch slab reduction (last-block counters, fused worker put): kernel / engine / multi-process
# GPU tests, then the headline and a 2-rank rehearsal.  Usage: bash tools/gpu_reduce_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-reduce}"
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/b1.json" > "$OUT/b1.log" 2>&1 || { tail -20 "$OUT/b1.log"; exit 2; }
timeout -k 10 300 python bench.py --gpus 2 --steps 30 --warmup 5 --no-floor --json-out "$OUT/b2.json" > "$OUT/b2.log" 2>&1 || { tail -20 "$OUT/b2.log"; exit 3; }
for f in b1 b2; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'],4), d['phases_us'])"; done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python "$ROOT/bench.py" --steps 30 --warmup 5 --no-floor --no-breakdown > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 4; }
f=$(ls "$OUT"/prof/*kernel_stats.csv | head -1); head -8 "$f" | cut -c1-160
