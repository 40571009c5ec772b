#!/bin/bash
# Quick perf snapshot of the current tree: one-wave/staged kernel tests, AGC / cyclic / FRC headline
# rounds over 95 timed steps, and the 1/2/4/8-GPU rank shapes.  Usage: bash tools/gpu_quick_perf.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-quick_perf}"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "one_wave or staged or bundle or dense" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
echo "kernel tests: $(tail -1 "$OUT/pytest.log")"
: > "$OUT/perf.jsonl"
for rep in 1 2; do
  for sch in "agc:--coded-ver 3 --stragglers 2 --num-collect 6" "cyclic:--coded-ver 0 --stragglers 2" "frc:--coded-ver 1 --stragglers 1"; do
    name=${sch%%:*}; args=${sch#*:}
    timeout -k 10 300 python bench.py $args --steps 95 --warmup 5 --no-floor --no-breakdown --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 2; }
    python -c "import json; d=json.load(open('$OUT/b.json')); print(json.dumps(dict(scheme='$name', rep=$rep, ms=round(d['ms_per_step'],4))))" | tee -a "$OUT/perf.jsonl"
  done
  for n in 1 2 4 8; do
    timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
    python -c "import json; d=json.load(open('$OUT/one.json')); d.update(rep=$rep); print(json.dumps(d))" >> "$OUT/perf.jsonl"
    python -c "import json; d=json.load(open('$OUT/one.json')); print('rep $rep N=$n:', round(d['kernel_ms'], 4), 'variant', d['variant'])"
  done
done
