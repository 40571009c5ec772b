#!/bin/bash
# A/B of one staged-kernel env knob: kernel tests with the first non-zero value on, then the 1-GPU
# headline (fp64, 50 steps; fp32 too) and the per-rank shapes of the 2/4/8-GPU placement, two reps.
# Usage: bash tools/gpu_env_ab.sh OUTDIR VAR "V1 V2 ..."     e.g. ... early ERASUREHEAD_STAGE_EARLY "0 1"
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-env_ab}"
VAR=$2
VALS=${3:-"0 1"}
mkdir -p "$OUT"
ON=$(for v in $VALS; do [ "$v" != 0 ] && { echo $v; break; }; done)
env $VAR=$ON timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
echo "$VAR=$ON: $(tail -1 "$OUT/pytest.log")"
: > "$OUT/ab.jsonl"
for rep in 1 2; do
  for v in $VALS; do
    for p in fp64 fp32; do
      env $VAR=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-floor --no-breakdown --precision $p --json-out "$OUT/n1.json" > "$OUT/n1.log" 2>&1 || { tail -20 "$OUT/n1.log"; exit 2; }
      python -c "import json; d=json.load(open('$OUT/n1.json')); print(json.dumps(dict(shape='N1_bench_$p', value='$v', rep=$rep, ms=d['ms_per_step'])))" | tee -a "$OUT/ab.jsonl"
    done
    for n in 2 4 8; do
      env $VAR=$v timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 3; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(value='$v', rep=$rep); print(json.dumps(d))" >> "$OUT/ab.jsonl"
      python -c "import json; d=json.load(open('$OUT/one.json')); print('   N=$n $VAR=$v:', round(d['kernel_ms'], 4))"
    done
  done
done
