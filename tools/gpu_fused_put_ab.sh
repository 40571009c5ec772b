#!/bin/bash
# Worker message put fused into the final slab reduction (ERASUREHEAD_FUSED_PUT, default on)
# vs the separate put_signal kernel: multi-process GPU tests, then 2/4-rank rehearsals A/B.
# Usage (via gpurun):  bash tools/gpu_fused_put_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-fused_put}"
mkdir -p "$OUT"
echo "== multi-process GPU tests"
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_mp.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_mp.log"; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  for f in 0 1; do
    ERASUREHEAD_FUSED_PUT=$f timeout -k 10 600 python bench.py --gpus $n --steps 30 --warmup 5 --no-floor --json-out "$OUT/b${n}_f$f.json" > "$OUT/b${n}_f$f.log" 2>&1 || { tail -30 "$OUT/b${n}_f$f.log"; exit 5; }
    python -c "import json; d=json.load(open('$OUT/b${n}_f$f.json')); print('N=$n fused=$f', round(d['ms_per_step'],4)); [print('  ', {k: r.get(k) for k in ('rank','fused_put','kernel_us','msg_put_us','beta_wait_us','wait_k_us')}) for r in d['ranks']]"
  done
done
