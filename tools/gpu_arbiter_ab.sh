#!/bin/bash
# Device arbiter (ERASUREHEAD_DEVICE_MASTER=on) vs host-driven master rounds, ranks time-sharing one
# GPU: small problem (host + transport latency exposed) at 2 ranks and the headline at 2 ranks.
# Usage (via gpurun):  bash tools/gpu_arbiter_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-arbiter_ab}"
mkdir -p "$OUT"
show() {
  python -c "
import json; d=json.load(open('$1'))
print('$2', round(d['ms_per_step'], 4), d['config']['round_loop'], 'host-driven', round(d.get('host_driven_ms_per_step') or 0, 4))"
}
for rep in 1 2; do
  for m in off on; do
    ERASUREHEAD_DEVICE_MASTER=$m ERASUREHEAD_WORKER_WAIT=device timeout -k 10 300 python bench.py --gpus 2 --n-rows 80000 --steps 200 --warmup 20 --no-floor --no-breakdown --json-out "$OUT/s2_$m$rep.json" > "$OUT/s2_$m$rep.log" 2>&1 || { tail -30 "$OUT/s2_$m$rep.log"; exit 5; }
    show "$OUT/s2_$m$rep.json" "small N=2 arbiter=$m rep $rep"
  done
done
for m in off on; do
  ERASUREHEAD_DEVICE_MASTER=$m ERASUREHEAD_WORKER_WAIT=device timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 10 --no-floor --no-breakdown --json-out "$OUT/h2_$m.json" > "$OUT/h2_$m.log" 2>&1 || { tail -30 "$OUT/h2_$m.log"; exit 6; }
  show "$OUT/h2_$m.json" "headline N=2 arbiter=$m"
done
