#!/bin/bash
# Worker beta wait on the device (hipStreamWaitValue64, default) vs on the host: multi-process
# GPU tests, then the small-problem overhead runs (host + transport latency exposed) and the
# headline at 2 ranks, each A/B.   Usage (via gpurun):  bash tools/gpu_worker_wait_ab.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-worker_wait}"
mkdir -p "$OUT"
echo "== multi-process GPU tests"
timeout -k 10 600 python -u -m pytest tests/test_multiproc_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_mp.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_mp.log"; [ $rc -ne 0 ] && exit $rc
show() {
  python -c "
import json; d=json.load(open('$1'))
print('$2', round(d['ms_per_step'], 4), 'host-driven', round(d.get('host_driven_ms_per_step') or 0, 4))
for r in d['ranks']: print('   ', {k: r.get(k) for k in ('rank','device_wait','fused_put','kernel_us','msg_put_us','beta_wait_us','wait_k_us','decode_update_us')})"
}
for NP in 2 4; do
  for W in host device; do
    ERASUREHEAD_WORKER_WAIT=$W timeout -k 10 300 python bench.py --gpus $NP --n-rows 80000 --steps 200 --warmup 20 --no-floor --device-loop off --json-out "$OUT/ov${NP}_$W.json" > "$OUT/ov${NP}_$W.log" 2>&1 || { tail -30 "$OUT/ov${NP}_$W.log"; exit 5; }
    show "$OUT/ov${NP}_$W.json" "small N=$NP wait=$W"
  done
done
for W in host device; do
  ERASUREHEAD_WORKER_WAIT=$W timeout -k 10 600 python bench.py --gpus 2 --steps 30 --warmup 5 --no-floor --json-out "$OUT/h2_$W.json" > "$OUT/h2_$W.log" 2>&1 || { tail -30 "$OUT/h2_$W.log"; exit 6; }
  show "$OUT/h2_$W.json" "headline N=2 wait=$W"
done
