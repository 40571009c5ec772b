#!/bin/bash
# GPU tests + smoke + 1-GPU bench + 2/4-rank rehearsals (ranks time-sharing the one GPU over the
# IPC mailbox) through bench.py's one-command launcher.
# Usage (via gpurun):  bash tools/gpu_round_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-round}"
mkdir -p "$OUT"
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 2; }
tail -1 "$OUT/smoke.log"
echo "== bench (1 GPU)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d.get(k) for k in ('ms_per_step','host_driven_ms_per_step','hbm_distinct_TBps','iters_to_loss_floor','eval_s')})"
for n in 2 4; do
  echo "== bench --gpus $n (ranks time-share the GPU)"
  timeout -k 10 600 python bench.py --gpus $n --steps 10 --warmup 3 --no-floor --json-out "$OUT/bench_${n}rank.json" > "$OUT/bench_${n}rank.log" 2>&1 || { tail -30 "$OUT/bench_${n}rank.log"; exit 5; }
  python -c "import json; d=json.load(open('$OUT/bench_${n}rank.json')); print({k: d.get(k) for k in ('ms_per_step','host_driven_ms_per_step','shard')}); [print(r) for r in d['ranks']]"
done
echo "== precision modes (headline shape)"
for p in fp32 bf16; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown --precision $p --json-out "$OUT/bench_$p.json" > "$OUT/bench_$p.log" 2>&1 || { tail -20 "$OUT/bench_$p.log"; exit 6; }
  python -c "import json; d=json.load(open('$OUT/bench_$p.json')); print('$p', round(d['ms_per_step'], 4), 'ms', round(d['hbm_distinct_TBps'], 2), 'TB/s distinct')"
done
echo "== eval profile"
timeout -k 10 300 python tools/profile_eval.py --out "$OUT/eval.json" > "$OUT/eval.log" 2>&1 || { tail -20 "$OUT/eval.log"; exit 7; }
tail -c 700 "$OUT/eval.json"
