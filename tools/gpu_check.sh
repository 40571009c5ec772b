#!/bin/bash
# One GPU round: kernel/engine tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Usage (via gpurun):  bash tools/gpu_check.sh [steps]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
STEPS=${1:-20}
python tools/build_ext.py > "$OUT/build.log" 2>&1 || { echo "build failed"; tail -20 "$OUT/build.log"; exit 1; }
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=5 > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 2; }
tail -2 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 5 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 3; }
tail -1 "$OUT/bench.log"
echo "== bench, 2 ranks sharing the GPU (IPC transport path)"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-floor --json-out "$OUT/bench_2rank.json" > "$OUT/bench_2rank.log" 2>&1 || { tail -30 "$OUT/bench_2rank.log"; exit 5; }
tail -c 600 "$OUT/bench_2rank.json"
echo "== rocprofv3"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-floor > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 4; }
find "$OUT/prof" -name "*stats*" | head
exit $rc
