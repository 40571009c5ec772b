#!/bin/bash
# rocprofv3 kernel statistics of the current tree: the 1-GPU headline (fp64, 20 timed rounds, no
# convergence runs), the same through the 2-rank one-GPU rehearsal, and the heaviest rank of the
# 8-GPU placement (tools/bench_rank_shapes.py --one 8).  Usage: bash tools/gpu_prof_round3.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-prof3}"
mkdir -p "$OUT"
run() {  # name, command...
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- "$@" > "$OUT/$name.log" 2>&1) || { tail -20 "$OUT/$name.log"; exit 3; }
  local f=$(find "$OUT/$name" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$OUT/${name}_kernel_stats.csv"
  echo "== $name"; head -6 "$f" | cut -d, -f1-8
}
run n1 python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-floor --no-breakdown --json-out "$OUT/n1.json"
run n8_rank python3 "$ROOT/tools/bench_rank_shapes.py" --one 8
run n1_bf16 python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-floor --no-breakdown --precision bf16 --json-out "$OUT/n1_bf16.json"
