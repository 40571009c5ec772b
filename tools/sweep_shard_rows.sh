#!/bin/bash
# Bundle rows at the sharded per-rank shapes, three repetitions each (same box), default kernel form.
# Usage (via gpurun): bash tools/sweep_shard_rows.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/${1:-shard_rows}"
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for rep in 1 2 3; do
  for n in 2 4 8; do
    for br in 128 192 256; do
      ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 120 python tools/bench_rank_shapes.py --one $n > "$OUT/one.json" 2> "$OUT/one.err" || { tail -5 "$OUT/one.err"; exit 1; }
      python -c "import json; d=json.load(open('$OUT/one.json')); d.update(rep=$rep, bundle_rows_env=$br); print(json.dumps(d))" >> "$OUT/sweep.jsonl"
    done
  done
done
python - "$OUT/sweep.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(r["n_gpus"], r["bundle_rows_env"])].append(r["kernel_ms"])
for k in sorted(d): print("N=%d bundle %d: %s  median %.4f" % (k[0], k[1], " ".join("%.4f" % x for x in d[k]), sorted(d[k])[1]))
PY
