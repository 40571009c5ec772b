#!/bin/bash
# Does the headline step time depend on how long the GPU has been busy (clock ramp)?  The same
# bench with 5 / 50 / 300 warmup rounds, and the per-round kernel times of a 300-round run.
# Usage (via gpurun):  bash tools/gpu_warmup_study.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-warmup}"
mkdir -p "$OUT"
for W in 5 50 300; do
  timeout -k 10 300 python bench.py --steps 20 --warmup $W --no-floor --no-breakdown --json-out "$OUT/w$W.json" > "$OUT/w$W.log" 2>&1 || { tail -20 "$OUT/w$W.log"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/w$W.json')); print('warmup $W: ms/step', round(d['ms_per_step'],4))"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python "$ROOT/bench.py" --steps 300 --warmup 5 --no-floor --no-breakdown > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 2; }
python - "$OUT" <<'PY'
import csv, glob, sys, json
out = sys.argv[1]
f = glob.glob(out + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "grad_dense_staged" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
gaps = [(int(rows[i+1]["Start_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3 for i in range(len(rows)-1)]
json.dump({"kernel_us": us, "start_to_start_us": gaps}, open(out + "/per_call.json", "w"))
for a in range(0, len(us), 25):
    seg = us[a:a+25]
    print(f"calls {a:3d}-{a+len(seg)-1:3d}: mean {sum(seg)/len(seg):7.1f} us  min {min(seg):7.1f}  max {max(seg):7.1f}")
PY
