#!/bin/bash
# Issue anatomy of grad_dense_staged at the headline, fp64 and fp32: VALU / LDS / SALU instruction
# counts and active cycles per launch (one rocprofv3 pass per counter group, <= 8 SQ counters).
# Usage (via gpurun):  bash tools/pmc_staged_issue.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${1:-pmc_issue}; mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM"
for p in fp64 fp32; do
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O -o ${p}_$i -- python $R/bench.py --precision $p --no-floor --no-breakdown --steps 4 --warmup 1 > $O/${p}_$i.log 2>&1 || { tail -5 $O/${p}_$i.log; exit 3; }
  done
done
python - "$O" <<'PY'
import collections, csv, glob, json, sys
o = sys.argv[1]
res = {}
for f in sorted(glob.glob(o + "/**/*counter_collection.csv", recursive=True)):
    p = f.split("/")[-1].split("_")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "grad_dense_staged" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        res.setdefault(p, {})[k] = sum(v) / len(v)
json.dump(res, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
