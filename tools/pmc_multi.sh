#!/bin/bash
# Counters of the one-wave replica bundles (grad_dense_multi) at the headline, fp64, against the
# LDS-staged kernel (ERASUREHEAD_STAGED=1): instruction mix, wave time, HBM bytes.  One rocprofv3
# pass per counter group (<= 8 SQ counters, FETCH_SIZE alone in its TCC pass).
# Usage (via gpurun):  bash tools/pmc_multi.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${1:-pmc_multi}; mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
G2="SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM"
G3="FETCH_SIZE"
for k in multi staged; do
  if [ $k = staged ]; then E="ERASUREHEAD_STAGED=1"; else E="ERASUREHEAD_AB=0"; fi
  i=0
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1))
    env $E timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O -o ${k}_$i -- python3 $R/bench.py --no-floor --no-breakdown --steps 4 --warmup 1 > $O/${k}_$i.log 2>&1 || { tail -5 $O/${k}_$i.log; exit 3; }
  done
done
python3 - "$O" <<'PY'
import collections, csv, glob, json, sys
o = sys.argv[1]
res = {}
for f in sorted(glob.glob(o + "/**/*counter_collection.csv", recursive=True)):
    k = f.split("/")[-1].split("_")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "grad_dense_multi" in r["Kernel_Name"] or "grad_dense_staged" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in agg.items():
        res.setdefault(k, {})[c] = sum(v) / len(v)
json.dump(res, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
PY
