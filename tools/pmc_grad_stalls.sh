#!/bin/bash
# Stall anatomy of grad_dense_fused on the headline (replica-interleaved) and on distinct rows (naive):
# one rocprofv3 pass per counter group (gfx950 per-block limits: 8 SQ, 4 TCP, 2 TA).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/stall; mkdir -p $O
cd /tmp
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD"
TA="TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
TCP="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
for mode in agc naive; do
  EXTRA=""; [ $mode = naive ] && EXTRA=--naive
  i=0
  for grp in "$SQ" "$TA" "$TCP"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O -o ${mode}_$i -- python $R/bench.py $EXTRA --no-floor --steps 4 --warmup 1 > $O/${mode}_$i.log 2>&1 || exit 3
  done
done
python - "$O" <<'EOF'
import collections, csv, glob, json, sys
o = sys.argv[1]
res = {}
for f in sorted(glob.glob(o + "/*_counter_collection.csv")):
    mode = f.split("/")[-1].split("_")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "grad_dense_fused" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        res.setdefault(mode, {})[k] = sum(v) / len(v)
json.dump(res, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(res, indent=1))
EOF
