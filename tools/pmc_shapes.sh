#!/bin/bash
# Occupancy / issue counters of the staged gradient kernel at the N=1 headline and the N=2 rank shape
# with 512- and 128-row bundles (why do 512-row bundles stream slower on the N=2 rank?).
# Usage (via gpurun): bash tools/pmc_shapes.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/${1:-pmc_shapes}; mkdir -p $O
cd /tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
for cfg in "1 512" "2 512" "2 128"; do
  set -- $cfg
  tag=n$1_b$2
  ERASUREHEAD_BUNDLE_ROWS=$2 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o tr_$tag -- python $R/tools/bench_rank_shapes.py --one $1 > $O/tr_$tag.log 2>&1 || { tail -5 $O/tr_$tag.log; exit 3; }
  ERASUREHEAD_BUNDLE_ROWS=$2 timeout -s KILL 120 rocprofv3 --pmc $G1 --output-format csv -d $O -o pmc_$tag -- python $R/tools/bench_rank_shapes.py --one $1 > $O/pmc_$tag.log 2>&1 || { tail -5 $O/pmc_$tag.log; exit 4; }
done
python - "$O" <<'PY'
import collections, csv, glob, json, sys
o = sys.argv[1]
out = {}
for f in sorted(glob.glob(o + "/**/tr_*kernel_stats.csv", recursive=True)):
    tag = f.split("tr_")[1].split("_kernel_stats")[0]
    for r in csv.DictReader(open(f)):
        if "grad_dense_staged" in r["Name"]:
            out.setdefault(tag, {})["staged_avg_us"] = float(r["AverageNs"]) / 1e3
for f in sorted(glob.glob(o + "/**/pmc_*counter_collection.csv", recursive=True)):
    tag = f.split("pmc_")[1].split("_counter_collection")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "grad_dense_staged" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out.setdefault(tag, {})[k] = sum(v) / len(v)
json.dump(out, open(o + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
