#!/bin/bash
# Env-only sweep of the staged-bundle geometry (rows per stage, ring depth) on the headline bench.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/sweep_env; mkdir -p $O
for cfg in "2 2" "1 2" "3 2" "4 2" "1 3" "2 3" "2 2"; do
  set -- $cfg
  ERASUREHEAD_STAGE_ROWS=$1 ERASUREHEAD_STAGES=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-floor --json-out $O/r$1_s$2.json > $O/r$1_s$2.log 2>&1 || exit 2
  python -c "import json;a=json.load(open('$O/r$1_s$2.json'));print('rows $1 stages $2 ms %.4f' % a['ms_per_step'])" | tee -a $O/sweep.txt
done
