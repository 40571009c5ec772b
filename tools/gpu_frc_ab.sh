#!/bin/bash
# FRC s=1 (bundles of 2 replicas): default kernel vs one-wave bundles with either epilogue, 95 timed rounds.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/frc_ab
for rep in 1 2; do
  for k in "default:ERASUREHEAD_AB=0" "multi-wave:ERASUREHEAD_STAGED=multi ERASUREHEAD_MULTI_EPI=wave" "multi-lane:ERASUREHEAD_STAGED=multi ERASUREHEAD_MULTI_EPI=lane"; do
    name=${k%%:*}; E=${k#*:}
    env $E timeout -k 10 300 python bench.py --coded-ver 1 --stragglers 1 --steps 95 --warmup 5 --no-floor --no-breakdown --json-out gpurun_out/frc_ab/b.json > gpurun_out/frc_ab/b.log 2>&1 || { tail -20 gpurun_out/frc_ab/b.log; exit 2; }
    python -c "import json; d=json.load(open('gpurun_out/frc_ab/b.json')); print('rep $rep FRC s=1 $name', round(d['ms_per_step'],4), d['ranks'][0].get('grad_kernel'))" | tee -a gpurun_out/frc_ab/summary.txt
  done
done
