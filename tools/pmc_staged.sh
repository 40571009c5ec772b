#!/bin/bash
# PMC A/B of the gradient kernel: LDS-staged replica bundles (default) vs the replica-interleaved
# dispatch (ERASUREHEAD_STAGED=0): FETCH_SIZE and L2 hits/misses per gradient launch.
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_staged; mkdir -p $O
cd /tmp
for mode in staged interleaved; do
  if [ $mode = interleaved ]; then export ERASUREHEAD_STAGED=0; else unset ERASUREHEAD_STAGED; fi
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o fetch_$mode -- python $R/bench.py --no-floor --steps 4 --warmup 1 > $O/fetch_$mode.log 2>&1 || exit 3
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O -o hit_$mode -- python $R/bench.py --no-floor --steps 4 --warmup 1 > $O/hit_$mode.log 2>&1 || exit 3
done
python $R/tools/pmc_summary.py $O > $O/summary.json && cat $O/summary.json
