#!/bin/bash
# PMC A/B of the gradient kernel: replica-interleaved dispatch vs message-major (FETCH_SIZE, L2 hits).
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc; mkdir -p $O
cd /tmp
for mode in on off; do
  if [ $mode = off ]; then export ERASUREHEAD_NO_INTERLEAVE=1; else unset ERASUREHEAD_NO_INTERLEAVE; fi
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o fetch_$mode -- python $R/bench.py --no-floor --steps 4 --warmup 1 > $O/fetch_$mode.log 2>&1 || exit 3
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O -o hit_$mode -- python $R/bench.py --no-floor --steps 4 --warmup 1 > $O/hit_$mode.log 2>&1 || exit 3
done
ls $O
