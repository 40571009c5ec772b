#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/staged_prof; mkdir -p $O
for v in base c1 c4; do
  case $v in base) E="";; c1) E="ERASUREHEAD_STAGED=1 ERASUREHEAD_BUNDLE_ROWS=512 ERASUREHEAD_STAGE_ROWS=2";; c4) E="ERASUREHEAD_STAGED=0";; esac
  (cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python $OLDPWD/bench.py --steps 10 --warmup 3 --no-floor > $O/$v.log 2>&1) || exit 3
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1); echo "== $v"; head -4 $f | cut -d, -f1-8
done
