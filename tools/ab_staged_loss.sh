#!/bin/bash
# Interleaved vs LDS-staged replica kernels (one row / pair mode), logistic vs least squares
# (no exp in the residual), one process per configuration.
# CFGS: "<stage rows>:<1|pair>[:<waves per replica>]".
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/staged_loss; mkdir -p $O; rm -f $O/res.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bundle" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 2
for loss in ${LOSSES:-logistic ls}; do
  ERASUREHEAD_STAGED=0 timeout -k 10 120 python tools/bench_staged.py --layout ${LAYOUT:-agc} --loss $loss --precision ${PREC:-fp64} --tag interleaved >> $O/res.jsonl 2> $O/err.log || exit 3
  for cfg in ${CFGS:-"2:1" "2:pair"}; do
    IFS=: read sr md wpr <<< "$cfg"
    ERASUREHEAD_STAGED=$md ERASUREHEAD_BUNDLE_ROWS=${BR:-512} ERASUREHEAD_STAGE_ROWS=$sr ERASUREHEAD_STAGED_WPR=${wpr:-1} \
      timeout -k 10 120 python tools/bench_staged.py --layout ${LAYOUT:-agc} --loss $loss --precision ${PREC:-fp64} --tag "staged $cfg" >> $O/res.jsonl 2>> $O/err.log || exit 3
  done
done
cat $O/res.jsonl
