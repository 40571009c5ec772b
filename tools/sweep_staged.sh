#!/bin/bash
# LDS-staged replica bundles (grad_dense_staged): tests, then bench A/B against the interleaved
# dispatch, over rows per bundle task (BR_LIST), rows per LDS stage (SR_LIST) and ring depth (ST_LIST).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/staged; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "bundle" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 2
row() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['ms_per_step'],4))"; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py ${EXTRA:-} --no-floor --steps 20 --warmup 5 > $O/base.$rep.log 2>&1 || exit 3
  row $O/base.$rep.log "interleaved"
  for br in ${BR_LIST:-256 512}; do for sr in ${SR_LIST:-0}; do for ns in ${ST_LIST:-0}; do
    ERASUREHEAD_STAGED=1 ERASUREHEAD_BUNDLE_ROWS=$br ERASUREHEAD_STAGE_ROWS=$sr ERASUREHEAD_STAGES=$ns timeout -k 10 200 python bench.py ${EXTRA:-} --no-floor --steps 20 --warmup 5 > $O/s$br.$sr.$ns.$rep.log 2>&1 || exit 3
    row $O/s$br.$sr.$ns.$rep.log "staged bundle_rows=$br stage_rows=$sr stages=$ns"
  done; done; done
done
