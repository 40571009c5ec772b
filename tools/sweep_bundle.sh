#!/bin/bash
# Replica-bundle kernel (one wave per replica in one workgroup) vs the interleaved dispatch.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/bundle; mkdir -p $O
ERASUREHEAD_BUNDLE_ROWS=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "test_dense_grad and not interleaved" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do for br in ${BR_LIST:-0 64 128 256 512}; do
  ERASUREHEAD_BUNDLE_ROWS=$br timeout -k 10 200 python bench.py ${EXTRA:-} --no-floor --steps 20 --warmup 5 > $O/$br.$rep.log 2>&1 || exit 3
  tail -1 $O/$br.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bundle_rows=$br', round(d['ms_per_step'],4))"
done; done
