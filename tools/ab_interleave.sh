#!/bin/bash
# A/B: replica-interleaved task dispatch vs message-major, headline bench + cyclic + fp32.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/inter; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do for mode in on off; do for cv in 3 0; do
  if [ $mode = off ]; then export ERASUREHEAD_NO_INTERLEAVE=1; else unset ERASUREHEAD_NO_INTERLEAVE; fi
  timeout -k 10 200 python bench.py --coded-ver $cv --no-floor --steps 20 --warmup 5 > $O/$mode.$cv.$rep.log 2>&1 || exit 3
  tail -1 $O/$mode.$cv.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('interleave=$mode coded_ver=$cv', round(d['ms_per_step'],4))"
done; done; done
