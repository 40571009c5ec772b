#!/bin/bash
# Kernel + engine GPU tests, then the headline bench in fp64 / fp32 / bf16 (ms per round and
# message-row GB/s).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/g6
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/g6/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/g6/pytest.log; [ $rc -le 1 ] || exit $rc
for p in fp64 fp32 bf16; do
  timeout -k 10 200 python bench.py --precision $p --no-floor --steps 20 --warmup 5 > gpurun_out/g6/$p.log 2>&1 || exit 3
  tail -1 gpurun_out/g6/$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', round(d['ms_per_step'],4), round(d['rank0_message_rows_GBps']))"
done
