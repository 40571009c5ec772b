#!/bin/bash
# Rows-in-flight sweep of grad_dense_fused (ERASUREHEAD_GRAD_ROWS) at full headline scale, every precision.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/rows
mkdir -p $O
for p in ${PREC_LIST:-fp64 fp32 bf16}; do for r in ${ROWS_LIST:-1 2 4 5 6 7}; do
  ERASUREHEAD_GRAD_ROWS=$r timeout -k 10 200 python bench.py --precision $p --no-floor --steps 20 --warmup 5 > $O/$p.$r.log 2>&1 || exit 3
  tail -1 $O/$p.$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p rows=$r', round(d['ms_per_step'],4), round(d['time_to_decode_ms_median'],4))"
done; done
