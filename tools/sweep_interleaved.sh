#!/bin/bash
# Interleaved dispatch: rows-in-flight variant x task count, fp64 headline.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/isweep; mkdir -p $O
for t in ${TASKS_LIST:-2048 4096 8192}; do for r in ${ROWS_LIST:-1 2 4 5 6 7}; do
  ERASUREHEAD_GRAD_ROWS=$r timeout -k 10 200 python bench.py --precision ${PREC:-fp64} ${EXTRA:-} --tasks $t --no-floor --steps 20 --warmup 5 > $O/$t.$r.log 2>&1 || exit 3
  tail -1 $O/$t.$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tasks=$t rows=$r', round(d['ms_per_step'],4))"
done; done
