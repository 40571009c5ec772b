#!/bin/bash
# A/B of the replica dispatch stride: 8 = bundle members on one XCD (L2 sharing),
# 1 / 2 / 4 = members on different XCDs (sharing through the Infinity Cache), 16 = two rounds of XCDs.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/stride; mkdir -p $O
for rep in 1 2; do for st in ${STRIDES:-8 1 2 4 16}; do
  ERASUREHEAD_REPLICA_STRIDE=$st timeout -k 10 200 python bench.py --no-floor --steps 20 --warmup 5 > $O/$st.$rep.log 2>&1 || exit 3
  tail -1 $O/$st.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stride=$st', round(d['ms_per_step'],4))"
done; done
