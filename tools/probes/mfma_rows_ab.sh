#!/bin/bash
# bf16 MFMA bundles at the N = 1 rank shape: the LDS-DMA ring with 32- / 16-row stages, the VGPR-staged
# ring (--mfma-stream 3); whole kernel (probe 0) and the stage stream alone (probe 1), two alternating reps
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-r8a}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-"32 0 0" "32 0 1" "32 3 0" "32 3 1" "32 4 0" "32 4 1"}; do
    set -- $cfg
    timeout -k 10 200 python -u tools/bench_rank_shapes.py --one 1 --precision bf16 --mfma-rows $1 --mfma-stream $2 \
      --mfma-probe $3 >> $O/rows_ab.jsonl 2>> $O/rows_ab.err
  done
done
echo done
