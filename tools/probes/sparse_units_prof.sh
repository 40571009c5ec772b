#!/bin/bash
# per-kernel times of the sparse gradient, naive vs FRC / AGC units, one shape per traced run
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-r7c}; mkdir -p $O
for s in amazon-dataset kc_house_data covtype; do
  for l in naive frc_s1; do
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${s}_$l -o run -- \
      python -u tools/bench_kernels.py --only sparse --sparse-shapes $s --sparse-layouts $l --sparse-rows auto \
      --out $O/${s}_$l.jsonl > $O/${s}_$l.log 2>&1
  done
done
echo done
