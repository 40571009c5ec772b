#!/bin/bash
# units tile pass: both message rows vs the first row only (timing probe), per kernel under the tracer
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-r7d}; mkdir -p $O
for s in amazon-dataset kc_house_data; do
  for p in "" "--units-probe"; do
    t=${p:+_probe}
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${s}$t -o run -- \
      python -u tools/bench_kernels.py --only sparse --sparse-shapes $s --sparse-layouts frc_s1 --sparse-rows auto $p \
      --out $O/${s}$t.jsonl > $O/${s}$t.log 2>&1
  done
done
echo done
