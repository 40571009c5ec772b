set -o pipefail
mkdir -p gpurun_out/r4d
B="--gpus 3 --steps 60 --warmup 5 --no-floor --preflight 0"
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r4d/tag_ab.jsonl --timeout 200 --reps 3 --interleave --summary \
  --run "tagged | | $B" --run "untagged | | $B --no-integrity" \
  --run "arb tagged | ERASUREHEAD_DEVICE_MASTER=on | $B" --run "arb untagged | ERASUREHEAD_DEVICE_MASTER=on | $B --no-integrity"
