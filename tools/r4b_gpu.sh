set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_integrity_gpu.py tests/test_multiproc_gpu.py -v -k "integrity or physically or dead_worker or arbiter or tagged or torn or preflight or untagged" --timeout 300 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -3 gpurun_out/r4b/tests.log
B="--gpus 8 --steps 20 --warmup 5 --no-floor --no-breakdown"
D="--add-delay 1 --delay-on worker --delay-mode fixed --fixed-stragglers 4 --fixed-sleep 0.005"
timeout -k 10 1000 python tools/ab.py --out gpurun_out/r4b/ab8.jsonl --timeout 240 --summary \
  --run "p8 | | $B" \
  --run "p8 untagged | | $B --no-integrity" \
  --run "p8 arbiter | ERASUREHEAD_DEVICE_MASTER=on | $B" \
  --run "p8 arbiter untagged | ERASUREHEAD_DEVICE_MASTER=on | $B --no-integrity" \
  --run "m8 | | $B --shard message" \
  --run "m8 late w3 | | $B --shard message $D" \
  --run "p8 late w3 | | $B $D"
