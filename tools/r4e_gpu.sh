set -o pipefail
mkdir -p gpurun_out/r4e
timeout -k 10 600 python -u -m pytest tests/test_integrity_gpu.py tests/test_multiproc_gpu.py -v -k "integrity or arbiter or tagged or torn or preflight or untagged or sabotage or loopback" --timeout 300 --timeout-method thread > gpurun_out/r4e/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r4e/tests.log | head -30; tail -40 gpurun_out/r4e/tests.log; exit 1; }
tail -3 gpurun_out/r4e/tests.log
B="--gpus 3 --steps 60 --warmup 5 --no-floor --preflight 0"
timeout -k 10 900 python tools/ab.py --out gpurun_out/r4e/tag_ab.jsonl --timeout 200 --reps 3 --interleave --summary \
  --run "tagged | | $B" --run "untagged | | $B --no-integrity" \
  --run "arb tagged | ERASUREHEAD_DEVICE_MASTER=on | $B" --run "arb untagged | ERASUREHEAD_DEVICE_MASTER=on | $B --no-integrity"
