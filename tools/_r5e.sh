set -o pipefail
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "wide or dense_grad" > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 600 python -u tools/bench_kernels.py --only choices --shapes fp64:4096:1e6,fp32:4096:1e6,fp64:4096:1e5,fp64:3000:1e6,fp64:256:1e6,fp64:512:1e6,fp32:512:1e6 --out $O/choices.jsonl > $O/choices.log 2>&1 &&
timeout -k 10 300 python -u tools/probes/clock_trace.py --no-floor --no-breakdown --steps 100 --clock-warmup-ms 0 > $O/clock_nowarm.json 2> $O/clock_nowarm.err &&
timeout -k 10 300 python -u tools/probes/clock_trace.py --no-floor --no-breakdown --steps 20 > $O/clock_warm.json 2> $O/clock_warm.err &&
for p in fp64 fp32 bf16; do timeout -k 10 300 python -u bench.py --no-floor --precision $p > $O/bench_$p.log 2>&1 || exit 1; tail -1 $O/bench_$p.log > $O/bench_$p.json; done
