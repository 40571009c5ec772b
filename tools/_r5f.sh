set -o pipefail
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 120 python -u tools/probes/mall_reuse.py > $O/mall.json 2> $O/mall.err &&
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "wide or dense_grad" > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python -u tools/bench_kernels.py --only choices --shapes fp64:4096:1e6,fp32:4096:1e6,fp64:3000:1e6 --out $O/choices.jsonl > $O/choices.log 2>&1 &&
timeout -k 10 900 python -u tools/bench_kernels.py --only sweep --out $O/sweep.jsonl > $O/sweep.log 2>&1
