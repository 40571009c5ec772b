set -o pipefail
mkdir -p gpurun_out/r4c
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests/test_multiproc_gpu.py -k "loopback or physically" -v --timeout 300 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r4c/tests.log | head -30; tail -40 gpurun_out/r4c/tests.log; exit 1; }
tail -3 gpurun_out/r4c/tests.log
for tag in tagged untagged; do
  extra=""; [ $tag = untagged ] && extra="--no-integrity"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c/prof_$tag -o run -- python bench.py --gpus 3 --steps 60 --warmup 5 --no-floor --no-breakdown --preflight 0 $extra > gpurun_out/r4c/b3_$tag.json 2> gpurun_out/r4c/b3_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/r4c/b3_$tag.err; exit 1; }
done
ls -R gpurun_out/r4c | head -40
