#!/bin/bash
# GPU round: eval GEMM tests + v1/v2 microbenchmark.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/g5
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log"
  case $rc in 0|1) ;; *) exit $rc ;; esac
}
step pytest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "eval"
step v2 300 python tools/bench_kernels.py --only eval --out $O/eval_v2.jsonl
export ERASUREHEAD_EVAL_V1=1
step v1 300 python tools/bench_kernels.py --only eval --out $O/eval_v1.jsonl
