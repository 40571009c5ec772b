#!/bin/bash
# GPU round: sparse kernel tests, ELL microbenchmarks and the covtype / kc_house suite rows.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/g4
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log"
  case $rc in 0|1) ;; *) exit $rc ;; esac
}
step pytest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "sparse or ell or onehot"
step kernels 300 python tools/bench_kernels.py --only sparse --out $O/kernels_sparse.jsonl
step suite 400 python tools/bench_suite.py --only agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k6 --out $O/suite
