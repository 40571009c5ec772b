#!/bin/bash
# GPU round: device-driven loop (hipGraph) tests, headline bench graph vs host-driven, small-config suite.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/g3
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log"
  case $rc in 0|1) ;; *) exit $rc ;; esac
}
step pytest 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k "matches_cpu or device_loop"
step bench_graph 300 python bench.py --no-floor --steps 20 --warmup 5 --device-loop graph
step bench_stream 300 python bench.py --no-floor --steps 20 --warmup 5 --device-loop stream
step suite_graph 400 python tools/bench_suite.py --only agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k4,ls_kc_house_agc_k6 --out $O/suite_graph --device-loop graph
step suite_stream 400 python tools/bench_suite.py --only agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k4,ls_kc_house_agc_k6 --out $O/suite_stream --device-loop stream
