#!/bin/bash
# Sparse (one-hot ELL) GPU tests, then the covtype- and kc_house-shaped suite rows.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "sparse or ell or onehot" > gpurun_out/sp.log 2>&1; rc=$?; tail -1 gpurun_out/sp.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/bench_suite.py --only agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k4,ls_kc_house_agc_k6 --out gpurun_out/sp_suite > gpurun_out/sp_suite.log 2>&1 && tail -5 gpurun_out/sp_suite/suite.md
