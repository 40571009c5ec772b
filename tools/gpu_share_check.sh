#!/bin/bash
# GPU round: shared-partition tests + bench, then the bench at 4 and 8 ranks sharing the one GPU
# (rehearsal of the driver's multi-GPU launch over the IPC mailbox).  Stops at the first step
# that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/g2
mkdir -p $O
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log"
  case $rc in 0|1) ;; *) exit $rc ;; esac
}
step pytest 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "share or encode"
step bench_share 300 python bench.py --share-partitions --no-floor --steps 20 --warmup 5
step bench4 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --steps 10 --warmup 3 --no-floor
step bench8 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 8 --steps 10 --warmup 3
