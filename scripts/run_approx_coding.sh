#!/bin/bash
# Canonical approximate-gradient-coding run (ref run_approx_coding.sh) on one MI355X node.
# Logical workers (N_PROCS-1) are spread over NGPUS processes, one per GPU (RCCL over xGMI).
# MODES (is_coded partitions coded_ver):  1 0 1 = FRC exact ("EGC"),  1 0 3 = AGC,  0 x x = vanilla GD.
set -euo pipefail
N_PROCS=${N_PROCS:-9}
N_STRAGGLERS=${N_STRAGGLERS:-1}
N_COLLECT=${N_COLLECT:-6}
UPDATE_RULE=${UPDATE_RULE:-AGD}
N_PARTITIONS=${N_PARTITIONS:-0}
ADD_DELAY=${ADD_DELAY:-0}
DATA_FOLDER=${DATA_FOLDER:-./straggdata/}
IS_REAL=${IS_REAL:-1}
DATASET=${DATASET:-kc_house_data}
N_ROWS=${N_ROWS:-17290}
N_COLS=${N_COLS:-27654}
MODE=${MODE:-"1 0 3"}
NGPUS=${NGPUS:-1}
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$(dirname "$0")/.."
ARGS="${N_PROCS} ${N_ROWS} ${N_COLS} ${DATA_FOLDER} ${IS_REAL} ${DATASET} ${MODE%% *} ${N_STRAGGLERS} ${N_PARTITIONS} ${MODE##* } ${N_COLLECT} ${ADD_DELAY} ${UPDATE_RULE}"
if [ "$NGPUS" -gt 1 ]; then
  exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPUS" --master-addr 127.0.0.1 \
       --master-port "${PORT:-29500}" main.py $ARGS "$@"
fi
exec python main.py $ARGS "$@"
