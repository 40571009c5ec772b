#!/bin/bash
# Real-dataset partitioning (ref data_prepare.sh): raw table -> one-hot CSR partitions.
# RAW_ROWS>0 first writes a synthetic raw table with the dataset's schema (no network here).
set -euo pipefail
N_PROCS=${N_PROCS:-9}
N_STRAGGLERS=${N_STRAGGLERS:-1}
N_PARTITIONS=${N_PARTITIONS:-0}
PARTIAL_CODED=${PARTIAL_CODED:-0}
DATA_FOLDER=${DATA_FOLDER:-./straggdata/}
DATASET=${DATASET:-kc_house_data}
RAW_ROWS=${RAW_ROWS:-0}
cd "$(dirname "$0")/.."
EXTRA=""
[ "$RAW_ROWS" -gt 0 ] && EXTRA="--make-raw $RAW_ROWS"
python -m erasurehead_amd.data.prepare ${N_PROCS} ${DATA_FOLDER} ${DATASET} ${N_STRAGGLERS} ${N_PARTITIONS} ${PARTIAL_CODED} $EXTRA
