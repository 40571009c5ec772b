#!/bin/bash
# Confirmation runs of the rows-in-flight choice (tools/sweep_grad_rows.sh) on a second box.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for rep in 1 2; do
ROWS_LIST="1 2" PREC_LIST="fp64 bf16" bash tools/sweep_grad_rows.sh || exit 3
ROWS_LIST="4 2" PREC_LIST="fp32" bash tools/sweep_grad_rows.sh || exit 3
done
