#!/bin/bash
# bf16 MFMA gradient: tests, headline in bf16 (MFMA vs VALU) and fp32, kernel stats and a PMC
# VALU-vs-MFMA instruction count A/B.   Usage (via gpurun): bash tools/gpu_mfma_check.sh OUTDIR
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-mfma}"
mkdir -p "$OUT"
echo "== tests"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "mfma or transpose or bf16" > "$OUT/pytest.log" 2>&1 || { grep -E "FAIL|Error" "$OUT/pytest.log" | head -20; tail -5 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
B="python bench.py --steps 20 --warmup 5 --no-floor --no-breakdown"
echo "== bf16 MFMA"
timeout -k 10 300 $B --precision bf16 --json-out "$OUT/bf16_mfma.json" > "$OUT/bf16_mfma.log" 2>&1 || { tail -20 "$OUT/bf16_mfma.log"; exit 2; }
echo "== bf16 VALU (ERASUREHEAD_MFMA=0)"
ERASUREHEAD_MFMA=0 timeout -k 10 300 $B --precision bf16 --json-out "$OUT/bf16_valu.json" > "$OUT/bf16_valu.log" 2>&1 || { tail -20 "$OUT/bf16_valu.log"; exit 3; }
echo "== fp32"
timeout -k 10 300 $B --precision fp32 --json-out "$OUT/fp32.json" > "$OUT/fp32.log" 2>&1 || { tail -20 "$OUT/fp32.log"; exit 4; }
for f in bf16_mfma bf16_valu fp32; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'], 4), 'ms', round(d.get('hbm_distinct_TBps', 0), 2), 'TB/s')"; done
echo "== kernel stats (bf16 MFMA)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bf16 -- python "$ROOT/bench.py" --precision bf16 --steps 10 --warmup 3 --no-floor --no-breakdown > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 5; }
cd "$ROOT"
head -4 "$OUT/prof/bf16_kernel_stats.csv" | cut -c1-160
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
grep -o "SQ_INSTS_[A-Z0-9_]*" "$OUT/counters.txt" | sort -u > "$OUT/sq_insts.txt"
C=""
for c in SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS; do grep -qx "$c" "$OUT/sq_insts.txt" && C="$C $c"; done
echo "== PMC:$C"
[ -n "$C" ] || exit 0
cd /tmp
for v in 1 0; do
  ERASUREHEAD_MFMA=$v timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_mfma$v" -o p -- python "$ROOT/bench.py" --precision bf16 --steps 3 --warmup 1 --no-floor --no-breakdown > "$OUT/pmc_mfma$v.log" 2>&1 || { tail -10 "$OUT/pmc_mfma$v.log"; exit 6; }
done
echo done
