#!/bin/bash
# Same-box A/B of two prebuilt extensions (build/ab/old.so vs build/ab/new.so) on the headline bench
# and FRC s = 1, alternating so that box drift hits both.  Usage (via gpurun): bash tools/ab_so.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
SO=erasurehead_amd/_C.cpython-310-x86_64-linux-gnu.so
O=gpurun_out/ab_so; mkdir -p $O
cp build/ab/new.so $SO
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "staged or bundle or dense" > $O/pytest_new.log 2>&1 || { tail -20 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
for rep in 1 2; do
  for v in old new; do
    cp build/ab/$v.so $SO
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-floor --json-out $O/agc_$v$rep.json > $O/agc_$v$rep.log 2>&1 || exit 2
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-floor --coded-ver 1 --stragglers 1 --json-out $O/frc_$v$rep.json > $O/frc_$v$rep.log 2>&1 || exit 3
    python -c "import json;a=json.load(open('$O/agc_$v$rep.json'));b=json.load(open('$O/frc_$v$rep.json'));print('$v$rep agc %.4f frc %.4f' % (a['ms_per_step'], b['ms_per_step']))"
  done
done
cp build/ab/new.so $SO
