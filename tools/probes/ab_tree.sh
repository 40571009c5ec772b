# Same-box A/B of two trees: the current one and an older one exported + built under build/ab_old
# (git archive <rev> | tar -x -C build/ab_old; python -c "import __graft_entry__ as g; g.build()" there),
# fp64 / fp32 headline, 100 steps, interleaved twice.  gpurun -- bash tools/probes/ab_tree.sh
set -o pipefail
O=$PWD/gpurun_out/ab_yload
mkdir -p $O
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then D=build/ab_old; else D=.; fi
    for p in fp64 fp32; do
      (cd $D && timeout -k 10 200 python -u bench.py --no-floor --no-breakdown --precision $p --steps 100 --warmup 10 > $O/${v}_${p}_$rep.json 2>$O/${v}_${p}_$rep.err) || exit 1
      tail -c 300 $O/${v}_${p}_$rep.json | head -c 0
    done
  done
done
echo done
