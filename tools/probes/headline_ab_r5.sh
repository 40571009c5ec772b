set -e
# same-box A/B of the fp64 headline: the round-5 final tree (build/ab_r5: git archive b9b02c4, built in place)
# against this tree, 100 timed steps, three alternating reps, old first
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-abr5}; mkdir -p $O
for rep in 1 2 3; do
  (cd build/ab_r5 && timeout -k 10 200 python -u bench.py --no-floor --no-breakdown --precision fp64 --steps 100 --warmup 10 > $O/old_$rep.json 2> $O/old_$rep.err)
  timeout -k 10 200 python -u bench.py --no-floor --no-breakdown --precision fp64 --steps 100 --warmup 10 > $O/new_$rep.json 2> $O/new_$rep.err
done
echo done
