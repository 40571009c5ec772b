set -e
# same-box A/B of the sparse gradient: the round-5 tree built in build/ab_old against this tree, alternating
# (build/ab_old: mkdir -p build/ab_old && git archive <round-5 commit> | tar -x -C build/ab_old && (cd build/ab_old && python tools/build_ext.py))
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-r7a}; mkdir -p $O
for rep in 1 2; do
  (cd build/ab_old && timeout -k 10 300 python -u tools/bench_kernels.py --only sparse --out $O/old_$rep.jsonl > $O/old_$rep.log 2>&1)
  timeout -k 10 300 python -u tools/bench_kernels.py --only sparse --out $O/new_$rep.jsonl > $O/new_$rep.log 2>&1
done
echo done
