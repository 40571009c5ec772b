set -e
# same-box A/B of the ELL row pass's fields per batch, covtype only (profiles/round6/sparse/rowbuf_kb/): the
# old tree (build/ab_old) and variant trees build/ab_v16, build/ab_v20 against the tree under test (28).  The
# variant (ell_rows_lds loading through buffer descriptors, the field offset in an SGPR) was measured and
# reverted; the variant trees were copies of that tree with the fields per batch edited.
O=$GRAFT_REPO_ROOT/gpurun_out/${OUT:-rowkb}; mkdir -p $O
B="tools/bench_kernels.py --only sparse --sparse-shapes covtype --ell-only --sparse-layouts naive"
for rep in 1 2 3; do
  for v in ab_old ab_v16 ab_v20; do
    (cd build/$v && timeout -k 10 200 python -u $B --out $O/${v}_$rep.jsonl > $O/${v}_$rep.log 2>&1)
  done
  timeout -k 10 200 python -u $B --out $O/new_$rep.jsonl > $O/new_$rep.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
for v in ab_old ab_v16 ab_v20; do
  (cd $GRAFT_REPO_ROOT/build/$v && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 -u $B --out $O/prof_${v}.jsonl > $O/prof_$v.log 2>&1)
done
(cd $GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run -- python3 -u $B --out $O/prof_new.jsonl > $O/prof_new.log 2>&1)
echo done
