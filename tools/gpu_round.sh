#!/bin/bash
# One GPU round on a fresh MI355X box, in stages (each under its own time limit; the first failure
# ends the script, nothing more touches the GPU after it):
#
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh OUT=gpurun_out/r5 tests smoke bench prec'
#
#   tests    python -m pytest tests -m gpu (thread timeouts, so a hang names its test)
#   smoke    __graft_entry__.smoke()
#   bench    bench.py at N=1 (20 steps as the driver runs it, then 100 settled steps)
#   prec     the headline in fp32 and bf16 (20 steps)
#   shapes   the heaviest rank's gradient at every N-GPU placement (tools/bench_rank_shapes.py)
#   sweep    dense gradient shape sweep vs the copy ceiling (tools/bench_kernels.py --only sweep)
#   rehearse 2/4/8 ranks time-sharing this GPU through bench.py --gpus N (host pump and arbiter)
#   prof     rocprofv3 --kernel-trace --stats of the fp64 / fp32 / bf16 headline
#   pmc      counter passes (one rocprofv3 --pmc run each) of the fp64 / fp32 headline
#   eval     evaluation phase profile (tools/profile_eval.py)
#   suite    tools/bench_suite.py (every BASELINE.json config)
#   conv     tools/convergence_study.py (all schemes, drain and lazy rows)
#   convlazy the same for the lazy rows + naive + drained uneven AGC, serially (one scheme at a time)
#   wide     the d = 2048 / 4096 rows of the sweep
#   sparse   sparse gradients at the real-data shapes (timings, then rocprofv3 kernel stats)
#   rccl     the RCCL self-loop GPU tests under rocprofv3 --kernel-trace (RCCL kernel names)
#   pmcsparse counter passes over the covtype-shaped sparse gradient
#   pmcbytes FETCH_SIZE / raw read requests / WRITE_SIZE over known-byte workloads (tools/pmc_calibrate.py)
#   abtree   same-box A/B against an older tree exported and built under build/ab_old
#            (git archive <rev> | tar -x -C build/ab_old, then __graft_entry__.build() there):
#            fp64 / fp32 headline, 100 steps, old / new interleaved twice
set -o pipefail
OUT=gpurun_out/round
STAGES=()
for a in "$@"; do
  case "$a" in
    OUT=*) OUT="${a#OUT=}" ;;
    *) STAGES+=("$a") ;;
  esac
done
mkdir -p "$OUT"
OUT=$(cd "$OUT" && pwd)
export TMPDIR=/tmp
log() { echo "[$(date +%T)] $*"; }
run() {  # run <seconds> <log> <cmd...>
  local t=$1 f=$2; shift 2
  log "start $f"
  timeout -k 10 "$t" "$@" > "$OUT/$f" 2>&1
  local rc=$?
  log "end $f rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "$OUT/$f"; exit $rc; fi
}
BENCH="python -u bench.py --no-floor"
for s in "${STAGES[@]}"; do
  case "$s" in
    tests)
      # TESTS="files..." narrows the run (default: every GPU test)
      # KEXPR="expr" selects tests by keyword expression (pytest -k)
      if [ -n "${KEXPR:-}" ]; then
        run 1500 pytest.log python -u -m pytest ${TESTS:-tests} -m gpu -k "$KEXPR" -x -v --timeout 120 --timeout-method thread
      else
        run 1500 pytest.log python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread
      fi
      tail -3 "$OUT/pytest.log" ;;
    smoke)
      run 300 smoke.log python -c 'import __graft_entry__ as g; g.build(); g.smoke(); print("smoke ok")' ;;
    bench)
      run 600 bench.log python -u bench.py && tail -1 "$OUT/bench.log" > "$OUT/bench.json"
      run 600 bench100.log $BENCH --steps 100 --warmup 10 && tail -1 "$OUT/bench100.log" > "$OUT/bench100.json"
      cat "$OUT/bench.json" ;;
    prec)
      for p in fp32 bf16; do
        run 600 "bench_$p.log" $BENCH --precision $p && tail -1 "$OUT/bench_$p.log" > "$OUT/bench_$p.json"
      done ;;
    shapes)
      run 900 shapes.log python -u tools/bench_rank_shapes.py --ab-slab --out "$OUT/shapes.jsonl"
      run 300 prof_shape8.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_shape8" -o run -- \
        python tools/bench_rank_shapes.py --one 8 ;;
    sweep)
      run 1100 sweep.log python -u tools/bench_kernels.py --only sweep --out "$OUT/sweep.jsonl" ;;
    wide)  # the off-headline widths only (d = 2048 / 4096, fp64 and fp32)
      run 600 wide.log python -u tools/bench_kernels.py --only sweep --ds 2048,4096 --out "$OUT/wide.jsonl" ;;
    choices)  # every valid kernel choice at the d = 2048 replica shapes (CHOICE_SHAPES overrides)
      run 900 choices.log python -u tools/bench_kernels.py --only choices \
        --shapes "${CHOICE_SHAPES:-fp64:2048:1e6,fp32:2048:1e6,fp64:2048:1e5,fp32:2048:1e5}" --out "$OUT/choices.jsonl" ;;
    sparse)  # sparse gradients at the real-data shapes, then their kernel stats
      run 600 sparse.log python -u tools/bench_kernels.py --only sparse --out "$OUT/sparse.jsonl"
      run 600 prof_sparse.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_sparse" -o run -- \
        python tools/bench_kernels.py --only sparse --out /tmp/sparse_prof.jsonl ;;
    bf16ab)  # the bf16 MFMA bundles: LDS-DMA ring vs VGPR-staged ring, kernel alone (rank shape N = 1) and headline
      for m in ${MFMA_MODES:-0 3 0 3}; do
        run 300 "bf16_shape_$m.log" python -u tools/bench_rank_shapes.py --one 1 --precision bf16 --mfma-stream $m
        cat "$OUT/bf16_shape_$m.log" >> "$OUT/bf16_shapes.jsonl"
      done
      for m in ${MFMA_BENCH:-0 3}; do
        run 600 "bench_bf16_s$m.log" $BENCH --precision bf16 --mfma-stream $m --steps 100 --warmup 10 \
          && tail -1 "$OUT/bench_bf16_s$m.log" > "$OUT/bench_bf16_s$m.json"
      done
      run 300 prof_bf16_vring.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bf16_vring" -o run -- \
        python bench.py --no-floor --no-breakdown --precision bf16 --mfma-stream 3 --steps 50 ;;
    sparseab)  # sparse gradients at the real shapes (naive / cyclic-style / FRC layouts), then the sparse suite rows
      run 600 sparse.log python -u tools/bench_kernels.py --only sparse --out "$OUT/sparse.jsonl"
      run 900 suite_sparse.log python -u tools/bench_suite.py --out "$OUT/suite" \
        --only naive_covtype,agc_covtype,ls_kc_house_naive,ls_kc_house_agc_k6,naive_amazon,agc_amazon ;;
    rccl)  # the RCCL self-loop comm path under the kernel tracer (RCCL kernel names in the stats)
      run 600 prof_rccl.log rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_rccl" -o run -- \
        python -u -m pytest tests/test_rccl_gpu.py -k self_loop -x -q --timeout 120 --timeout-method thread ;;
    pmcbytes)  # FETCH_SIZE against the raw memory-side read requests and known byte counts
      run 120 counters.log rocprofv3 -L
      i=0
      for grp in "FETCH_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B" "WRITE_SIZE"; do
        i=$((i+1))
        want=""
        for c in $grp; do  # only counters this box lists (an unknown name would end the stage)
          if grep -qw "$c" "$OUT/counters.log"; then want="$want $c"; fi
        done
        [ -z "$want" ] && { log "skip pass $i: none of $grp listed"; continue; }
        [ "$grp" = "FETCH_SIZE" ] || [ "$grp" = "WRITE_SIZE" ] || want=$(echo $want | sed 's/\([A-Z0-9_]*\)/\1_sum/g')
        run 180 "pmcb_$i.log" timeout -s KILL 170 rocprofv3 --pmc $want --output-format csv -d "$OUT/pmcb" -o "p$i" -- \
          python tools/pmc_calibrate.py --known "$OUT/known.json"
      done
      python tools/pmc_summary.py "$OUT/pmcb" --by-kernel > "$OUT/pmcb_summary.json" ;;
    pmcsparse)  # counter passes over the covtype-shaped sparse gradient (ELL rows)
      run 120 counters.log rocprofv3 -L
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
                 "SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
                 "FETCH_SIZE"; do
        i=$((i+1))
        want=""
        for c in $grp; do
          if grep -qw "$c" "$OUT/counters.log"; then want="$want $c"; fi
        done
        [ -z "$want" ] && { log "skip pass $i: none of $grp listed"; continue; }
        run 180 "pmcs_$i.log" timeout -s KILL 170 rocprofv3 --pmc $want --output-format csv -d "$OUT/pmcs" -o "p$i" -- \
          python tools/bench_kernels.py --only sparse --sparse-shapes covtype --ell-only --sparse-layouts naive --out /tmp/sparse_pmc.jsonl
      done
      python tools/pmc_summary.py "$OUT/pmcs" --by-kernel > "$OUT/pmcs_summary.json" ;;
    rehearse)
      for n in 2 4 8; do
        run 600 "rehearse_$n.log" python -u bench.py --gpus $n --steps 20 --warmup 5 --no-floor \
          --json-out "$OUT/rehearse_$n.json"
      done ;;
    prof)
      for p in fp64 fp32 bf16; do
        run 600 "prof_$p.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$p" -o run -- \
          python bench.py --no-floor --no-breakdown --precision $p --steps 50
      done ;;
    pmc)
      G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
      G2="SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM"
      for p in fp64 fp32; do
        i=0
        for grp in "$G1" "$G2" "FETCH_SIZE"; do
          i=$((i+1))
          run 120 "pmc_${p}_$i.log" rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc" -o "${p}_$i" -- \
            python bench.py --no-floor --no-breakdown --precision $p --steps 4 --warmup 1
        done
      done
      python tools/pmc_summary.py "$OUT/pmc" > "$OUT/pmc_summary.json" ;;
    abtree)
      for rep in 1 2; do
        for v in old new; do
          D=.; [ $v = old ] && D=build/ab_old
          for p in fp64 fp32; do
            (cd $D && run 300 "ab_${v}_${p}_$rep.log" python -u bench.py --no-floor --no-breakdown --precision $p \
              --steps 100 --warmup 10) || exit 1
          done
        done
      done ;;
    release)  # what the strict release forms cost per round: 2 and 8 ranks on this GPU, arbiter on, auto vs strict
      run 900 release.log env TAG=_rel NO_BF16=1 MODES=on RELEASE="auto strict" bash tools/probes/overhead_tiny.sh
      cp -r gpurun_out/overhead_rel "$OUT/" ;;
    overhead)  # per-round chain on a tiny problem (tools/probes/overhead_tiny.sh), 2 and 8 ranks, arbiter on,
               # slab reduction forms 1 (fused put) and 2 (two-stage put)
      run 900 overhead.log env TAG=_r4 NO_BF16=1 MODES=on SLAB="1 2" bash tools/probes/overhead_tiny.sh
      cp -r gpurun_out/overhead_r4 "$OUT/" ;;
    suite)  # every BASELINE.json config (tools/bench_suite.py)
      run 1000 suite.log python -u tools/bench_suite.py --out "$OUT/suite" ;;
    conv)  # convergence vs wall-clock, every scheme incl. the lazy-drain rows (11 processes on the GPU)
      run 900 conv.log python -u tools/convergence_study.py --out "$OUT/convergence" ;;
    convlazy)  # the lazy rows, naive and the drained uneven AGC, ONE scheme at a time (no GPU sharing)
      run 1100 convlazy.log python -u tools/convergence_study.py --serial \
        --only naive,agc_s2_k6_uneven,cyclic_s2_lazy,frc_s1_lazy,agc_s1_k6_lazy,agc_s2_k6_uneven_lazy \
        --out "$OUT/convergence_lazy" ;;
    eval)
      run 600 eval.log python -u tools/profile_eval.py --out "$OUT/eval.json" ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
log "all stages done"
