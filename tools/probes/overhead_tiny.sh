# Per-round overhead chain on one GPU: a tiny AGC problem (16k x 1000 rows, kernels of a few us)
# so the round time is mostly messaging + arbiter / host pump; 2 and 8 ranks, arbiter off / on.
#   gpurun -- bash tools/probes/overhead_tiny.sh   (writes gpurun_out/overhead${TAG}/)
#   RANKS="2 8" MODES="on off" SLAB="1 2" (slab reduction forms to A/B: bench.py --slab-mode)
#   RELEASE="auto strict relaxed" (ERASUREHEAD_RELEASE: ranks sharing one GPU select relaxed by default)
set -o pipefail
O=gpurun_out/overhead${TAG:-}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "${NO_BF16:-}" ]; then
  timeout -k 10 300 python -u bench.py --precision bf16 --no-floor --json-out $O/bf16.json > $O/bf16.log 2>&1 || exit 1
fi
for n in ${RANKS:-2 8}; do
  for m in ${MODES:-off on}; do
    for sm in ${SLAB:-1}; do
      for rel in ${RELEASE:-auto}; do
        t=tiny_${n}_${m}_s$sm; [ "$rel" = auto ] || t=${t}_$rel
        ERASUREHEAD_RELEASE=$rel ERASUREHEAD_DEVICE_MASTER=$m timeout -k 10 300 python -u bench.py --gpus $n --steps 200 \
          --warmup 20 --no-floor --no-straggler --slab-mode $sm --n-rows ${NROWS:-16000} --n-cols 1000 \
          --json-out $O/$t.json > $O/$t.log 2>&1 || exit 1
        echo "tiny $n $m slab $sm release $rel done"
      done
    done
  done
done
echo done
