#!/bin/bash
# A/B of the round loop on the headline (same box, 2 runs each): host-driven native pump (off),
# device-driven stream launches (stream) and hipGraph replay (graph).  docs/PERF_NOTES.md.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out/ab
for r in 1 2; do for m in off stream graph; do
timeout -k 10 200 python bench.py --no-floor --steps 30 --warmup 5 --device-loop $m > gpurun_out/ab/$m.$r.log 2>&1 || exit 3
tail -1 gpurun_out/ab/$m.$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['time_to_decode_ms_median'])"
done; done
