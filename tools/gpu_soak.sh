#!/bin/bash
# Soak: long device-driven run (1000 rounds), then 8 ranks on one GPU for 200 rounds.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/soak; mkdir -p $O
timeout -k 10 300 python bench.py --no-floor --steps 1000 --warmup 10 > $O/long1.log 2>&1 || exit 3
tail -1 $O/long1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('1 GPU 1000 rounds', round(d['ms_per_step'],4))"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --steps 200 --warmup 10 --no-floor > $O/long8.log 2>&1 || exit 4
tail -1 $O/long8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('8 ranks 200 rounds', round(d['ms_per_step'],4))"
