"""Per-rank round breakdown of a real-data stand-in over N ranks (IPC mailbox transport).

    python tools/rank_breakdown.py --gpus 2 --data amazon [--rounds 30] [--json-out FILE]

Runs AGC W=8, s=1, k=6 on the one-hot stand-in of a reference dataset (amazon 26215 x 241915,
45 nnz/row: 1.94 MB fp64 messages; covtype 396112 x 15509; kc_house 17290 x 27654; synthetic,
parity unpinned), host-driven with HIP-event instrumentation, and prints every rank's report
(Trainer.rank_report): gradient kernel, beta / message put+signal, beta wait, master wait-for-k,
decode and combine+update microseconds.  With --gpus N > 1 it relaunches itself under
torch.distributed.run like bench.py; on a one-GPU box the ranks time-share the GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DATA = {"amazon": "amazon-dataset", "covtype": "covtype", "kc_house": "kc_house_data"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--data", default="amazon", choices=sorted(DATA))
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--json-out", default=None)
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        import bench  # noqa: E402  (repo root on sys.path)

        return bench.relaunch(a.gpus, argv, script=os.path.abspath(__file__))
    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.data.source import ArraySource
    from erasurehead_amd.data.synthetic import REAL_SHAPES, onehot_partitions
    from erasurehead_amd.engine import Trainer
    from erasurehead_amd.parallel.dist import init_distributed

    env = init_distributed("auto")
    n, d, f = REAL_SHAPES[DATA[a.data]]
    W = 8
    parts, test, dd = onehot_partitions(n, d, f, W, seed=21, least_squares=a.data == "kc_house")
    src = ArraySource(parts, test, sparse=True)
    nr = sum(p[0].shape[0] for p in parts)
    cfg = RunConfig(W + 1, nr, dd, "/tmp/eh_ranks/", 1, DATA[a.data], 1, 1, 0, 3, 6, 0, "AGD", num_itrs=a.rounds,
                    seed=0, verbose=False, device_loop="off", instrument=True, round_timeout=120.0,
                    loss="least_squares" if a.data == "kc_house" else "auto")
    tr = Trainer(cfg, env, src)
    res = tr.run(timed_start=a.warmup)
    t = env.allreduce_max(res.timed_seconds if env.is_master else tr.worker_timed_seconds)
    reps = env.gather_objects(tr.rank_report())
    if env.is_master:
        out = {"data": DATA[a.data] + " (one-hot stand-in, parity unpinned)", "n_rows": nr, "n_cols": dd,
               "ranks_launched": env.world, "ms_per_round": 1e3 * t / (a.rounds - a.warmup),
               "message_bytes": tr.ld * 8, "transport": tr.transport, "ranks": reps}
        print(json.dumps(out), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as fo:
                fo.write(json.dumps(out) + "\n")
    env.barrier()
    tr.close()
    env.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
