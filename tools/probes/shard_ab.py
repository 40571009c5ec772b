"""One-GPU A/B of the placement unit at the dense headline: whole messages vs partition shards.

    python tools/probes/shard_ab.py [--schemes agc,cyclic,frc,naive] [--out FILE]

At one rank both units hold every logical worker's rows; they differ only in the local plan's
message slots (8 messages of s+1 segments, or one slot per (worker, partition) segment summed by the
combine).  Prints the isolated gradient launch (Trainer.time_local_grad, clock warmed) and the kernel
choice of each, one JSON line per (scheme, shard); the two trainers of a scheme are timed alternately.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SCHEMES = {  # RunConfig overrides of the BASELINE.json dense configs (tools/bench_suite.py)
    "naive": dict(is_coded=0),
    "agc": dict(is_coded=1, n_stragglers=2, coded_ver=3, num_collect=6, allow_uneven_groups=True),
    "cyclic": dict(is_coded=1, n_stragglers=2, coded_ver=0),
    "frc": dict(is_coded=1, n_stragglers=1, coded_ver=1),
}


def main():
    import numpy as np
    import torch

    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.engine import Trainer
    from erasurehead_amd.parallel.dist import DistEnv

    ap = argparse.ArgumentParser()
    ap.add_argument("--schemes", default="agc,cyclic,frc,naive")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dense = dict(n_procs=9, n_rows=1_000_000, n_cols=1000, input_dir="/tmp/eh_shard_ab/", is_real=0, dataset="synthetic",
                 data="synthetic", data_seed=1234, update_rule="AGD")
    recs = []
    for name in a.schemes.split(","):
        trs = {}
        for shard in ("message", "partition"):
            cfg = RunConfig(**dense, **SCHEMES[name], num_itrs=5, verbose=False, seed=0, shard=shard)
            trs[shard] = Trainer(cfg, DistEnv(device=torch.device("cuda")))
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.3:  # clock ramp (profiles/round3/clocks)
            for tr in trs.values():
                tr.warmup()
            torch.cuda.synchronize()
        samples = {k: [] for k in trs}
        for _ in range(7):  # interleaved, so box drift hits both alike
            for k, tr in trs.items():
                samples[k].append(tr.time_local_grad(reps=20))
        for shard, tr in trs.items():
            plan = getattr(tr.plan, "inner", tr.plan)
            choice = plan.choice.label() if hasattr(plan, "choice") else type(plan).__name__
            r = {"scheme": name, "shard": shard, "slots": len(tr.local_msgs),
                 "grad_us_median": float(np.median(samples[shard])), "grad_us": samples[shard], "kernel": choice}
            print(json.dumps(r), flush=True)
            recs.append(r)
        for tr in trs.values():
            tr.close()
        del trs, tr
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
