"""Known-byte workloads for reading memory-side PMC counters against byte counts (run under
``rocprofv3 --pmc``, tools/gpu_round.sh stage ``pmcbytes``).

    python tools/pmc_calibrate.py [--known FILE]

Three dispatch families, each with a byte count fixed by its shape:
  * ``copy``   torch device copy of 2 GiB fp64: reads 2 GiB, writes 2 GiB;
  * ``naive``  the headline gradient over 8 distinct partitions of 125000 x 1000 fp64 (8 GB read once,
               one-wave bundles of one replica);
  * ``agc``    the same 8 GB through the headline's replica bundles (22 messages, every row read once).
``--known`` writes {kernel-name substring: {"read": bytes, "write": bytes, "calls": n}} for
tools/pmc_summary.py --known, which divides the counters by these counts.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--known", default=None)
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    n = a.calls
    src = torch.empty(2 << 30 >> 3, device="cuda", dtype=torch.float64).uniform_(-1, 1)
    dst = torch.empty_like(src)
    for _ in range(n):
        dst.copy_(src)
    torch.cuda.synchronize()
    del src, dst
    torch.cuda.empty_cache()

    prec = get_precision("fp64")
    d, rpp = 1000, 125_000
    parts = {}
    for p in range(8):
        X = torch.empty(rpp, prec.ld(d), device="cuda", dtype=torch.float64).uniform_(-1, 1)
        y = torch.where(torch.rand(rpp, device="cuda") > 0.5, 1.0, -1.0).double()
        parts[p] = (X, y)
    distinct = 8 * rpp * prec.ld(d) * 8
    beta = torch.randn(prec.ld(d), device="cuda", dtype=torch.float64) * 0.01
    known = {"elementwise": {"read": 2 << 30, "write": 2 << 30, "calls": n, "what": "torch copy 2 GiB fp64"}}
    layouts = {"naive": [[p] for p in range(8)], "agc": [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2}
    for lay, msgs in layouts.items():
        plan = DenseGradPlan([[(p, 1.0) for p in m] for m in msgs], parts, prec, LOGISTIC, d)
        G = plan.out_buffer()[0]
        for _ in range(n):
            plan.run(beta, G)
        torch.cuda.synchronize()
        name = plan.kernel_name() if hasattr(plan, "kernel_name") else None
        known[f"grad_dense {lay}"] = {"read": distinct, "write": None, "calls": n, "choice": plan.choice.label(),
                                      "kernel": name}
        print(lay, plan.choice.label(), flush=True)
        del plan, G
    if a.known:
        with open(a.known, "w") as f:
            json.dump(known, f, indent=1)
    print(json.dumps(known))


if __name__ == "__main__":
    main()
