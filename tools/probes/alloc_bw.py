"""Does where a 1 GB partition lands in HBM change how fast it streams?

    python tools/probes/alloc_bw.py [--count 16] [--out FILE]

Allocates --count fp64 partitions of 125000 x 1000 (1 GB each, the headline's partition) one after
another, the way SyntheticSource does (torch caching allocator, one hipMalloc each), then times the
R = 1 gradient (grad_dense_multi, the naive plan) over each partition alternately, clock warmed, 15
samples each.  Identical work per partition: any spread between them is the allocation's.  Also times
the same over one 8 GB allocation cut into eight 1 GB views, and prints the device memory map hints
the allocator exposes (each block's address modulo 2 MB / 1 GB).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    prec = get_precision("fp64")
    rows, d = 125_000, 1000
    ld = prec.ld(d)
    dev = torch.device("cuda")
    beta = torch.randn(ld, device=dev, dtype=torch.float64) * 1e-3

    def plan_of(X):
        y = torch.ones(rows, device=dev, dtype=torch.float64)
        p = DenseGradPlan([[(0, 1.0)]], {0: (X, y)}, prec, LOGISTIC, d)
        return p, p.out_buffer()[0]

    sets = []
    for i in range(a.count):
        X = torch.empty((rows, ld), device=dev, dtype=torch.float64)
        X.normal_()
        sets.append(("separate", i, X) + plan_of(X))
    big = torch.empty((8 * rows, ld), device=dev, dtype=torch.float64)
    big.normal_()
    for i in range(8):
        X = big[i * rows:(i + 1) * rows]
        sets.append(("one_8GB", i, X) + plan_of(X))
    torch.cuda.synchronize()
    tw = time.perf_counter()
    while time.perf_counter() - tw < 0.3:
        for s in sets:
            s[3].run(beta, s[4])
        torch.cuda.synchronize()
    samples = [[] for _ in sets]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(15):
        for j, s in enumerate(sets):
            e0.record()
            for _ in range(4):
                s[3].run(beta, s[4])
            e1.record()
            e1.synchronize()
            samples[j].append(1e3 * e0.elapsed_time(e1) / 4)
    recs = []
    for j, s in enumerate(sets):
        addr = s[2].data_ptr()
        us = float(np.median(samples[j]))
        r = {"layout": s[0], "i": s[1], "us_median": us, "us_min": float(np.min(samples[j])),
             "TBps": rows * ld * 8 / us / 1e6, "addr_mod_2MB": addr % (2 << 20), "addr_GB": addr / 2 ** 30}
        print(json.dumps(r), flush=True)
        recs.append(r)
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
