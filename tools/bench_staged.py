"""Headline-layout gradient kernel timing (FRC replicas on one GPU: 22 GB of message rows over 8 GB).

Used by tools/sweep_staged.sh-style A/B runs: the kernel choice comes from the environment
(ERASUREHEAD_STAGED, ERASUREHEAD_BUNDLE_ROWS, ERASUREHEAD_STAGE_ROWS, ...), the loss from --loss
(least squares has no exp in the residual: the difference isolates the per-row scalar work).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loss", choices=["logistic", "ls"], default="logistic")
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    ap.add_argument("--layout", choices=["agc", "frc1"], default="agc")
    a = ap.parse_args()
    import torch

    from erasurehead_amd.models.losses import LEAST_SQUARES, LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    prec = get_precision(a.precision)
    d, rpp = 1000, 125000
    g = torch.Generator(device="cuda").manual_seed(0)
    parts = {}
    for p in range(8):
        X = (torch.randn(rpp, prec.ld(d), device="cuda", dtype=torch.float32, generator=g) * 0.03).to(prec.storage)
        y = torch.where(torch.rand(rpp, device="cuda", generator=g) > 0.5, 1.0, -1.0).to(prec.acc)
        parts[p] = (X, y)
    beta = torch.randn(prec.ld(d), device="cuda", dtype=prec.acc, generator=g) * 0.01
    frc = [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2  # AGC W=8 s=2 (--layout agc)
    if a.layout == "frc1":  # exact FRC W=8 s=1: four groups of 2
        frc = [[0, 1]] * 2 + [[2, 3]] * 2 + [[4, 5]] * 2 + [[6, 7]] * 2
    loss = LOGISTIC if a.loss == "logistic" else LEAST_SQUARES
    plan = DenseGradPlan([[(p, 1.0) for p in m] for m in frc], parts, prec, loss, d)
    G = plan.out_buffer()[0]
    for _ in range(5):
        plan.run(beta, G)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(a.reps):
        s.record()
        plan.run(beta, G)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    times.sort()
    print(json.dumps({"tag": a.tag, "layout": a.layout, "loss": a.loss, "precision": a.precision, "variant": plan.variant,
                      "ms_median": times[len(times) // 2], "ms_min": times[0],
                      "distinct_TBps": plan.distinct_bytes / 1e9 / times[len(times) // 2]}), flush=True)


if __name__ == "__main__":
    main()
