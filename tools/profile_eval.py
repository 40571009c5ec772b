"""Where the post-hoc evaluation's time goes (ref src/naive.py:184-198: every stored beta is
evaluated on the training and test sets after training).

    python tools/profile_eval.py [--out FILE] [--rounds 100]

Headline shapes: 8 resident training partitions (1e6 x 1000 fp64, on-device GMM), the 2e5-row
test set and R = 100 betas.  The three phases of engine/evaluate.py are timed separately with a
device sync around each — training-loss GEMM (MFMA, loss fused in the epilogue), test GEMM that
also writes the predictions, batched device AUC — first COLD (the first call in the process:
code-object loading of every kernel involved) and then warm (median of 5).  Achieved fp64
TFLOP/s of the GEMMs are against the 78.6 TF fp64 matrix peak.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--n-rows", type=int, default=1_000_000)
    ap.add_argument("--n-cols", type=int, default=1000)
    a = ap.parse_args()
    import torch

    from erasurehead_amd.data.source import SyntheticSource
    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import get_precision
    from erasurehead_amd.ops.eval import auc_columns, loss_sums, predictions_and_loss

    dev = torch.device("cuda")
    prec = get_precision("fp64")
    d, R = a.n_cols, a.rounds
    src = SyntheticSource(a.n_rows, d, 8, 1234)
    t0 = time.perf_counter()
    parts = [src.partition(p, prec, dev) for p in range(8)]
    Xt, yt = src.test(prec, dev)
    torch.cuda.synchronize()
    t_data = time.perf_counter() - t0
    ld = prec.ld(d)
    B = torch.zeros((R, ld), dtype=torch.float64, device=dev)
    B[:, :d] = torch.randn(R, d, device=dev, dtype=torch.float64) * 0.05

    def phases():
        out = {}
        torch.cuda.synchronize()
        t = time.perf_counter()
        sums, n = loss_sums(iter(parts), B, d, LOGISTIC)
        torch.cuda.synchronize()
        out["train_loss_gemm_s"] = time.perf_counter() - t
        t = time.perf_counter()
        P, tsum = predictions_and_loss(Xt, yt, B, d, LOGISTIC)
        torch.cuda.synchronize()
        out["test_gemm_s"] = time.perf_counter() - t
        t = time.perf_counter()
        auc = auc_columns(yt, P)
        torch.cuda.synchronize()
        out["auc_s"] = time.perf_counter() - t
        out["total_s"] = sum(out.values())
        return out

    cold = phases()
    warm_runs = [phases() for _ in range(5)]
    # the same training GEMM as ONE launch over a contiguous 1e6-row copy (launch count / tail effects)
    from erasurehead_amd._ext import native as _nat

    Xall = torch.cat([x for x, _ in parts])
    yall = torch.cat([y for _, y in parts])
    s1 = torch.zeros(R, dtype=torch.float64, device=dev)
    ts1 = []
    for _ in range(6):
        s1.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        _nat().eval_gemm_loss(LOGISTIC, Xall, Xall.shape[0], d, yall, B, s1, None)
        torch.cuda.synchronize()
        ts1.append(time.perf_counter() - t)
    one_launch_s = float(np.median(ts1[1:]))
    del Xall, yall
    warm = {k: float(np.median([w[k] for w in warm_runs])) for k in warm_runs[0]}
    flop_train = 2.0 * a.n_rows * d * R
    flop_test = 2.0 * Xt.shape[0] * d * R
    rec = {"n_rows": a.n_rows, "n_test": int(Xt.shape[0]), "d": d, "R": R, "data_setup_s": t_data,
           "cold": cold, "warm": warm,
           "train_gemm_TFps_warm": flop_train / warm["train_loss_gemm_s"] / 1e12,
           "test_gemm_TFps_warm": flop_test / warm["test_gemm_s"] / 1e12,
           "fp64_peak_TF": 78.6,
           "cold_minus_warm_s": cold["total_s"] - warm["total_s"],
           "train_gemm_one_launch_s": one_launch_s,
           "train_gemm_one_launch_TFps": flop_train / one_launch_s / 1e12}
    rec["train_gemm_frac_of_peak"] = rec["train_gemm_TFps_warm"] / 78.6
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
