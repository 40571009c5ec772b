"""Sparse evaluation: the hand CSR kernel (eval_sparse.hip) vs the library path it replaced.

    python tools/bench_sparse_eval.py [--out FILE]

For the one-hot stand-ins of the reference's real datasets (covtype 396112 x 15509, kc_house
17290 x 27654, amazon 26215 x 241915; synthetic, parity unpinned) and R = 100 betas: the
training-loss pass (no predictions stored) and the test pass (predictions for the AUC), timed
with a device sync (median of 5 after a warm-up), against torch.sparse_csr_tensor @ dense + the
unfused torch loss (round 1's path), once including the scipy CSR -> device upload (what one
evaluation pays) and once on operands already on the device (the kernels alone).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch

    from erasurehead_amd.data.synthetic import REAL_SHAPES, onehot_partitions
    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops.eval import _csr, _csr_operands, _loss_torch, sparse_eval_device

    warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta state")
    recs = []
    for name in ("covtype", "kc_house_data", "amazon-dataset"):
        n, d, f = REAL_SHAPES[name]
        parts, test, dd = onehot_partitions(n, d, f, 1, seed=4)
        X, y = parts[0]
        R = 100
        B = torch.randn(R, dd, dtype=torch.float64, device="cuda") * 0.1
        yd = torch.from_numpy(y).cuda()

        def native_loss():
            Bt = B.t().contiguous()
            return sparse_eval_device(X, yd, Bt, LOGISTIC, False)[1]

        def native_pred():
            Bt = B.t().contiguous()
            return sparse_eval_device(X, yd, Bt, LOGISTIC, True)

        ops = _csr_operands(X, "cuda", torch.float64)
        Xt_dev = _csr(X, "cuda", torch.float64)

        def native_kernel_only():
            return sparse_eval_device(ops, yd, B.t().contiguous(), LOGISTIC, False)[1]

        def torch_spmm_only():
            return _loss_torch(LOGISTIC, yd, Xt_dev @ B.t().contiguous())

        def torch_loss():
            Xt = _csr(X, "cuda", torch.float64)
            P = Xt @ B.t().contiguous()
            return _loss_torch(LOGISTIC, yd, P)

        def timeit(fn):
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            return 1e3 * float(np.median(ts))

        s_nat = native_loss().cpu().numpy()
        s_ref = torch_loss().cpu().numpy()
        rec = {"data": name, "rows": X.shape[0], "cols": dd, "nnz_per_row": f, "R": R,
               "native_loss_ms": timeit(native_loss), "native_pred_and_loss_ms": timeit(native_pred),
               "torch_csr_spmm_loss_ms": timeit(torch_loss),
               "native_kernel_only_ms": timeit(native_kernel_only),
               "torch_spmm_only_ms": timeit(torch_spmm_only),
               "max_rel_diff": float(np.max(np.abs(s_nat - s_ref) / np.abs(s_ref)))}
        rec["speedup"] = rec["torch_csr_spmm_loss_ms"] / rec["native_loss_ms"]
        rec["kernel_speedup"] = rec["torch_spmm_only_ms"] / rec["native_kernel_only_ms"]
        rec["gather_GBps"] = X.nnz * R * 8 / rec["native_kernel_only_ms"] / 1e6
        print(json.dumps(rec), flush=True)
        recs.append(rec)
    if a.out:
        with open(a.out, "w") as fo:
            for r in recs:
                fo.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
