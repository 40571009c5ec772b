"""Post-hoc evaluation of every stored beta (K9-K11; ref src/naive.py:186-198).

Dense data: the MFMA GEMM P = X B^T with the loss reduction fused in its epilogue
(csrc/kernels/eval.hip), streamed partition by partition so the training set never
has to be resident at once.  Test predictions are materialised for the ROC AUC, which
is a rank statistic computed on the device with a sort per round (ties count 1/2, i.e.
exactly sklearn's trapezoidal roc_curve + auc).
Sparse data (the reference's one-hot real datasets): the hand-written CSR kernel
(csrc/kernels/eval_sparse.hip) gathers rows of the transposed betas Bt [ld, R] per non-zero and
fuses the same loss epilogue; pattern-only rows (every value 1) carry no value array.  CPU
tensors use torch CSR products (tests).
"""
from __future__ import annotations

from typing import Iterable, Tuple

import numpy as np
import torch

from .._ext import native
from ..models.losses import LOGISTIC


def _loss_torch(kind: int, y: torch.Tensor, P: torch.Tensor) -> torch.Tensor:
    y = y.double()[:, None]
    P = P.double()
    if kind == LOGISTIC:
        m = -y * P
        return (torch.clamp(m, min=0) + torch.log1p(torch.exp(-m.abs()))).sum(0)
    e = y - P
    return (e * e).sum(0)


def _is_sparse(X) -> bool:
    return not isinstance(X, torch.Tensor) or X.layout != torch.strided


def _to_torch_sparse(X, device, dtype):
    import warnings

    import scipy.sparse as sps

    X = sps.csr_matrix(X)
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta state")
        return _csr(X, device, dtype)


def _csr(X, device, dtype):
    return torch.sparse_csr_tensor(torch.from_numpy(X.indptr.astype(np.int64)),
                                   torch.from_numpy(X.indices.astype(np.int64)),
                                   torch.from_numpy(X.data.astype(np.float64)), size=X.shape,
                                   dtype=dtype, device=device)


def _csr_operands(X, device, acc):
    """(row_ptr int64, col int32, vals or None if pattern-only, n, max column + 1) of a scipy CSR
    matrix on the device (a tuple already in this form is passed through)."""
    if isinstance(X, tuple):
        return X
    import scipy.sparse as sps

    X = X if sps.isspmatrix_csr(X) else sps.csr_matrix(X)
    npacc = np.float64 if acc == torch.float64 else np.float32
    pattern = X.nnz == 0 or (X.data.min() == 1.0 and X.data.max() == 1.0)
    ind = X.indices if X.indices.dtype == np.int32 else X.indices.astype(np.int32)
    row_ptr = torch.from_numpy(np.asarray(X.indptr, dtype=np.int64)).to(device)
    col = torch.from_numpy(ind).to(device)
    vals = None if pattern else torch.from_numpy(np.asarray(X.data, dtype=npacc)).to(device)
    # the kernel gathers Bt[col]: bound every index on the host (scipy does not validate them)
    return row_ptr, col, vals, X.shape[0], (int(ind.max()) + 1 if X.nnz else 0)


def sparse_eval_device(X, y: torch.Tensor, Bt: torch.Tensor, kind: int, want_P: bool):
    """(P [n, R] or None, per-beta loss sums [R] fp64 on the device) with the native CSR kernel.

    X: scipy CSR, or the operands of :func:`_csr_operands` (already on the device).
    Bt: the betas transposed, [ld, R] in the accumulator dtype (R > 256 runs in column passes)."""
    acc = Bt.dtype
    row_ptr, col, vals, n, maxc = _csr_operands(X, Bt.device, acc)
    if maxc > Bt.shape[0]:
        raise ValueError(f"sparse eval: column index {maxc - 1} outside the {Bt.shape[0]} beta features")
    R = Bt.shape[1]
    yd = y.to(device=Bt.device, dtype=acc).contiguous()
    s = torch.zeros(R, dtype=torch.float64, device=Bt.device)
    P = torch.empty((n, R), dtype=acc, device=Bt.device) if want_P else None
    C = native()
    for c0 in range(0, R, 256):
        c1 = min(R, c0 + 256)
        Bc = Bt[:, c0:c1].contiguous()
        Pc = torch.empty((n, c1 - c0), dtype=acc, device=Bt.device) if want_P and (c0 or c1 < R) else P
        sc = s[c0:c1] if (c0 == 0 and c1 == R) else torch.zeros(c1 - c0, dtype=torch.float64, device=Bt.device)
        C.eval_csr_loss(kind, row_ptr, col, vals, n, yd, Bc, sc, Pc)
        if sc is not s:
            s[c0:c1] = sc
        if want_P and Pc is not P:
            P[:, c0:c1] = Pc
    return P, s


def _transposed(B: torch.Tensor, acc) -> torch.Tensor:
    return B.to(acc).t().contiguous()


def predictions(X, B: torch.Tensor, d: int) -> torch.Tensor:
    """P = X[:, :d] @ B[:, :d]^T  ([n, R], accumulator dtype of X)."""
    if _is_sparse(X):
        Xt = _to_torch_sparse(X, B.device, torch.float64)
        return (Xt @ B[:, :d].double().t().contiguous())
    n = X.shape[0]
    acc = torch.float64 if X.dtype == torch.float64 else torch.float32
    Bc = B.to(acc).contiguous()
    if X.is_cuda:
        P = torch.empty((n, B.shape[0]), dtype=acc, device=X.device)
        junk = torch.zeros(B.shape[0], dtype=torch.float64, device=X.device)
        yz = torch.zeros(n, dtype=acc, device=X.device)
        native().eval_gemm_loss(LOGISTIC, X, n, d, yz, Bc, junk, P)
        return P
    return X[:, :d].to(acc) @ Bc[:, :d].t()


def predictions_and_loss(X, y: torch.Tensor, B: torch.Tensor, d: int, kind: int) -> Tuple[torch.Tensor, np.ndarray]:
    """(P = X B^T, per-beta loss sums) — on the GPU one MFMA GEMM with the loss fused in its epilogue."""
    if _is_sparse(X) and B.is_cuda:
        P, s = sparse_eval_device(X, y, _transposed(B, torch.float64), kind, True)
        return P, s.cpu().numpy()
    if not _is_sparse(X) and X.is_cuda:
        n = X.shape[0]
        acc = torch.float64 if X.dtype == torch.float64 else torch.float32
        P = torch.empty((n, B.shape[0]), dtype=acc, device=X.device)
        s = torch.zeros(B.shape[0], dtype=torch.float64, device=X.device)
        native().eval_gemm_loss(kind, X, n, d, y.to(acc).contiguous(), B.to(acc).contiguous(), s, P)
        return P, s.cpu().numpy()
    P = predictions(X, B, d)
    return P, _loss_torch(kind, y.to(P.device), P).double().cpu().numpy()


def loss_sums(chunks: Iterable[Tuple[object, torch.Tensor]], B: torch.Tensor, d: int, kind: int) -> Tuple[np.ndarray, int]:
    """Sum over all chunk rows of the per-row loss for every beta row of B -> ([R], n)."""
    R = B.shape[0]
    total = None
    n = 0
    Bt = None
    for X, y in chunks:
        if _is_sparse(X) and B.is_cuda:
            if Bt is None:
                Bt = _transposed(B, torch.float64)
            _, s = sparse_eval_device(X, y, Bt, kind, False)
        elif _is_sparse(X):
            P = predictions(X, B, d)
            s = _loss_torch(kind, y.to(P.device), P)
        elif X.is_cuda:
            acc = torch.float64 if X.dtype == torch.float64 else torch.float32
            s = torch.zeros(R, dtype=torch.float64, device=X.device)
            native().eval_gemm_loss(kind, X, X.shape[0], d, y.to(acc).contiguous(), B.to(acc).contiguous(), s, None)
        else:
            P = predictions(X, B, d)
            s = _loss_torch(kind, y, P)
        total = s if total is None else total + s.to(total.device)
        n += X.shape[0]
    if total is None:
        return np.zeros(R), 0
    return total.double().cpu().numpy(), n


def warm_auc(device) -> None:
    """Load the code objects of the AUC path (torch's segmented sort, scans, index_add) once.

    Measured (profiles/round2/s1_eval): the first auc_columns call of a process costs 0.6 s, all of it
    first-use code-object loading (the same call warm: 4.5 ms for 100 x 2e5).  The trainer runs
    this on the master while it generates / loads the training data, so the post-hoc evaluation
    does not pay it."""
    y = torch.tensor([1.0, -1.0, 1.0, -1.0], dtype=torch.float64, device=device)
    P = torch.tensor([[0.1, 0.2], [0.3, 0.1], [0.3, 0.4], [0.0, 0.4]], dtype=torch.float64, device=device)
    auc_columns(y, P)


def auc_columns(y: torch.Tensor, P: torch.Tensor, chunk: int = 0) -> np.ndarray:
    """ROC AUC of every column of P against labels y in {-1, +1} (ties count 1/2).

    Batched Mann-Whitney U over all columns at once (sklearn's trapezoidal roc_curve + auc is
    the same statistic): one column-wise sort, tie groups found by comparing neighbours, the
    average rank of each tie group via a segmented scatter-add, one reduction per column.
    No per-column host synchronisation; ``chunk`` bounds the columns per pass (memory).
    """
    y = y.to(P.device)
    pos = (y == 1)
    n = y.numel()
    n_pos = int(pos.sum().item())
    n_neg = n - n_pos
    R = P.shape[1]
    out = np.full(R, np.nan)
    if n_pos == 0 or n_neg == 0 or R == 0:
        return out
    if chunk <= 0:
        chunk = max(1, min(R, (1 << 26) // max(1, n)))
    ar = torch.arange(1, n + 1, dtype=torch.float64, device=P.device)
    for c0 in range(0, R, chunk):
        S = P[:, c0:c0 + chunk].double().t().contiguous()  # [m, n]: every scan runs along contiguous memory
        m = S.shape[0]
        ss, order = torch.sort(S, dim=1, stable=True)
        pos_s = pos[order]  # [m, n] labels in sorted order
        start = torch.ones_like(ss, dtype=torch.bool)
        start[:, 1:] = ss[:, 1:] != ss[:, :-1]
        seg = torch.cumsum(start.to(torch.int64), dim=1) - 1  # tie-group id within the column
        flat = (seg + torch.arange(m, device=P.device)[:, None] * n).reshape(-1)
        ranks = ar[None, :].expand(m, n).reshape(-1)
        ssum = torch.zeros(n * m, dtype=torch.float64, device=P.device).index_add_(0, flat, ranks)
        scnt = torch.zeros(n * m, dtype=torch.float64, device=P.device).index_add_(0, flat, torch.ones_like(ranks))
        avg = (ssum / scnt.clamp(min=1))[flat].view(m, n)  # average rank of every element
        u = (avg * pos_s).sum(1) - n_pos * (n_pos + 1) / 2.0
        out[c0:c0 + m] = (u / (n_pos * n_neg)).cpu().numpy()
    return out
