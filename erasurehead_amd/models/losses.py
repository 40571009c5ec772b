"""Model math: logistic regression (L2) and least squares — fp64 NumPy oracles.

These are the reference formulas verbatim (SURVEY §2.2 "Math spec"), kept independent
of the device path so the HIP kernels can be checked against them:

  logistic worker gradient   g = -X^T( y_mod / (exp(y * (X beta)) + 1) )   ref src/naive.py:137-139
  least-squares gradient     g = -2 X^T (y - X beta)                        ref src/naive.py:345-346
  GD                         beta <- (1 - 2 alpha eta) beta - (eta/n) g      ref src/naive.py:112-115
  AGD (theta = 2/(i+2))      y = (1-theta) beta + theta u
                             beta' = y - (eta/n) g - 2 alpha eta beta
                             u = beta + (beta' - beta)/theta                 ref src/naive.py:116-122
  training loss              (1/n) sum log(1 + exp(-y * p))                 ref src/util.py:136-137
  MSE                        mean (y - p)^2                                  ref src/util.py:139-141
  AUC                        area under ROC of scores p vs labels in {-1,1}  ref src/naive.py:196-197
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

LOGISTIC = 0
LEAST_SQUARES = 1
LOSS_NAMES = {"logistic": LOGISTIC, "least_squares": LEAST_SQUARES}


def _sigmoid_neg(t: np.ndarray) -> np.ndarray:
    """1 / (exp(t) + 1) without overflow warnings."""
    out = np.empty_like(t, dtype=np.float64)
    pos = t > 0
    e = np.exp(-t[pos])
    out[pos] = e / (1.0 + e)
    out[~pos] = 1.0 / (1.0 + np.exp(t[~pos]))
    return out


def logistic_grad(X, y: np.ndarray, beta: np.ndarray, coef=None) -> np.ndarray:
    """-X^T (coef*y / (exp(y * X beta) + 1)); X dense ndarray or scipy sparse."""
    z = X.dot(beta)
    ymod = y if coef is None else coef * y
    r = -ymod * _sigmoid_neg(y * z)
    return np.asarray(X.T.dot(r)).ravel()


def least_squares_grad(X, y: np.ndarray, beta: np.ndarray, coef=None) -> np.ndarray:
    z = X.dot(beta)
    c = 1.0 if coef is None else coef
    r = -2.0 * c * (y - z)
    return np.asarray(X.T.dot(r)).ravel()


def worker_grad(kind: int, X, y, beta, coef=None) -> np.ndarray:
    return logistic_grad(X, y, beta, coef) if kind == LOGISTIC else least_squares_grad(X, y, beta, coef)


def logistic_loss(y: np.ndarray, p: np.ndarray, n: Optional[int] = None) -> float:
    """(1/n) sum log(1 + exp(-y p)) in a stable form (identical where the reference is finite)."""
    m = -np.asarray(y) * np.asarray(p)
    v = np.maximum(m, 0.0) + np.log1p(np.exp(-np.abs(m)))
    return float(v.sum() / (len(y) if n is None else n))


def mse(y: np.ndarray, p: np.ndarray) -> float:
    d = np.asarray(y, dtype=np.float64) - np.asarray(p, dtype=np.float64)
    return float(np.mean(d * d))


def roc_auc(y: np.ndarray, scores: np.ndarray, pos_label: float = 1) -> float:
    """ROC AUC with ties counted 1/2 — equal to sklearn roc_curve + auc (trapezoid)."""
    y = np.asarray(y)
    s = np.asarray(scores, dtype=np.float64)
    pos = y == pos_label
    n_pos = int(pos.sum())
    n_neg = len(y) - n_pos
    if n_pos == 0 or n_neg == 0:
        return float("nan")
    order = np.argsort(s, kind="mergesort")
    ss = s[order]
    ranks = np.empty(len(s))
    # average ranks over ties
    i = 0
    n = len(s)
    idx = np.flatnonzero(np.diff(ss)) + 1
    starts = np.concatenate([[0], idx])
    ends = np.concatenate([idx, [n]])
    avg = (starts + ends - 1) / 2.0 + 1.0
    ranks_sorted = np.repeat(avg, ends - starts)
    ranks[order] = ranks_sorted
    u = ranks[pos].sum() - n_pos * (n_pos + 1) / 2.0
    return float(u / (n_pos * n_neg))


@dataclass
class UpdateRule:
    """GD / AGD with the reference's constants (alpha = 1/n_rows, eta schedule)."""

    rule: str  # "GD" | "AGD"
    alpha: float
    n_samples: int
    grad_scale: float = 1.0

    def coeffs(self, i: int, eta: float) -> Tuple[float, float, float, float, int]:
        """(decay, grad_multiplier, l2, theta, rule_code) for round i."""
        gm = eta / self.n_samples * self.grad_scale
        decay = 1.0 - 2.0 * self.alpha * eta
        l2 = 2.0 * self.alpha * eta
        theta = 2.0 / (i + 2.0)
        return decay, gm, l2, theta, (0 if self.rule == "GD" else 1)

    def apply(self, i: int, eta: float, beta: np.ndarray, u: np.ndarray, g: np.ndarray) -> None:
        """In-place host update (oracle of the combine_update kernel)."""
        decay, gm, l2, theta, code = self.coeffs(i, eta)
        if code == 0:
            np.subtract(decay * beta, gm * g, out=beta)
        else:
            ytemp = (1 - theta) * beta + theta * u
            betatemp = ytemp - gm * g - l2 * beta
            u[:] = beta + (betatemp - beta) * (1 / theta)
            beta[:] = betatemp
