"""Synthetic two-component GMM data with logistic labels (ref src/generate_data.py).

Model (ref src/generate_data.py:23-45, src/util.py:39-47):
  beta*  = random +-1 vector of length d
  mu_1,2 = +-(1.5 / d) beta*
  per partition of n/P rows: c2 ~ Binomial(rows, 1/2) rows around mu_2, the rest around
  mu_1 (mu_1 rows first), each row = (10 / sqrt(d)) N(0, I) + mu_k
  y = 2 Bernoulli(sigmoid(X beta*)) - 1
  test set: 0.2 n rows from the same model.

Two generators share that model:
  * :func:`generate_to_disk` — the reference CLI's text layout, NumPy on the host;
  * :class:`DeviceGMM` — the same distribution drawn straight into HBM with the torch
    Philox generator, one independent deterministic stream per
    partition, so every rank regenerates exactly the partitions its logical workers
    hold without any file I/O (1e6 x 1e3 fp64 = 8 GB in well under a second).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import io as dio


def random_binvec(n: int, rng: np.random.RandomState) -> np.ndarray:
    """+-1 vector (ref src/util.py:46-47)."""
    return rng.randint(2, size=n) * 2 - 1


def gmm_matrix(mu1: np.ndarray, mu2: np.ndarray, n_rows: int, n_cols: int, rng: np.random.RandomState) -> np.ndarray:
    """ref src/util.py:39-43."""
    c2 = rng.binomial(n_rows, 0.5)
    c1 = n_rows - c2
    mfac = 10 / np.sqrt(n_cols)
    return np.concatenate((mfac * rng.standard_normal((c1, n_cols)) + mu1,
                           mfac * rng.standard_normal((c2, n_cols)) + mu2))


def generate_to_disk(n_rows: int, n_cols: int, partitions: int, out_dir: str,
                     rng: Optional[np.random.RandomState] = None, verbose: bool = True) -> None:
    """Write the reference layout <out_dir>/{1..P}.dat, label.dat, test_data.dat, label_test.dat."""
    assert n_rows % partitions == 0, "n_rows must be a multiple of the number of partitions"
    rng = rng if rng is not None else np.random.mtrand._rand
    rpw = n_rows // partitions
    os.makedirs(out_dir, exist_ok=True)
    if verbose:
        print("Generating Partitioned Matrix Of size %d x %d for a total of %d partitions" % (n_rows, n_cols, partitions))
        print(">>> Each worker gets a matrix of %d x %d doubles, %.2f MB each" % (rpw, n_cols, (rpw * n_cols * 8) / 1000000.0))
    beta = random_binvec(n_cols, rng)
    mu1 = (1.5 / n_cols) * beta
    mu2 = (-1.5 / n_cols) * beta
    labels = np.ndarray(n_rows)
    for i in range(1, partitions + 1):
        X = gmm_matrix(mu1, mu2, rpw, n_cols, rng)
        dio.save_matrix(X, os.path.join(out_dir, str(i) + ".dat"))
        prob = 1.0 / (1 + np.exp(-X.dot(beta)))
        labels[(i - 1) * rpw:i * rpw] = 2 * rng.binomial(1, prob) - 1
        if verbose:
            print("\t >>> Done with partition %d" % i)
    dio.save_vector(labels, os.path.join(out_dir, "label.dat"))
    Xt = gmm_matrix(mu1, mu2, int(0.2 * n_rows), n_cols, rng)
    prob = 1.0 / (1 + np.exp(-Xt.dot(beta)))
    yt = 2 * rng.binomial(1, prob) - 1
    dio.save_matrix(Xt, os.path.join(out_dir, "test_data.dat"))
    dio.save_vector(yt, os.path.join(out_dir, "label_test.dat"))
    if verbose:
        print("\t >>> Done with Test data")


def synthetic_dir(output_dir: str, n_procs: int, n_rows: int, n_cols: int, n_stragglers: int,
                  n_partitions: int, partial_coded: int) -> Tuple[str, int]:
    """Directory + partition count of ref src/generate_data.py:62-71."""
    output_dir = output_dir if output_dir.endswith("/") else output_dir + "/"
    base = output_dir + "artificial-data/" + str(n_rows) + "x" + str(n_cols) + "/"
    if not partial_coded:
        return base + str(n_procs - 1) + "/", n_procs - 1
    parts = (n_procs - 1) * (n_partitions - n_stragglers)
    return base + "partial/" + str(parts) + "/", parts


@dataclass
class DeviceGMM:
    """Deterministic on-device generator of the reference's synthetic model."""

    n_rows: int
    n_cols: int
    n_partitions: int
    seed: int = 0
    ld: Optional[int] = None

    def __post_init__(self):
        if self.n_rows % self.n_partitions:
            raise ValueError("n_rows must be a multiple of the number of partitions")
        rng = np.random.RandomState(self.seed)
        self.beta_star = random_binvec(self.n_cols, rng).astype(np.float64)
        if self.ld is None:
            self.ld = self.n_cols

    @property
    def rows_per_partition(self) -> int:
        return self.n_rows // self.n_partitions

    def _draw(self, n: int, stream: int, device, dtype):
        import torch

        d = self.n_cols
        host = np.random.RandomState((self.seed * 1000003 + stream * 7919 + 17) % (2 ** 31))
        c2 = int(host.binomial(n, 0.5))
        c1 = n - c2
        gen = torch.Generator(device=device)
        gen.manual_seed(int(host.randint(0, 2 ** 62)))
        X = torch.zeros((n, self.ld), dtype=torch.float64, device=device)
        body = X[:, :d]
        body.normal_(generator=gen)
        body.mul_(10.0 / math.sqrt(d))
        bstar = torch.as_tensor(self.beta_star, device=device)
        mu = (1.5 / d) * bstar
        body[:c1].add_(mu)
        body[c1:].sub_(mu)
        prob = torch.sigmoid(body @ bstar)
        y = 2.0 * torch.bernoulli(prob, generator=gen) - 1.0
        return X.to(dtype) if dtype != torch.float64 else X, y

    def partition(self, p: int, device="cpu", dtype=None):
        """(X [rows, ld], y [rows]) of 0-based partition p."""
        import torch

        return self._draw(self.rows_per_partition, p, device, dtype or torch.float64)

    def test(self, device="cpu", dtype=None):
        import torch

        return self._draw(int(0.2 * self.n_rows), 10 ** 6 + 1, device, dtype or torch.float64)


# ------------------------------------------------------------------ one-hot (real-data-shaped)
REAL_SHAPES = {  # (train rows, one-hot columns, original columns incl. bias) of the prepared datasets
    "covtype": (396112, 15509, 55),  # ref run_approx_coding.sh:26-28
    "kc_house_data": (17290, 27654, 19),  # ref run_approx_coding.sh:34-36
    "amazon-dataset": (26215, 241915, 45),  # ref run_approx_coding.sh:30-32 (9 + 35 interactions + bias)
}


def onehot_partitions(n_rows: int, n_cols: int, n_feat: int, n_partitions: int, seed: int = 0,
                      least_squares: bool = False, test_frac: float = 0.25):
    """Synthetic one-hot CSR data with the structure of the prepared real datasets.

    Every row has exactly ``n_feat`` nonzeros (one category of each original column, the
    last column being the single-category bias), all values 1.0 — the layout
    ``arrange_real_data.py`` produces.  Labels follow a planted model:
    logistic ``y = 2 Bernoulli(sigmoid(x . w*)) - 1`` or least squares ``y = x . w* + noise``.
    Returns (partitions [(csr, y)], (test_csr, y_test)) with ``n_rows // n_partitions`` rows
    per partition.
    """
    from scipy.sparse import csr_matrix

    rng = np.random.RandomState(seed)
    n_real = n_feat - 1
    base = max(2, (n_cols - 1) // max(1, n_real))
    cards = np.full(n_real, base, dtype=np.int64)
    cards[: max(0, (n_cols - 1) - base * n_real)] += 1  # spread the remainder: sum(cards) = n_cols - 1
    offs = np.concatenate([[0], np.cumsum(cards)])
    d = int(offs[-1]) + 1
    w_star = rng.normal(0, 1.0 / np.sqrt(n_feat), d)

    def draw(n):
        # skewed category frequencies (Zipf-like), like real categorical columns
        cols = np.empty((n, n_feat), dtype=np.int64)
        for j in range(n_real):
            u = rng.power(3.0, n)
            cols[:, j] = offs[j] + np.minimum((u * cards[j]).astype(np.int64), cards[j] - 1)
        cols[:, -1] = d - 1
        indptr = np.arange(0, n * n_feat + 1, n_feat, dtype=np.int64)
        X = csr_matrix((np.ones(n * n_feat), cols.ravel().astype(np.int32), indptr), shape=(n, d))
        z = np.asarray(X @ w_star).ravel()
        if least_squares:
            y = z + 0.1 * rng.standard_normal(n)
        else:
            y = 2.0 * rng.binomial(1, 1.0 / (1.0 + np.exp(-3.0 * z))) - 1.0
        return X, y

    rpw = n_rows // n_partitions
    parts = [draw(rpw) for _ in range(n_partitions)]
    test = draw(max(1, int(test_frac * n_rows)))
    return parts, test, d
