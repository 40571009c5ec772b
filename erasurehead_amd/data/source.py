"""Data sources: where worker partitions and the evaluation sets come from.

* :class:`FileSource`      — the reference on-disk layout (text ``.dat`` / CSR ``.npz``);
* :class:`SyntheticSource` — the reference GMM model drawn directly on the device;
* :class:`ArraySource`     — in-memory arrays (tests, notebooks).

Every source hands out partitions by 0-based index, already in the worker layout:
dense X as a contiguous ``[rows, ld]`` tensor in the storage precision (zero-padded
columns), labels in the accumulator precision; sparse X as ``scipy.sparse.csr_matrix``.
Labels of partition p are rows ``[p*rpw, (p+1)*rpw)`` of the full label vector, exactly
like the reference's slicing (ref src/replication.py:52).
"""
from __future__ import annotations

import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops.precision import Precision
from . import io as dio
from .synthetic import DeviceGMM


def _pad_dense(X, prec: Precision, device) -> torch.Tensor:
    if not isinstance(X, torch.Tensor):  # memory-mapped .npy twins are read-only: copy those
        X = torch.from_numpy(np.require(np.asarray(X, dtype=np.float64), requirements=["W", "C"]))
    if X.dim() == 1:
        X = X[None, :]
    n, d = X.shape
    ld = prec.ld(d)
    out = torch.zeros((n, ld), dtype=prec.storage, device=device)
    out[:, :d] = X.to(device=device, dtype=torch.float64).to(prec.storage)
    return out


class DataSource:
    is_sparse = False
    d: int

    def partition(self, p: int, prec: Precision, device):
        raise NotImplementedError

    def train_eval_chunks(self, parts: Sequence[int], prec: Precision, device) -> Iterator[Tuple[object, torch.Tensor]]:
        """(X, y) of the given partitions, in order, labels taken from the *prefix* of label.dat."""
        raise NotImplementedError

    def test(self, prec: Precision, device) -> Tuple[object, torch.Tensor]:
        raise NotImplementedError


class FileSource(DataSource):
    def __init__(self, data_dir: str, is_real: int, rows_per_partition: int, n_cols: int):
        self.data_dir = data_dir
        self.is_real = int(is_real)
        self.is_sparse = bool(is_real)
        self.rpw = int(rows_per_partition)
        self.d = int(n_cols)
        self._labels: Optional[np.ndarray] = None

    def labels(self) -> np.ndarray:
        if self._labels is None:
            self._labels = dio.load_labels(self.data_dir)
        return self._labels

    def partition(self, p: int, prec: Precision, device):
        X = dio.load_partition(self.data_dir, p, self.is_real)
        y = self.labels()[p * self.rpw:(p + 1) * self.rpw]
        if X.shape[0] != len(y):
            raise ValueError(f"partition {p + 1}: {X.shape[0]} rows but {len(y)} labels; check n_rows")
        if self.is_sparse:
            return X, np.asarray(y, dtype=np.float64)
        return _pad_dense(X, prec, device), torch.tensor(np.asarray(y), dtype=prec.acc, device=device)

    def train_eval_chunks(self, parts, prec, device):
        y = self.labels()
        off = 0
        for p in parts:
            X = dio.load_partition(self.data_dir, p, self.is_real)
            n = X.shape[0]
            yy = torch.tensor(np.asarray(y[off:off + n]), dtype=torch.float64, device=device)
            off += n
            yield (X if self.is_sparse else _pad_dense(X, prec, device)), yy

    def test(self, prec, device):
        X = dio.load_test(self.data_dir, self.is_real)
        y = torch.tensor(np.asarray(dio.load_labels(self.data_dir, test=True)), dtype=torch.float64, device=device)
        return (X if self.is_sparse else _pad_dense(X, prec, device)), y


class SyntheticSource(DataSource):
    """Partitions of the reference synthetic model generated on the device (no files)."""

    def __init__(self, n_rows: int, n_cols: int, n_partitions: int, seed: int = 0):
        self.gen = DeviceGMM(n_rows, n_cols, n_partitions, seed)
        self.d = n_cols

    def partition(self, p, prec, device):
        self.gen.ld = prec.ld(self.d)
        X, y = self.gen.partition(p, device=device, dtype=prec.storage)
        return X.contiguous(), y.to(prec.acc)

    def train_eval_chunks(self, parts, prec, device):
        self.gen.ld = prec.ld(self.d)
        for p in parts:
            X, y = self.gen.partition(p, device=device, dtype=prec.storage)
            yield X.contiguous(), y

    def test(self, prec, device):
        self.gen.ld = prec.ld(self.d)
        X, y = self.gen.test(device=device, dtype=prec.storage)
        return X.contiguous(), y


class ArraySource(DataSource):
    """parts: list of (X, y) numpy arrays or scipy CSR; test: (X, y)."""

    def __init__(self, parts: List[Tuple[object, np.ndarray]], test: Tuple[object, np.ndarray], sparse: bool = False):
        self.parts = parts
        self._test = test
        self.is_sparse = sparse
        self.d = parts[0][0].shape[1]

    def partition(self, p, prec, device):
        X, y = self.parts[p]
        if self.is_sparse:
            return X, np.asarray(y, dtype=np.float64)
        return _pad_dense(X, prec, device), torch.tensor(np.asarray(y), dtype=prec.acc, device=device)

    def train_eval_chunks(self, parts, prec, device):
        ys = np.concatenate([np.asarray(y) for _, y in self.parts])
        off = 0
        for p in parts:
            X = self.parts[p][0]
            n = X.shape[0]
            yy = torch.as_tensor(ys[off:off + n], dtype=torch.float64, device=device)
            off += n
            yield (X if self.is_sparse else _pad_dense(X, prec, device)), yy

    def test(self, prec, device):
        X, y = self._test
        yy = torch.as_tensor(np.asarray(y), dtype=torch.float64, device=device)
        return (X if self.is_sparse else _pad_dense(X, prec, device)), yy
