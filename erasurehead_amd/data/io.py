"""Reference on-disk formats (SURVEY §2.4 "On-disk contract").

  <DATA>/artificial-data/<n>x<d>/<W>/{1..W}.dat, label.dat, test_data.dat, label_test.dat   (text)
  <DATA>/<dataset>/<W>/{1..W}.npz, label.dat, label_test.dat, test_data.npz                 (CSR npz)
  <...>/partial/<(P-s)W>/...                                                                  (partial schemes)
  <input_dir>/results/<prefix>_{training_loss,testing_loss,auc,timeset,worker_timeset}.dat

Writers match ref src/util.py:26-36 byte for byte in layout (``save_vector`` writes
"%5.3f " per line, ``save_matrix`` space-joined ``str(x)`` rows).  Readers accept the
same text; because ``np.loadtxt`` on a multi-GB text partition takes minutes, the first
load of a ``.dat`` matrix leaves a binary ``.npy`` twin next to it (memory-mapped on
later loads).  CSR ``.npz`` files are read with ``allow_pickle=False``.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np


def _npy_twin(path: str) -> str:
    return path + ".npy"


def load_data(path: str, cache: bool = True, mmap: bool = True) -> np.ndarray:
    """Text matrix/vector -> float64 ndarray (ref src/util.py:13-15 np.loadtxt)."""
    twin = _npy_twin(path)
    if cache and os.path.exists(twin) and os.path.getmtime(twin) >= os.path.getmtime(path):
        return np.load(twin, mmap_mode="r" if mmap else None, allow_pickle=False)
    arr = _fast_loadtxt(path)
    if cache:
        try:
            tmp = twin + ".tmp.npy"
            np.save(tmp, arr, allow_pickle=False)
            os.replace(tmp, twin)
        except OSError:
            pass
    return arr


def _fast_loadtxt(path: str) -> np.ndarray:
    try:
        import pandas as pd

        df = pd.read_csv(path, sep=r"\s+", header=None, dtype=np.float64, engine="c")
        arr = df.to_numpy(dtype=np.float64)
    except Exception:
        arr = np.loadtxt(path, dtype=float)
    if arr.ndim == 2 and arr.shape[1] == 1:
        arr = arr[:, 0]
    return np.ascontiguousarray(arr)


def save_matrix(m, output: str) -> None:
    """Rows of space-joined str(x) (ref src/util.py:26-30)."""
    with open(output, "w") as f:
        for row in m:
            f.write(" ".join(str(float(x)) if not isinstance(x, (int, np.integer)) else str(x) for x in row))
            f.write("\n")


def save_vector(m, output: str) -> None:
    """One "%5.3f " value per line (ref src/util.py:32-36; 3 decimals, lossy by design)."""
    with open(output, "w") as f:
        for x in m:
            f.write("%5.3f" % x + " \n")


def save_vector_full(m, output: str) -> None:
    """Full-precision side file (%5.3f loses sub-ms timings)."""
    np.savetxt(output, np.asarray(m, dtype=np.float64), fmt="%.17g")


def save_sparse_csr(filename: str, array) -> None:
    """ref src/util.py:17-19 (np.savez of data/indices/indptr/shape)."""
    np.savez(filename, data=array.data, indices=array.indices, indptr=array.indptr, shape=array.shape)


def load_sparse_csr(filename: str):
    """ref src/util.py:21-24; ``filename`` without the .npz suffix, like the reference."""
    from scipy.sparse import csr_matrix

    path = filename if filename.endswith(".npz") else filename + ".npz"
    with np.load(path, allow_pickle=False) as z:
        return csr_matrix((z["data"], z["indices"], z["indptr"]), shape=tuple(z["shape"]))


def dataset_dir(input_dir: str, is_real: int, dataset: str, n_rows: int, n_cols: int) -> str:
    """ref main.py:59-60: synthetic data lives under artificial-data/<n>x<d>."""
    input_dir = input_dir if input_dir.endswith("/") else input_dir + "/"
    if not is_real:
        dataset = "artificial-data/" + str(n_rows) + "x" + str(n_cols)
    return input_dir + dataset + "/"


def partition_path(data_dir: str, idx0: int, is_real: int) -> str:
    """Partition files are 1-based on disk (ref src/naive.py:29-33)."""
    return os.path.join(data_dir, str(idx0 + 1) + ("" if is_real else ".dat"))


def load_partition(data_dir: str, idx0: int, is_real: int):
    p = partition_path(data_dir, idx0, is_real)
    return load_sparse_csr(p) if is_real else load_data(p)


def load_labels(data_dir: str, test: bool = False) -> np.ndarray:
    return np.asarray(load_data(os.path.join(data_dir, "label_test.dat" if test else "label.dat")), dtype=np.float64)


def load_test(data_dir: str, is_real: int):
    return load_sparse_csr(os.path.join(data_dir, "test_data")) if is_real else load_data(
        os.path.join(data_dir, "test_data.dat"))


def results_dir(input_dir: str) -> str:
    d = os.path.join(input_dir, "results")
    os.makedirs(d, exist_ok=True)
    return d + "/"


def maybe_int(x) -> Optional[int]:
    try:
        return int(x)
    except (TypeError, ValueError):
        return None
