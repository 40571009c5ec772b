"""Real-dataset preparation (L2): raw table -> one-hot CSR partitions in the reference layout.

Reference: ``src/arrange_real_data.py`` (CLI ``n_procs input_dir real_dataset n_stragglers
n_partitions partial_coded``, ref :23-25).  Four datasets, one shared pipeline:

  ============== ======================================================== ======================
  dataset        feature construction                                     ref lines
  ============== ======================================================== ======================
  amazon-dataset label-encode every column of train.csv[RESOURCE:], add     :34-91
                 hashed degree-2 interaction columns (skipping the (5,7)
                 and (2,3) pairs, ref util.py:49-55), label-encode again,
                 bias column 1; y = 2*ACTION - 1
  dna-dataset/dna first 500k rows of features.csv (col 0 = label), bias    :93-143
                 column 1/sqrt(n); no label encoding
  covtype        classes {1,2} of the UCI covertype table (1 -> -1,        :145-205
                 2 -> +1), label-encode, bias column 1
  kc_house_data  kc_house_data.csv columns bedrooms: as features, y =      :207-253
                 price / 1e6, bias column 1 (least-squares dataset)
  ============== ======================================================== ======================

then: ``train_test_split(test_size=0.2, random_state=0)``; a one-hot encoder fit on
train+test (categories = sorted distinct values per column); the training rows are cut
into ``partitions`` blocks of ``n_rows // partitions`` rows (the remainder is dropped,
ref :79), written as ``{1..P}.npz`` CSR + ``label.dat`` / ``label_test.dat`` (``%5.3f``)
+ ``test_data.npz``.

The one-hot encoding is computed directly (``np.unique`` inverse codes + per-column
offsets -> a CSR matrix with exactly one 1.0 per original column per row), which is
identical to scikit-learn's ``OneHotEncoder(categories='auto')`` output (tested) and
produces the constant-nnz, value-free layout the sparse HIP kernel exploits.

No network: covtype is read from a local ``covtype.data[.gz]`` under the dataset directory
(or scikit-learn's offline cache); :func:`make_raw_dataset` writes synthetic raw tables
with each dataset's exact schema for tests and benchmarks.
"""
from __future__ import annotations

import argparse
import gzip
import itertools
import math
import os
import sys
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import io as dio

DATASETS = ("amazon-dataset", "dna-dataset/dna", "covtype", "kc_house_data")

AMAZON_COLUMNS = ["ACTION", "RESOURCE", "MGR_ID", "ROLE_ROLLUP_1", "ROLE_ROLLUP_2", "ROLE_DEPTNAME", "ROLE_TITLE",
                  "ROLE_FAMILY_DESC", "ROLE_FAMILY", "ROLE_CODE"]
KC_HOUSE_COLUMNS = ["id", "date", "price", "bedrooms", "bathrooms", "sqft_living", "sqft_lot", "floors", "waterfront",
                    "view", "condition", "grade", "sqft_above", "sqft_basement", "yr_built", "yr_renovated", "zipcode",
                    "lat", "long", "sqft_living15", "sqft_lot15"]
DNA_MAX_ROWS = 500000  # ref :96 (itertools.islice(fin, 0, 500000))


# ----------------------------------------------------------------------------- encoders
def label_encode_columns(X: np.ndarray) -> np.ndarray:
    """Per-column LabelEncoder (ref :42-44): value -> rank among the column's distinct values."""
    X = np.asarray(X)
    out = np.empty(X.shape, dtype=np.int64)
    for c in range(X.shape[1]):
        _, inv = np.unique(X[:, c], return_inverse=True)
        out[:, c] = inv.reshape(-1)
    return out


def interaction_terms(X: np.ndarray, degree: int = 2, skip: Sequence[Tuple[int, int]] = ((5, 7), (2, 3))) -> np.ndarray:
    """Hashed interaction columns of ref util.py:49-55 (interactionTermsAmazon).

    Every ``degree``-combination of columns except those containing a skipped pair becomes
    one new column whose value identifies the row's tuple of values.  The reference uses
    Python's ``hash(tuple)`` only as an identifier that the next label-encoding pass turns
    into ranks; a collision-free tuple id gives the same partition of rows into categories
    (deterministic across processes, unlike string hashing).
    """
    X = np.asarray(X)
    cols = []
    for idx in itertools.combinations(range(X.shape[1]), degree):
        if any(a in idx and b in idx for a, b in skip):
            continue
        sub = np.ascontiguousarray(X[:, idx])
        _, inv = np.unique(sub, axis=0, return_inverse=True)
        cols.append(inv.reshape(-1))
    if not cols:
        return np.zeros((X.shape[0], 0), dtype=np.int64)
    return np.stack(cols, axis=1).astype(np.int64)


def add_bias(X: np.ndarray, value: float) -> np.ndarray:
    """Append a constant column (ref :54 ``np.vstack([X.T, ones]).T``; dna uses 1/sqrt(n))."""
    X = np.asarray(X, dtype=np.float64)
    return np.hstack([X, np.full((X.shape[0], 1), float(value))])


@dataclass
class OneHot:
    """Fitted one-hot encoder: sorted categories per column (== sklearn categories='auto')."""

    categories: List[np.ndarray]

    @classmethod
    def fit(cls, X: np.ndarray) -> "OneHot":
        X = np.asarray(X)
        return cls([np.unique(X[:, c]) for c in range(X.shape[1])])

    @property
    def offsets(self) -> np.ndarray:
        return np.concatenate([[0], np.cumsum([len(c) for c in self.categories])]).astype(np.int64)

    @property
    def n_features(self) -> int:
        return int(self.offsets[-1])

    def transform(self, X: np.ndarray):
        from scipy.sparse import csr_matrix

        X = np.asarray(X)
        n, m = X.shape
        off = self.offsets
        idx = np.empty((n, m), dtype=np.int64)
        for c, cats in enumerate(self.categories):
            pos = np.searchsorted(cats, X[:, c])
            if np.any(pos >= len(cats)) or np.any(cats[np.minimum(pos, len(cats) - 1)] != X[:, c]):
                raise ValueError(f"column {c}: value not seen during fit")
            idx[:, c] = off[c] + pos
        indices = idx.reshape(-1).astype(np.int32)
        indptr = np.arange(0, n * m + 1, m, dtype=np.int32 if n * m < 2 ** 31 else np.int64)
        data = np.ones(n * m, dtype=np.float64)
        return csr_matrix((data, indices, indptr), shape=(n, self.n_features))


def train_test_split_rs0(X, y, test_size: float = 0.2):
    """scikit-learn ``train_test_split(test_size=0.2, random_state=0)`` (ref :56)."""
    try:
        from sklearn.model_selection import train_test_split

        return train_test_split(X, y, test_size=test_size, random_state=0)
    except ImportError:  # same ShuffleSplit arithmetic
        n = len(y)
        n_test = int(math.ceil(test_size * n))
        perm = np.random.RandomState(0).permutation(n)
        te, tr = perm[:n_test], perm[n_test:]
        return X[tr], X[te], y[tr], y[te]


# ---------------------------------------------------------------------------- raw loaders
def _read_csv(path: str):
    import pandas as pd

    return pd.read_csv(path)


def load_amazon(ddir: str) -> Tuple[np.ndarray, np.ndarray, float]:
    df = _read_csv(os.path.join(ddir, "train.csv"))
    X = df.loc[:, "RESOURCE":].values
    y = 2 * df["ACTION"].values.astype(np.float64) - 1
    X = label_encode_columns(X)
    X = np.hstack([X, interaction_terms(X, 2)])
    X = label_encode_columns(X)
    return X, y, 1.0


def load_dna(ddir: str, max_rows: int = DNA_MAX_ROWS) -> Tuple[np.ndarray, np.ndarray, float]:
    with open(os.path.join(ddir, "features.csv")) as f:
        data = np.genfromtxt(itertools.islice(f, 0, max_rows, 1), delimiter=",")
    data = np.atleast_2d(data)
    X, y = data[:, 1:], data[:, 0]
    return X, y, 1.0 / math.sqrt(X.shape[0])


def load_covtype(ddir: str) -> Tuple[np.ndarray, np.ndarray, float]:
    raw = None
    for name in ("covtype.data.gz", "covtype.data", "covtype.csv"):
        p = os.path.join(ddir, name)
        if os.path.exists(p):
            opener = gzip.open if p.endswith(".gz") else open
            with opener(p, "rt") as f:
                raw = np.loadtxt(f, delimiter=",")
            break
    if raw is None:
        from sklearn.datasets import fetch_covtype

        b = fetch_covtype(download_if_missing=False)  # offline cache only
        raw = np.hstack([b.data, b.target[:, None]])
    Xall, t = raw[:, :-1], raw[:, -1].astype(np.int64)
    keep = np.where(t <= 2)[0]
    X = Xall[keep]
    y = np.where(t[keep] == 1, -1.0, 1.0)
    X = label_encode_columns(label_encode_columns(X))
    return X, y, 1.0


def load_kc_house(ddir: str) -> Tuple[np.ndarray, np.ndarray, float]:
    df = _read_csv(os.path.join(ddir, "kc_house_data.csv"))
    X = df.loc[:, "bedrooms":].values.astype(np.float64)
    y = df["price"].values.astype(np.float64)
    return X, y, 1.0


_LOADERS = {"amazon-dataset": load_amazon, "dna-dataset/dna": load_dna, "covtype": load_covtype,
            "kc_house_data": load_kc_house}


# --------------------------------------------------------------------------- pipeline
def output_layout(dataset_dir: str, n_procs: int, n_stragglers: int, n_partitions: int, partial_coded: int):
    """(output dir, number of partition files) — ref :67-75."""
    dataset_dir = dataset_dir if dataset_dir.endswith("/") else dataset_dir + "/"
    if not partial_coded:
        return dataset_dir + str(n_procs - 1) + "/", n_procs - 1
    parts = (n_procs - 1) * (n_partitions - n_stragglers)
    return dataset_dir + "partial/" + str(parts) + "/", parts


@dataclass
class Prepared:
    out_dir: str
    partitions: int
    n_train: int
    n_test: int
    n_cols: int
    rows_per_partition: int


def prepare_arrays(X: np.ndarray, y: np.ndarray, bias: float, out_dir: str, partitions: int,
                   scale_y: float = 1.0, verbose: bool = True, log=print) -> Prepared:
    """bias column -> 80/20 split -> one-hot -> partition files (the shared tail of every dataset)."""
    X = add_bias(X, bias)
    X_train, X_valid, y_train, y_valid = train_test_split_rs0(X, np.asarray(y, dtype=np.float64))
    enc = OneHot.fit(np.vstack((X_train, X_valid)))
    Xtr = enc.transform(X_train)
    Xte = enc.transform(X_valid)
    y_train = y_train / scale_y
    y_valid = y_valid / scale_y
    n_rows, n_cols = Xtr.shape
    if verbose:
        log("No. of training samples = %d, Dimension = %d" % (n_rows, n_cols))
        log("No. of testing samples = %d, Dimension = %d" % (Xte.shape[0], Xte.shape[1]))
    os.makedirs(out_dir, exist_ok=True)
    rpw = n_rows // partitions
    for i in range(1, partitions + 1):
        dio.save_sparse_csr(os.path.join(out_dir, str(i)), Xtr[(i - 1) * rpw:i * rpw, :])
        if verbose:
            log("\t >>> Done with partition %d" % i)
    dio.save_vector(y_train, os.path.join(out_dir, "label.dat"))
    dio.save_vector(y_valid, os.path.join(out_dir, "label_test.dat"))
    dio.save_sparse_csr(os.path.join(out_dir, "test_data"), Xte)
    return Prepared(out_dir, partitions, n_rows, Xte.shape[0], n_cols, rpw)


def prepare_dataset(n_procs: int, input_dir: str, dataset: str, n_stragglers: int, n_partitions: int,
                    partial_coded: int, verbose: bool = True, log=print) -> Prepared:
    """Full ref arrange_real_data.py run for one dataset."""
    if dataset not in _LOADERS:
        raise ValueError(f"unknown dataset {dataset!r}; expected one of {DATASETS}")
    input_dir = input_dir if input_dir.endswith("/") else input_dir + "/"
    ddir = input_dir + dataset + "/"
    if verbose:
        log("Preparing data for " + dataset)
    X, y, bias = _LOADERS[dataset](ddir)
    out_dir, parts = output_layout(ddir, n_procs, n_stragglers, n_partitions, partial_coded)
    scale = 1e6 if dataset == "kc_house_data" else 1.0
    return prepare_arrays(X, y, bias, out_dir, parts, scale_y=scale, verbose=verbose, log=log)


# ------------------------------------------------------------------ synthetic raw tables
def make_raw_dataset(dataset: str, input_dir: str, n_rows: int, seed: int = 0,
                     cardinality: Optional[Sequence[int]] = None) -> str:
    """Write a synthetic raw table with ``dataset``'s exact schema (no network for the real one).

    amazon: 9 categorical id columns + ACTION; covtype: 54 integer columns + class 1..7
    (classes 3..7 present so the <=2 filter is exercised); kc_house: the 21 Kaggle columns;
    dna: label in {-1, 1} + 200 integer features.  Returns the dataset directory.
    """
    rng = np.random.RandomState(seed)
    input_dir = input_dir if input_dir.endswith("/") else input_dir + "/"
    ddir = input_dir + dataset + "/"
    os.makedirs(ddir, exist_ok=True)
    import pandas as pd

    if dataset == "amazon-dataset":
        card = list(cardinality or [700, 400, 12, 18, 45, 60, 50, 25, 60])
        cols = {"ACTION": rng.binomial(1, 0.9, n_rows)}
        for name, c in zip(AMAZON_COLUMNS[1:], card):
            cols[name] = rng.randint(0, c, n_rows) * 7 + 1000
        pd.DataFrame(cols, columns=AMAZON_COLUMNS).to_csv(ddir + "train.csv", index=False)
    elif dataset == "covtype":
        card = list(cardinality or ([400, 40, 30, 300, 200, 500, 60, 60, 60, 500] + [2] * 44))
        X = np.stack([rng.randint(0, c, n_rows) for c in card], axis=1)
        t = rng.choice(np.arange(1, 8), n_rows, p=[0.36, 0.49, 0.06, 0.005, 0.016, 0.03, 0.039])
        np.savetxt(ddir + "covtype.data", np.hstack([X, t[:, None]]), fmt="%d", delimiter=",")
    elif dataset == "kc_house_data":
        card = list(cardinality or [10, 20, 300, 400, 6, 2, 5, 5, 10, 250, 100, 110, 50, 70, 300, 300, 200, 300])
        feats = {}
        for name, c in zip(KC_HOUSE_COLUMNS[3:], card):
            feats[name] = rng.randint(0, c, n_rows).astype(np.float64)
        price = 2e5 + 3e4 * feats["bedrooms"] + 1e3 * feats["sqft_living"] + rng.normal(0, 5e4, n_rows)
        df = pd.DataFrame({"id": np.arange(n_rows), "date": ["20141013T000000"] * n_rows,
                           "price": np.round(np.abs(price)), **feats}, columns=KC_HOUSE_COLUMNS)
        df.to_csv(ddir + "kc_house_data.csv", index=False)
    elif dataset == "dna-dataset/dna":
        card = list(cardinality or [4] * 200)
        X = np.stack([rng.randint(0, c, n_rows) for c in card], axis=1)
        y = np.where(rng.rand(n_rows) < 0.05, 1, -1)
        np.savetxt(ddir + "features.csv", np.hstack([y[:, None], X]), fmt="%d", delimiter=",")
    else:
        raise ValueError(f"unknown dataset {dataset!r}")
    return ddir


# ---------------------------------------------------------------------------------- CLI
USAGE = "Usage: python arrange_real_data.py n_procs input_dir real_dataset n_stragglers n_partitions partial_coded"


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser(prog="arrange_real_data.py", add_help=True)
    ap.add_argument("positional", nargs="*")
    ap.add_argument("--make-raw", type=int, default=0,
                    help="first write a synthetic raw table of this many rows with the dataset's schema")
    ap.add_argument("--raw-seed", type=int, default=0)
    a = ap.parse_args(argv)
    if len(a.positional) != 6:
        print(USAGE)
        return 0
    n_procs, input_dir, dataset, s, P, partial = a.positional
    np.random.seed(0)  # ref :27
    input_dir = input_dir if input_dir.endswith("/") else input_dir + "/"
    if a.make_raw:
        make_raw_dataset(dataset, input_dir, a.make_raw, a.raw_seed)
    prepare_dataset(int(n_procs), input_dir, dataset, int(s), int(P), int(partial))
    print("Data Setup Finished.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
