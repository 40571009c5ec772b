"""Data pipeline (L2): real-dataset preparation, synthetic generator CLI, reference on-disk layout.

Parity notes: the raw Kaggle/UCI tables are not available offline, so every dataset is
exercised on a synthetic raw table with the exact schema (data/prepare.py
make_raw_dataset).  The one-hot encoder is pinned against scikit-learn's
OneHotEncoder(categories='auto'); the amazon hashed-interaction column ordering
depends on Python 2's tuple hash in the reference and is "parity unpinned" (only the
induced partition of rows into categories is tested).
"""
import os

import numpy as np
import pytest

from erasurehead_amd.data import io as dio
from erasurehead_amd.data.prepare import (DATASETS, OneHot, interaction_terms, label_encode_columns, main as prep_main,
                                          make_raw_dataset, output_layout, prepare_dataset)


def test_onehot_matches_sklearn():
    sk = pytest.importorskip("sklearn.preprocessing")
    rng = np.random.RandomState(0)
    X = np.hstack([rng.randint(0, 5, (200, 3)), rng.rand(200, 1).round(1), np.ones((200, 1))])
    enc = OneHot.fit(X)
    ours = enc.transform(X)
    try:
        ref = sk.OneHotEncoder(categories="auto", sparse_output=True).fit(X).transform(X)
    except TypeError:
        ref = sk.OneHotEncoder(categories="auto", sparse=True).fit(X).transform(X)
    assert ours.shape == ref.shape
    assert (ours != ref).nnz == 0
    assert np.all(np.diff(ours.indptr) == X.shape[1])  # constant nnz per row (ELL-exact)


def test_label_encode_and_interactions():
    X = np.array([[10, 7, 3], [5, 7, 3], [10, 1, 4], [5, 1, 3]])
    E = label_encode_columns(X)
    np.testing.assert_array_equal(E, [[1, 1, 0], [0, 1, 0], [1, 0, 1], [0, 0, 0]])
    I = interaction_terms(E, 2, skip=())
    assert I.shape == (4, 3)
    # rows share an interaction category iff they share the pair of values
    for c, (a, b) in enumerate([(0, 1), (0, 2), (1, 2)]):
        for r1 in range(4):
            for r2 in range(4):
                assert (I[r1, c] == I[r2, c]) == (tuple(E[r1, [a, b]]) == tuple(E[r2, [a, b]]))
    # the reference skips pairs containing both 5 and 7, and both 2 and 3 (ref util.py:53)
    wide = np.zeros((3, 9), dtype=np.int64)
    assert interaction_terms(wide, 2).shape[1] == 36 - 2


@pytest.mark.parametrize("dataset", DATASETS)
def test_prepare_layout(dataset, tmp_path):
    root = str(tmp_path) + "/"
    make_raw_dataset(dataset, root, 600, seed=1)
    prep = prepare_dataset(5, root, dataset, 1, 0, 0, verbose=False)
    out, parts = output_layout(root + dataset + "/", 5, 1, 0, 0)
    assert prep.out_dir == out and parts == 4
    n_train = prep.n_train
    assert prep.n_test == int(np.ceil(0.2 * (n_train + prep.n_test)))
    for i in range(1, parts + 1):
        A = dio.load_sparse_csr(os.path.join(out, str(i)))
        assert A.shape == (n_train // parts, prep.n_cols)
        assert np.all(A.data == 1.0)
        nnz = np.diff(A.indptr)
        assert np.all(nnz == nnz[0])
    y = dio.load_labels(out)
    assert len(y) == n_train
    if dataset == "kc_house_data":
        assert np.all(y > 0) and np.max(y) < 10  # price / 1e6
    else:
        assert set(np.unique(y)) <= {-1.0, 1.0}
    T = dio.load_sparse_csr(os.path.join(out, "test_data"))
    assert T.shape[1] == prep.n_cols


def test_covtype_class_filter(tmp_path):
    root = str(tmp_path) + "/"
    ddir = make_raw_dataset("covtype", root, 1000, seed=3)
    raw = np.loadtxt(ddir + "covtype.data", delimiter=",")
    keep = int(np.sum(raw[:, -1] <= 2))
    prep = prepare_dataset(3, root, "covtype", 0, 0, 0, verbose=False)
    assert prep.n_train + prep.n_test == keep


def test_partial_layout(tmp_path):
    root = str(tmp_path) + "/"
    make_raw_dataset("covtype", root, 800, seed=2)
    prep = prepare_dataset(5, root, "covtype", 1, 3, 1, verbose=False)
    assert prep.out_dir.endswith("covtype/partial/8/") and prep.partitions == 8


def test_prepare_cli_and_train(tmp_path, capsys):
    """arrange_real_data CLI -> main.py CLI (is_real=1, sparse path) end to end on CPU."""
    from erasurehead_amd.cli import main as cli_main

    root = str(tmp_path) + "/"
    assert prep_main(["7", root, "covtype", "2", "0", "0", "--make-raw", "900"]) == 0
    out = capsys.readouterr().out
    assert "Data Setup Finished." in out
    line = [l for l in out.splitlines() if l.startswith("No. of training samples")][0]
    n_rows, n_cols = [int(t) for t in line.replace(",", " ").split() if t.isdigit()]
    rc = cli_main(["7", str(n_rows), str(n_cols), root, "1", "covtype", "1", "2", "0", "3", "4", "0", "AGD",
                   "--num-itrs", "5", "--device", "cpu", "--seed", "0"])
    assert rc == 0
    out = capsys.readouterr().out
    assert "Iteration 4: Train Loss" in out
    res = os.path.join(root, "covtype", "6", "results")  # <data dir>/results (ref naive.py:200)
    assert os.path.exists(os.path.join(res, "replication_acc_2_training_loss.dat"))


def test_generate_cli(tmp_path, capsys):
    from erasurehead_amd.data.generate import main as gen_main

    root = str(tmp_path)
    assert gen_main(["4", "60", "5", root, "1", "0", "0", "--seed", "0", "--quiet", "--binary"]) == 0
    d = os.path.join(root, "artificial-data", "60x5", "3")
    for f in ["1.dat", "2.dat", "3.dat", "label.dat", "test_data.dat", "label_test.dat", "1.dat.npy"]:
        assert os.path.exists(os.path.join(d, f)), f
    X = dio.load_data(os.path.join(d, "1.dat"))
    assert X.shape == (20, 5)
    assert gen_main([]) == 0 and "Usage" in capsys.readouterr().out


@pytest.mark.parametrize("coded_ver,prefix", [(1, "partialreplication_1_3_"), (0, "partialcoded_1_3_")])
def test_partial_schemes_on_prepared_real_data(coded_ver, prefix, tmp_path, capsys):
    """arrange_real_data with partial_coded=1 -> main.py partial schemes on the partial/ layout."""
    from erasurehead_amd.cli import main as cli_main

    root = str(tmp_path) + "/"
    # W = 4, s = 1, P = 3  ->  (P - s) * W = 8 partition files under covtype/partial/8/
    assert prep_main(["5", root, "covtype", "1", "3", "1", "--make-raw", "1500"]) == 0
    line = [l for l in capsys.readouterr().out.splitlines() if l.startswith("No. of training samples")][0]
    n_rows, n_cols = [int(t) for t in line.replace(",", " ").split() if t.isdigit()]
    rc = cli_main(["5", str(n_rows), str(n_cols), root, "1", "covtype", "1", "1", "3", str(coded_ver), "0", "0", "AGD",
                   "--num-itrs", "4", "--device", "cpu", "--seed", "0"])
    assert rc == 0
    out = capsys.readouterr().out
    assert "Stragglers are allowed to be atmost 3.00 times slower" in out
    assert "Iteration 3: Train Loss" in out
    res = os.path.join(root, "covtype", "partial", "8", "results")
    assert os.path.exists(os.path.join(res, prefix + "auc.dat"))
