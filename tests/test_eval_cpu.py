"""Evaluation epilogue ops (K10/K11) on CPU tensors against scikit-learn."""
import numpy as np
import pytest
import torch

from erasurehead_amd.models.losses import LEAST_SQUARES, LOGISTIC
from erasurehead_amd.ops.eval import _loss_torch, auc_columns


@pytest.mark.parametrize("chunk", [0, 1, 3])
def test_auc_columns_matches_sklearn_with_ties(chunk):
    metrics = pytest.importorskip("sklearn.metrics")
    rng = np.random.RandomState(1)
    y = rng.choice([-1.0, 1.0], 400)
    P = np.round(rng.randn(400, 6), 1)  # many ties
    P[:, 5] = 0.0  # a constant column: AUC 0.5
    got = auc_columns(torch.tensor(y), torch.tensor(P), chunk=chunk)
    ref = [metrics.auc(*metrics.roc_curve(y, P[:, j], pos_label=1)[:2]) for j in range(6)]
    np.testing.assert_allclose(got, ref, atol=1e-12)


def test_auc_single_class_is_nan():
    assert np.all(np.isnan(auc_columns(torch.ones(10), torch.randn(10, 2))))


def test_loss_sums():
    rng = np.random.RandomState(2)
    y = rng.choice([-1.0, 1.0], 50)
    P = rng.randn(50, 3) * 30  # large margins: stable softplus
    got = _loss_torch(LOGISTIC, torch.tensor(y), torch.tensor(P)).numpy()
    ref = np.logaddexp(0, -y[:, None] * P).sum(0)
    np.testing.assert_allclose(got, ref, rtol=1e-12)
    got = _loss_torch(LEAST_SQUARES, torch.tensor(y), torch.tensor(P)).numpy()
    np.testing.assert_allclose(got, ((y[:, None] - P) ** 2).sum(0), rtol=1e-12)
