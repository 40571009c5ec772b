"""Master epilogue: evaluate every stored beta, print, save (ref src/naive.py:153-209).

Reference quirks reproduced unless ``fix_quirks``:
  * the training set is partitions 1..W-1 — partition W is skipped (ref src/naive.py:161,167
    ``range(2, n_procs-1)``), labels are the matching prefix of label.dat (ref :172);
  * linear-regression runs print but do not write result files (ref src/naive.py:413-417);
  * result names follow each scheme's (colliding) prefixes (codes/schemes.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from ..data import io as dio
from ..models.losses import LOGISTIC
from ..ops.eval import auc_columns, loss_sums, predictions_and_loss
from ..utils import report
from .trainer import TrainResult, Trainer


@dataclass
class EvalResult:
    training_loss: np.ndarray
    testing_loss: np.ndarray
    auc: np.ndarray
    n_train: int
    n_test: int
    files: Optional[Dict[str, str]] = None


def eval_partitions(trainer: Trainer):
    W = trainer.cfg.n_workers
    if trainer.cfg.fix_quirks:
        return list(range(trainer.scheme.n_partition_files))
    return list(range(max(1, W - 1)))


def _train_chunks(trainer: Trainer, parts, prec, dev):
    """Training partitions for the evaluation, in order.

    Dense partitions this rank already holds in HBM (all of them on one GPU) are evaluated in
    place instead of being re-read from disk or regenerated.  The reference reloads every file
    (ref src/naive.py:161-172).  Its labels are the prefix of label.dat, which for partitions
    taken in order 0..k is exactly each partition's own labels.
    """
    resident = getattr(trainer, "_parts", None) or {}
    if trainer.source.is_sparse or not all(p in resident for p in parts) or list(parts) != sorted(parts):
        yield from trainer.source.train_eval_chunks(parts, prec, dev)
        return
    for p in parts:
        yield resident[p]


def evaluate(trainer: Trainer, res: TrainResult, log=None, write: bool = True) -> EvalResult:
    log = log or report.log
    cfg = trainer.cfg
    dev = trainer.env.device
    prec = trainer.prec
    d, ld = trainer.d, trainer.ld
    R = res.betaset.shape[0]
    B = torch.zeros((R, ld), dtype=torch.float64, device=dev)
    B[:, :d] = torch.from_numpy(res.betaset).to(dev)
    kind = trainer.loss
    parts = eval_partitions(trainer)
    if cfg.verbose:
        log(report.total_time_line(res.total_time))
        if trainer.scheme.logs_eval_loading and not trainer.source.is_sparse:
            for p in parts:
                log(">> Loaded %d" % (p + 1))
    sums, n_train = loss_sums(_train_chunks(trainer, parts, prec, dev), B, d, kind)
    Xt, yt = trainer.source.test(prec, dev)
    P, tsum = predictions_and_loss(Xt, yt, B, d, kind)
    n_test = Xt.shape[0]
    training_loss = sums / max(1, n_train)
    testing_loss = tsum / max(1, n_test)
    auc = auc_columns(yt, P) if kind == LOGISTIC else np.zeros(R)
    if cfg.verbose:
        for i in range(R):
            if kind == LOGISTIC:
                log(report.logistic_line(i, training_loss[i], testing_loss[i], auc[i], res.timeset[i]))
            else:
                log(report.linear_line(i, training_loss[i], testing_loss[i], res.timeset[i]))
    files = None
    if write and (kind == LOGISTIC or cfg.save_linear):
        names = trainer.scheme.output_names(cfg.fix_quirks)
        data_dir = getattr(trainer.source, "data_dir", None) or cfg.input_dir
        files = report.write_results(dio.results_dir(data_dir), names, training_loss, testing_loss, auc,
                                     res.timeset, res.worker_timeset, cfg.full_precision_outputs)
    if cfg.verbose:
        log(">>> Done")
    return EvalResult(training_loss, testing_loss, auc, n_train, n_test, files)
