"""Console log lines and result files in the reference's exact formats.

  ---- Starting <Scheme> Iterations ... ----
  \t >>> At Iteration <i>                       (every 10 rounds)
  Total Time Elapsed: %.3f
  Iteration %d: Train Loss = %5.3f, Test Loss = %5.3f, AUC = %5.3f, Total time taken =%5.3f   (logistic)
  Iteration %d: Train Loss = %.6f, Test Loss = %.6f, Total time taken =%5.3f                  (least squares)
  >>> Done
ref src/naive.py:86,93,156,198,209 and :407; files via ref src/util.py:26-36.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, Optional

import numpy as np

from ..data import io as dio


def log(msg: str, stream=None) -> None:
    print(msg, file=stream or sys.stdout, flush=True)


def iteration_tick(i: int) -> Optional[str]:
    return "\t >>> At Iteration %d" % i if i % 10 == 0 else None


def total_time_line(t: float) -> str:
    return "Total Time Elapsed: %.3f" % t


def logistic_line(i: int, train: float, test: float, auc: float, t: float) -> str:
    return "Iteration %d: Train Loss = %5.3f, Test Loss = %5.3f, AUC = %5.3f, Total time taken =%5.3f" % (
        i, train, test, auc, t)


def linear_line(i: int, train: float, test: float, t: float) -> str:
    return "Iteration %d: Train Loss = %.6f, Test Loss = %.6f, Total time taken =%5.3f" % (i, train, test, t)


def write_results(out_dir: str, names: Dict[str, str], training_loss, testing_loss, auc, timeset,
                  worker_timeset, full_precision: bool = False) -> Dict[str, str]:
    os.makedirs(out_dir, exist_ok=True)
    paths = {k: os.path.join(out_dir, v) for k, v in names.items()}
    dio.save_vector(training_loss, paths["training_loss"])
    dio.save_vector(testing_loss, paths["testing_loss"])
    dio.save_vector(auc, paths["auc"])
    dio.save_vector(timeset, paths["timeset"])
    dio.save_matrix(np.asarray(worker_timeset), paths["worker_timeset"])
    if full_precision:
        dio.save_vector_full(timeset, paths["timeset"] + ".full")
        np.savetxt(paths["worker_timeset"] + ".full", np.asarray(worker_timeset), fmt="%.9g")
    return paths
