"""Reference-equivalent CPU timing of one AGC iteration (the baseline the reference never published).

BASELINE.md has no per-iteration number: the reference only ships a straggler CDF.  To give
the MI355X numbers something honest to be compared with, this tool times the *reference's
own per-iteration math* with NumPy/BLAS on the host CPU, restricted to the thread count of
the reference's worker instance (m4.2xlarge = 8 vCPU, ref README.md:43-44):

  worker (every logical worker runs on its own machine in the reference):
      predy = X_current.dot(beta)                                  ref src/approximate_coding.py:194
      g = -X_current.T.dot(y / (exp(predy * y) + 1))               ref src/approximate_coding.py:195-196
  master:
      g = sum of the first-arriving messages of each FRC group     ref src/approximate_coding.py:150-160
      AGD update                                                   ref src/approximate_coding.py:162-170

X_current holds the worker's (s+1) partitions: (s+1) * n / W rows of d fp64 columns.  Workers run
in parallel on separate machines, so the critical path of one iteration is one worker's
gradient + the master's combine/update; MPI latency and the injected delay are NOT included,
which makes this a LOWER bound on the reference's sec/iter (add_delay = 0).

Usage: python tools/reference_cpu_equiv.py [--n-rows 1000000] [--n-cols 1000] [--workers 8]
       [--stragglers 2] [--threads 8] [--iters 5] [--json-out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-rows", type=int, default=1_000_000)
    ap.add_argument("--n-cols", type=int, default=1000)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--stragglers", type=int, default=2)
    ap.add_argument("--num-collect", type=int, default=6)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    # BLAS thread pools read these at import time
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[k] = str(a.threads)
    import numpy as np

    rows = (a.stragglers + 1) * (a.n_rows // a.workers)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((rows, a.n_cols))
    y = np.where(rng.random(rows) < 0.5, -1.0, 1.0)
    beta = rng.standard_normal(a.n_cols) * 0.01
    utemp = np.zeros(a.n_cols)
    msgs = rng.standard_normal((a.workers, a.n_cols))
    alpha, eta, n = 1.0 / a.n_rows, 10.0, a.n_rows

    wt, mt = [], []
    for i in range(a.iters + 1):
        t0 = time.perf_counter()
        predy = X.dot(beta)
        g = X.T.dot(np.divide(y, np.exp(np.multiply(predy, y)) + 1))
        g *= -1
        t1 = time.perf_counter()
        # master: combine first arrivals of each group (k of W messages), AGD update
        gm = np.zeros(a.n_cols)
        for w in range(a.num_collect):
            gm += msgs[w]
        theta = 2.0 / (i + 2.0)
        ytemp = (1 - theta) * beta + theta * utemp
        betatemp = ytemp - (eta / n) * gm - (2 * alpha * eta) * beta
        utemp = beta + (betatemp - beta) * (1 / theta)
        beta = beta + 0.0 * (betatemp - beta)  # keep beta fixed: timing only, same flops
        t2 = time.perf_counter()
        if i:  # first iteration pages X in
            wt.append(t1 - t0)
            mt.append(t2 - t1)
    wt.sort()
    mt.sort()
    out = {
        "what": "reference per-iteration math (NumPy/BLAS, fp64) on the host CPU, lower bound of ref sec/iter",
        "cpu_threads": a.threads,
        "cpu_model": _cpu_model(),
        "blas": _blas_name(np),
        "n_rows": a.n_rows, "worker_rows": rows, "n_cols": a.n_cols, "workers": a.workers, "stragglers": a.stragglers,
        "worker_grad_s_median": wt[len(wt) // 2],
        "master_update_s_median": mt[len(mt) // 2],
        "sec_per_iter_lower_bound": wt[len(wt) // 2] + mt[len(mt) // 2],
        "worker_stream_GBps": rows * a.n_cols * 8 * 2 / wt[len(wt) // 2] / 1e9,
    }
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    return 0


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _blas_name(np) -> str:
    try:
        cfg = np.show_config(mode="dicts")
        return cfg["Build Dependencies"]["blas"]["name"]
    except Exception:
        return "unknown"


if __name__ == "__main__":
    sys.exit(main())
