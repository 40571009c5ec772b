"""Synthetic-data CLI (ref src/generate_data.py:50-71).

    python -m erasurehead_amd.data.generate n_procs n_rows n_cols output_dir n_stragglers n_partitions partial_coded

Writes ``<output_dir>/artificial-data/<n_rows>x<n_cols>/<W>/`` (or ``.../partial/<(P-s)W>/``)
in the reference text layout.  ``--binary`` additionally leaves the ``.npy`` twins the
loaders memory-map (a 1e6 x 1e3 text partition takes minutes to parse).  The on-device
generator (:class:`~erasurehead_amd.data.synthetic.DeviceGMM`, ``--data synthetic`` on the
training CLI) draws the same model without any files.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List, Optional

import numpy as np

from . import io as dio
from .synthetic import generate_to_disk, synthetic_dir

USAGE = "Usage: python generate_data.py n_procs n_rows n_cols output_dir n_stragglers n_partitions partial_coded"


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser(prog="generate_data.py")
    ap.add_argument("positional", nargs="*")
    ap.add_argument("--seed", type=int, default=None, help="seed the generator (reference: unseeded)")
    ap.add_argument("--binary", action="store_true", help="also write .npy twins of every .dat matrix")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    if len(a.positional) != 7:
        print(USAGE)
        return 0
    n_procs, n_rows, n_cols, out, s, P, partial = a.positional
    n_procs, n_rows, n_cols, s, P, partial = int(n_procs), int(n_rows), int(n_cols), int(s), int(P), int(partial)
    out_dir, parts = synthetic_dir(out, n_procs, n_rows, n_cols, s, P, partial)
    rng = np.random.RandomState(a.seed) if a.seed is not None else None
    generate_to_disk(n_rows, n_cols, parts, out_dir, rng=rng, verbose=not a.quiet)
    if a.binary:
        for name in [f"{i}.dat" for i in range(1, parts + 1)] + ["test_data.dat", "label.dat", "label_test.dat"]:
            dio.load_data(os.path.join(out_dir, name), cache=True)
    print("Data Generation Finished.")
    return 0


if __name__ == "__main__":
    sys.exit(main())
