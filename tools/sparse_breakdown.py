"""Per-kernel breakdown of a `gpu_round.sh sparse` / `pmcsparse` output directory.

    python tools/sparse_breakdown.py gpurun_out/<run>

Prints the sparse gradient times (sparse.jsonl), the median duration of every kernel of the
covtype-shaped ELL rounds from the rocprofv3 kernel trace (prof_sparse/), and the per-kernel
medians of the counter passes (pmcs/) with VALU / SALU instructions per wave.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

import numpy as np

KERNELS = r"(ell_rows_lds|ell_rows|csr_rows|csc_tiles_lds|csc_tiles|csc_spans|sub_reduce|encode_messages)<"


def main(d):
    if os.path.exists(f"{d}/sparse.jsonl"):
        for line in open(f"{d}/sparse.jsonl"):
            r = json.loads(line)
            print(r["dataset_shape"], r["layout"], r["kernel"], f"{r['ms'] * 1e3:.1f} us")
    trace = f"{d}/prof_sparse/run_kernel_trace.csv"
    if os.path.exists(trace):
        rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
        idx = [i for i, r in enumerate(rows) if "ell_rows_lds" in r["Kernel_Name"]]
        runs, cur = [], idx[:1]
        for a, b in zip(idx, idx[1:]):
            if b - a > 10:
                runs.append(cur)
                cur = [b]
            else:
                cur.append(b)
        if cur:
            runs.append(cur)
        for k, run in enumerate(runs):  # covtype naive, then covtype s = 1 replicas
            per = collections.defaultdict(list)
            for r in rows[run[0]:run[-1] + 4]:
                m = re.search(KERNELS, r["Kernel_Name"])
                if m:
                    per[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            print(f"covtype ELL rounds #{k}:", {n: f"{np.median(v):.1f} us x{len(v)}" for n, v in per.items()})
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/pmcs/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(KERNELS, r["Kernel_Name"])
            if m:
                acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in acc.items():
        med = {c: float(np.median(v)) for c, v in cs.items()}
        waves = med.get("SQ_WAVES", 0.0) or 1.0
        print(n, {c: f"{v:.3g}" for c, v in sorted(med.items())},
              f"VALU/wave {med.get('SQ_INSTS_VALU', 0) / waves:.0f}, SALU/wave {med.get('SQ_INSTS_SALU', 0) / waves:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
