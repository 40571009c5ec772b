"""Idle gaps between consecutive kernels of a rocprofv3 --kernel-trace CSV (one queue's timeline).

    python tools/kernel_gaps.py <dir with *kernel_trace.csv> [--match eh::] [--last N]

For every pair of consecutive dispatches whose names contain --match, the gap = start(next) -
end(previous), grouped by (previous kernel, next kernel): where a round loses time between its
kernels (launch latency, host work between enqueues, stream waits).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

import numpy as np


def short(name: str) -> str:
    name = name.split("(")[0]
    name = re.sub(r"^void ", "", name)
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="eh::")
    ap.add_argument("--last", type=int, default=0, help="only the last N matching dispatches (the timed steps)")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if a.match in r.get("Kernel_Name", ""):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    if a.last:
        rows = rows[-a.last:]
    gaps = defaultdict(list)
    dur = defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        gaps[(n0, n1)].append((s1 - e0) / 1e3)
    for s, e, n in rows:
        dur[n].append((e - s) / 1e3)
    out = {"dispatches": len(rows),
           "kernels_us": {n: {"n": len(v), "median": float(np.median(v))} for n, v in dur.items()},
           "gaps_us": [{"from": k[0], "to": k[1], "n": len(v), "median": float(np.median(v)),
                        "p10": float(np.percentile(v, 10)), "p90": float(np.percentile(v, 90))}
                       for k, v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
