"""Average each PMC counter over the dispatches of a rocprofv3 --pmc CSV directory.

    python tools/pmc_summary.py DIR                  # gradient-kernel dispatches, keyed counter_tag
    python tools/pmc_summary.py DIR --by-kernel      # every kernel, keyed by name, one entry per counter

``--by-kernel`` also derives, for every kernel with the memory-side read requests, the bytes they
stand for at 64 B and at 128 B per request (the two readings of FETCH_SIZE on gfx950,
/opt/skills/guides/MI355X_MICROARCH.md "HBM"), for comparison with the byte counts that
tools/pmc_calibrate.py's workloads fix by shape.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d):
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        tag = os.path.basename(f).replace("_counter_collection.csv", "")
        with open(f) as fh:
            for row in csv.DictReader(fh):
                yield tag, row


def gradient_summary(d):
    out = {}
    vals = defaultdict(list)
    for tag, row in _rows(d):
        if "grad_dense" in row.get("Kernel_Name", ""):
            vals[(row["Counter_Name"], tag)].append(float(row["Counter_Value"]))
    for (k, tag), v in sorted(vals.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        out[f"{k}_{tag}"] = sum(v) / len(v)
        out[f"{k}_{tag}_n"] = len(v)
    return out


def kernel_summary(d):
    vals = defaultdict(lambda: defaultdict(list))
    for _, row in _rows(d):
        name = row.get("Kernel_Name", "")
        name = name.replace("(anonymous namespace)::", "")  # (its parenthesis would cut the name short)
        name = name.split("(")[0] if name.startswith("void ") else name
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for name, cs in vals.items():
        e = {c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()}
        rd = cs.get("TCC_EA0_RDREQ_sum") or cs.get("TCC_EA0_RDREQ")
        if rd:
            m = sum(rd) / len(rd)
            e["read_bytes_at_64B"] = m * 64
            e["read_bytes_at_128B"] = m * 128
        if "FETCH_SIZE" in cs:
            e["fetch_bytes"] = e["FETCH_SIZE"]["mean"] * 1024
        if "WRITE_SIZE" in cs:
            e["write_bytes"] = e["WRITE_SIZE"]["mean"] * 1024
        out[name] = e
    return out


def main(argv):
    d = argv[0]
    json.dump(kernel_summary(d) if "--by-kernel" in argv else gradient_summary(d), sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
