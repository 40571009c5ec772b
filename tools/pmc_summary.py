"""Average each PMC counter over the gradient-kernel dispatches of a rocprofv3 --pmc CSV directory."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d):
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        tag = os.path.basename(f).replace("_counter_collection.csv", "")
        vals = defaultdict(list)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "grad_dense" in row.get("Kernel_Name", ""):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, v in vals.items():
            out[f"{k}_{tag}"] = sum(v) / len(v)
            out[f"{k}_{tag}_n"] = len(v)
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
