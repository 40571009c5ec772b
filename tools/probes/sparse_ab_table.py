"""Table of tools/probes/sparse_ab_tree.sh output: per shape / layout / row kernel, the old tree's (build/ab_old) and
this tree's times (us, one per rep)."""
import json
import sys

d = sys.argv[1]
rows = {}
for v in ("old", "new"):
    for r in (1, 2):
        try:
            f = open(f"{d}/{v}_{r}.jsonl")
        except OSError:
            continue
        for line in f:
            x = json.loads(line)
            k = (x["dataset_shape"], x["layout"], x["kernel"].split("(")[1].split(",")[0], x.get("units"))
            rows.setdefault(k, {}).setdefault(v, []).append(round(x["ms"] * 1e3, 1))
print("| shape | layout | rows | units | old tree (build/ab_old) us | this tree us |")
print("|---|---|---|---|---|---|")
for k, v in rows.items():
    print(f"| {k[0]} | {k[1]} | {k[2]} | {k[3]} | {v.get('old', '-')} | {v.get('new', '-')} |")
