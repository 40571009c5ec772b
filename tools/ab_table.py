"""Table of an ab.py jsonl: per label, medians of ms/step and of the per-round phase ticks."""
import json
import statistics
import sys
from collections import defaultdict


def main(path):
    rows = defaultdict(lambda: defaultdict(list))
    for line in open(path):
        r = json.loads(line)
        b = r.get("bench")
        if not b:
            continue
        d = rows[r["label"]]
        d["ms"].append(b["ms_per_step"])
        for k, v in (b.get("phases_us") or {}).items():
            d[k].append(v)
        r0 = (b.get("ranks") or [{}])[0]
        for k in ("arbiter_poll_us", "arbiter_update_us", "release_us", "decode_update_us", "put_beta_us"):
            if k in r0:
                d["r0." + k].append(r0[k])
    for label, d in rows.items():
        print(label.ljust(22), "  ".join(f"{k}={statistics.median(v):.4g}" for k, v in d.items()))


if __name__ == "__main__":
    main(sys.argv[1])
