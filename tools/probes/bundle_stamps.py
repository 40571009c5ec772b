"""Timeline of one grad_dense_multi launch at a rank shape of the headline (kernel-side stamps).

    python tools/probes/bundle_stamps.py [--gpus 8] [--rows 0] [--reps 5] [--out FILE]

Every bundle (one wave) writes {start, rows done, slab rows written, XCC id} in wall_clock64 ticks
(csrc/kernels/grad_dense.hip, set_grad_stamps).  Reported relative to the first start: the launch ramp
(start spread), per-wave stream time, the fold + slab tail, the finish spread (tail of the slowest
CUs) and per-XCD means -- what the fixed per-launch cost of a short bundle is made of.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    from bench_rank_shapes import build_plan
    from bench_kernels import clock_warm
    from erasurehead_amd._ext import native

    C = native()
    plan, beta, G = build_plan(a.gpus, "fp64", rows_override=a.rows)
    hz = 100e6  # wall_clock64: 100 MHz
    n = plan.ntasks
    st = torch.zeros(4 * n, dtype=torch.int64, device="cuda")
    clock_warm(lambda: plan.run(beta, G))
    recs = []
    for rep in range(a.reps):
        st.zero_()
        torch.cuda.synchronize()
        C._set_grad_stamps(st.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.run(beta, G)
        e1.record()
        torch.cuda.synchronize()
        C._set_grad_stamps(0)
        v = st.view(-1, 4).cpu().numpy()
        ids = np.nonzero(v[:, 0] > 0)[0]  # bundle ids (the grid's wave index)
        v = v[ids]
        t0 = v[:, 0].min()
        start = (v[:, 0] - t0) / hz * 1e6
        rows_done = (v[:, 1] - t0) / hz * 1e6
        has_done = v[:, 2] > 0  # FOLD: waves 1-3 of a workgroup return after the fold, wave 0 writes the slab
        done = (v[has_done, 2] - t0) / hz * 1e6
        xcc = v[:, 3]
        pct = lambda x, q: float(np.percentile(x, q))  # noqa: E731
        rec = {"gpus": a.gpus, "bundle_rows": plan.bundle_rows, "bundles": int(len(v)), "event_us": 1e3 * e0.elapsed_time(e1),
               "span_us": float(done.max()),
               "start_p50_p100_us": [pct(start, 50), float(start.max())],
               "stream_us_p0_p50_p100": [float((rows_done - start).min()), pct(rows_done - start, 50),
                                          float((rows_done - start).max())],
               "rows_done_p0_p50_p100_us": [float(rows_done.min()), pct(rows_done, 50), float(rows_done.max())],
               "slab_tail_us_p50_p100": [pct(done - rows_done[has_done], 50), float((done - rows_done[has_done]).max())],
               "done_p0_p10_p50_p90_p100_us": [float(done.min()), pct(done, 10), pct(done, 50), pct(done, 90),
                                               float(done.max())],
               "rows_done_p10_p25_p75_p90_p99_us": [pct(rows_done, q) for q in (10, 25, 75, 90, 99)],
               "per_xcc_rows_done_p50_max_us": {int(x): [pct(rows_done[xcc == x], 50), float(rows_done[xcc == x].max())]
                                                for x in sorted(set(xcc.tolist()))},
               "per_xcc_bundles": {int(x): int((xcc == x).sum()) for x in sorted(set(xcc.tolist()))}}
        live = rows_done > 5.0  # pad bundles finish at once
        order = np.argsort(-rows_done)
        rec["slowest_bundles"] = [[int(ids[b]), int(xcc[b]), round(float(rows_done[b]), 2), round(float(start[b]), 2)]
                                  for b in order[:12]]
        rec["live_bundles"] = int(live.sum())
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
