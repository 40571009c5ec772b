"""Per-rank gradient work of the headline at N = 1/2/4/8 GPUs, timed on one MI355X.

    python tools/bench_rank_shapes.py [--shard partition|message] [--rows-sweep [--rows-list 64,128,...]] [--out FILE]

With partition shards (parallel/placement.py) the rank of an N-GPU headline run (AGC W=8, s=2,
k=6, 1e6 x 1e3 fp64) holds 8/N partitions of 125k rows, each with its 2-3 replica messages; with
whole messages (the reference topology) it holds its logical workers' 3 partitions each.  This
builds exactly the heaviest rank's local plan (DenseGradPlan over its units) and times one
gradient launch with HIP events: the compute floor of one round at that N.  --rows-sweep also
times other bundle lengths of the chosen kernel at each shape.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_plan(n_gpus: int, precision: str, shard: str = "partition", rows_override: int = 0, fill: bool = False):
    """(plan, beta, G) of the heaviest rank's local gradient at the N-GPU placement (also
    tools/probes/bundle_stamps.py)."""
    import torch

    from erasurehead_amd.codes import make_scheme
    from erasurehead_amd.data.source import SyntheticSource
    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision
    from dataclasses import replace

    from erasurehead_amd.ops.grad import choose_cpl, choose_kernel
    from erasurehead_amd.parallel.placement import make_shards, place_spread, place_units

    prec = get_precision(precision)
    sch = make_scheme("approx", 8, 2, 1_000_000, 6, 0, allow_uneven=True)
    rows = sch.rows_per_partition
    mode = shard if n_gpus > 1 else "message"
    shards = make_shards(sch.messages, mode)
    owner = (place_units([[(p, rows) for p, _ in u.segments] for u in shards], n_gpus, 0.12) if mode == "partition"
             else place_spread([u.worker for u in shards], n_gpus))
    costs = []
    for r in range(n_gpus):  # time the heaviest rank
        mine = [u for u, o in zip(shards, owner) if o == r]
        costs.append((len({p for u in mine for p, _ in u.segments}), len(mine), r))
    _, _, r = max(costs)
    mine = [u for u, o in zip(shards, owner) if o == r]
    src = SyntheticSource(1_000_000, 1000, sch.n_partition_files, 1234)
    bundle_rows = rows_override
    need = sorted({p for u in mine for p, _ in u.segments})
    parts = {p: src.partition(p, prec, torch.device("cuda")) for p in need}
    msgs = [list(u.segments) for u in mine]
    choice = None
    if bundle_rows:  # the default kernel with another bundle length
        import collections

        max_rep = max(collections.Counter(p for m in msgs for p, _ in m).values())
        distinct = sum(parts[p][0].shape[0] for p in need)
        choice = replace(choose_kernel(prec.code, prec.ld(1000), choose_cpl(prec.ld(1000), prec.vec), max_rep, distinct),
                         bundle_rows=bundle_rows)
    if fill:  # the default kernel with every partition split evenly over the chip's workgroup slots
        import collections

        from erasurehead_amd.ops.grad import multi_slots

        max_rep = max(collections.Counter(p for m in msgs for p, _ in m).values())
        distinct = sum(parts[p][0].shape[0] for p in need)
        base = choice or choose_kernel(prec.code, prec.ld(1000), choose_cpl(prec.ld(1000), prec.vec), max_rep, distinct)
        if base.kind == "multi" and base.fold:
            cpl = choose_cpl(prec.ld(1000), prec.vec)
            choice = replace(base, fill=multi_slots(distinct, prec.code == 1, cpl=cpl) // 4)
    plan = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000, choice=choice)
    plan.rank, plan.n_parts, plan.n_shards, plan.shard_mode = r, len(need), len(mine), mode
    beta = torch.randn(prec.ld(1000), device="cuda", dtype=prec.acc) * 0.01
    G = plan.out_buffer()[0]
    return plan, beta, G


def one(n_gpus: int, precision: str, shard: str = "partition", rows_override: int = 0, fill: bool = False,
        slab_mode: int = 1, mfma_rows: int = 32, mfma_probe: int = 0, mfma_stream: int = 0) -> dict:
    import numpy as np
    import torch

    from erasurehead_amd._ext import native

    native().set_slab_reduce_mode(slab_mode)
    native().set_mfma_stage_rows(mfma_rows)
    native().set_mfma_probe(mfma_probe)  # (1 / 2: timing probes, not a gradient)
    native().set_mfma_stream(int(mfma_stream))
    plan, beta, G = build_plan(n_gpus, precision, shard, rows_override, fill)
    r, mode = plan.rank, plan.shard_mode
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_kernels import clock_warm  # ~150 ms of back-to-back launches: the clock ramp is over

    clock_warm(lambda: plan.run(beta, G))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for a, b in evs:
        a.record()
        plan.run(beta, G)
        b.record()
    torch.cuda.synchronize()
    all_ms = [a.elapsed_time(b) for a, b in evs]
    ms = float(np.median(all_ms))
    return {"n_gpus": n_gpus, "precision": precision, "shard": mode, "rank": r, "partitions": plan.n_parts,
            "shards": plan.n_shards, "bundle_rows": plan.bundle_rows, "kernel": plan.choice.label(), "ntasks": plan.ntasks,
            "kernel_ms": ms, "kernel_ms_min": float(np.min(all_ms)), "kernel_ms_max": float(np.max(all_ms)),
            "distinct_TBps": plan.distinct_bytes / ms / 1e9, "fill": plan.choice.fill,
            "slab_mode": slab_mode, "mfma_rows": mfma_rows, "mfma_probe": mfma_probe, "mfma_stream": mfma_stream}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rows-sweep", action="store_true")
    ap.add_argument("--rows-list", default="64,128,256,512", help="bundle lengths of --rows-sweep")
    ap.add_argument("--gpus-list", default="1,2,4,8")
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--shard", default="partition", choices=["partition", "message"])
    ap.add_argument("--one", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--rows", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--fill", action="store_true", help="also time even splits over the workgroup slots")
    ap.add_argument("--ab-slab", action="store_true", help="also time the two-stage slab reduction (mode 0)")
    ap.add_argument("--slab-mode", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--mfma-rows", type=int, default=32, help="bf16 MFMA bundles: rows per LDS stage (32 / 16)")
    ap.add_argument("--mfma-probe", type=int, default=0,
                    help="bf16 MFMA timing probe: 1 loads only, 2 compute only (3 / 4, --mfma-stream 3 / 4: loads with / "
                         "without the stage barriers, no LDS copies)")
    ap.add_argument("--mfma-stream", type=int, default=0,
                    help="bf16 packed bundles: 0 LDS-DMA ring (default), 3 VGPR-staged ring, 4 its three-set form")
    a = ap.parse_args()
    if a.one:
        print(json.dumps(one(a.one, a.precision, a.shard, a.rows, a.fill, a.slab_mode, a.mfma_rows, a.mfma_probe,
                             a.mfma_stream)),
              flush=True)
        return 0
    lines = []
    sweeps = [None] + ([int(x) for x in a.rows_list.split(",")] if a.rows_sweep else [])
    for n in [int(x) for x in a.gpus_list.split(",")]:
        variants = ([(r, False, 1) for r in sweeps] + ([(None, True, 1)] if a.fill else [])
                    + ([(None, False, 0)] if a.ab_slab else []))
        for rows, fill, mode in variants:
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", str(n), "--precision",
                                  a.precision, "--shard", a.shard, "--rows", str(rows or 0), "--slab-mode", str(mode)]
                                 + (["--fill"] if fill else []),
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-2000:], file=sys.stderr)
                return 1
            rec = json.loads(out.stdout.strip().splitlines()[-1])
            rec["rows_override"] = rows
            print(json.dumps(rec), flush=True)
            lines.append(rec)
    if a.out:
        with open(a.out, "w") as f:
            for r in lines:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
