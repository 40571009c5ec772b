"""Kernel microbenchmarks on one MI355X: the worker-gradient kernels in isolation.

    python tools/bench_kernels.py [--out FILE]

* dense ``grad_dense`` (fused single pass; two-pass above d = 2048 fp64) at several widths,
  reported as effective HBM bandwidth over the bytes of X it must stream;
* ``--only sweep``: d in {256, 1000, 2048, 4096} x n in {1e5, 1e6, 4e6} x fp64/fp32 against the
  device-copy ceiling, distinct-row and replica-bundle layouts;
* sparse one-hot gradients on covtype / kc_house / amazon-shaped data (the reference's real
  datasets, synthetic stand-ins of the same shape): the ELL path against the generic
  sorted-COO path.

Times are HIP-event medians over 50 launches after 5 warm-up launches.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def clock_warm(fn, ms: float = 150.0, min_calls: int = 5):
    """Run fn back to back for ~ms of wall-clock before timing: the GPU idles at ~160 MHz and its clock
    ramps over ~100 ms of streaming (profiles/round3/clocks); a 0.03-0.3 ms kernel timed after 5
    warm-up calls was measured on the ramp."""
    import time

    import torch

    t0, n = time.perf_counter(), 0
    while n < min_calls or (time.perf_counter() - t0) * 1e3 < ms:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def _time(fn, reps=50, warm=5):
    import torch

    clock_warm(fn, min_calls=warm)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))  # ms


def dense_cases(out):
    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    for prec_name in ("fp64", "fp32", "bf16"):
        prec = get_precision(prec_name)
        for d in (1000, 2048, 4000):
            rows = max(1, int(2e9 // (d * 8)))  # ~2 GB of fp64 X
            parts = {}
            for p in range(4):
                X = torch.randn(rows // 4, prec.ld(d), device="cuda", dtype=torch.float32).to(prec.storage)
                y = torch.where(torch.rand(rows // 4, device="cuda") > 0.5, 1.0, -1.0).to(prec.acc)
                parts[p] = (X.contiguous(), y)
            plan = DenseGradPlan([[(0, 1.0), (1, 1.0)], [(2, 1.0), (3, 1.0)]], parts, prec, LOGISTIC, d)
            beta = torch.randn(prec.ld(d), device="cuda", dtype=prec.acc) * 0.01
            G = plan.out_buffer()[0]
            ms = _time(lambda: plan.run(beta, G))
            gb = plan.bytes_per_round / 1e9
            r = {"kernel": "grad_dense" + ("" if plan.cpl else "_twopass"), "precision": prec_name, "d": d,
                 "rows": rows, "ms": ms, "x_gbytes": gb, "effective_TBps": gb / ms}
            out.append(r)
            print(json.dumps(r), flush=True)
            del parts, plan
            torch.cuda.empty_cache()


def scale_cases(out):
    """fp64 d = 1000 at the per-rank sizes of the headline at N = 8/4/2/1 GPUs, task-count sweep.

    Also times torch's sum over the same bytes as a read-bandwidth reference.
    """
    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    prec = get_precision("fp64")
    d, rpp = 1000, 125000  # headline partition: 1e6 / 8 rows
    parts = {}
    for p in range(22):
        X = torch.randn(rpp, prec.ld(d), device="cuda", dtype=torch.float64)
        y = torch.where(torch.rand(rpp, device="cuda") > 0.5, 1.0, -1.0).double()
        parts[p] = (X, y)
    beta = torch.randn(prec.ld(d), device="cuda", dtype=torch.float64) * 0.01
    # FRC-style replicas on one GPU (headline layout: groups {0,1,2} x3, {3,4,5} x3, {6,7} x2): 22 GB of
    # message rows over 8 GB of distinct partitions; concurrently running replica tasks share L2/MALL lines
    frc = [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2
    for tasks in (2048, 5120):
        plan = DenseGradPlan([[(p, 1.0) for p in m] for m in frc], {p: parts[p] for p in range(8)}, prec, LOGISTIC,
                             d, target_tasks=tasks)
        G = plan.out_buffer()[0]
        ms = _time(lambda: plan.run(beta, G), reps=20)
        gb = plan.bytes_per_round / 1e9
        r = {"kernel": "grad_dense_scale_frc_replicas", "message_gbytes": gb, "distinct_gbytes": 8.0,
             "tasks": plan.ntasks, "ms": ms, "effective_TBps": gb / ms, "distinct_TBps": 8.0 / ms}
        out.append(r)
        print(json.dumps(r), flush=True)
        del plan
    for nparts in (3, 6, 11, 22):
        msgs = [[(p, 1.0) for p in range(q, min(nparts, q + 3))] for q in range(0, nparts, 3)]
        X0 = parts[0][0]
        ref_ms = _time(lambda: [parts[p][0].sum() for p in range(nparts)], reps=10)
        for tasks in (1280, 2048, 2560, 3840, 5120):
            plan = DenseGradPlan(msgs, {p: parts[p] for p in range(nparts)}, prec, LOGISTIC, d, target_tasks=tasks)
            G = plan.out_buffer()[0]
            ms = _time(lambda: plan.run(beta, G), reps=20)
            gb = plan.bytes_per_round / 1e9
            r = {"kernel": "grad_dense_scale", "parts": nparts, "tasks": plan.ntasks, "ms": ms, "x_gbytes": gb,
                 "effective_TBps": gb / ms, "torch_sum_ms": ref_ms, "torch_sum_TBps": gb / ref_ms}
            out.append(r)
            print(json.dumps(r), flush=True)
            del plan


def sweep_cases(out, ds=(256, 1000, 2048, 4096), ns=(100_000, 1_000_000, 4_000_000), precs=("fp64", "fp32")):
    """Shape sweep of the dense gradient against the device-copy ceiling (round-2 verdict item 6).

    For every (precision, d, n): n rows in 8 partitions, two message layouts -- ``naive`` (one
    partition per message, distinct rows) and ``agc`` (the headline's replica bundles: groups
    {0,1,2}x3, {3,4,5}x3, {6,7}x2) -- with the kernel ``choose_kernel`` picks for that shape.  The
    ceiling is a device-to-device copy of one partition (read + write bytes / time); ``frac`` is the
    kernel's distinct-X read rate over it.
    """
    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision

    layouts = {"naive": [[p] for p in range(8)], "agc": [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2}
    for prec_name in precs:
        prec = get_precision(prec_name)
        for d in ds:
            for n in ns:
                rpp = n // 8
                parts = {}
                for p in range(8):
                    X = torch.empty(rpp, prec.ld(d), device="cuda", dtype=prec.storage).uniform_(-1, 1)
                    y = torch.where(torch.rand(rpp, device="cuda") > 0.5, 1.0, -1.0).to(prec.acc)
                    parts[p] = (X, y)
                nbytes = parts[0][0].numel() * parts[0][0].element_size()
                dst = torch.empty_like(parts[0][0])
                copy_ms = _time(lambda: dst.copy_(parts[0][0]), reps=20)
                ceiling = 2 * nbytes / copy_ms / 1e9  # TB/s
                del dst
                beta = torch.randn(prec.ld(d), device="cuda", dtype=prec.acc) * 0.01
                for lay, msgs in layouts.items():
                    plan = DenseGradPlan([[(p, 1.0) for p in m] for m in msgs], parts, prec, LOGISTIC, d)
                    G = plan.out_buffer()[0]
                    ms = _time(lambda: plan.run(beta, G), reps=20)
                    distinct = 8 * nbytes / 1e12  # TB
                    r = {"kernel": "grad_dense_sweep", "precision": prec_name, "d": d, "n": n, "layout": lay,
                         "choice": plan.choice.label() if plan.choice else "twopass", "ms": ms,
                         "distinct_TBps": distinct / ms * 1e3, "copy_TBps": ceiling,
                         "frac": distinct / ms * 1e3 / ceiling}
                    out.append(r)
                    print(json.dumps(r), flush=True)
                    del plan, G
                del parts
                torch.cuda.empty_cache()


def choice_cases(out, shapes=(("fp64", 256, 1_000_000), ("fp32", 256, 1_000_000), ("fp64", 256, 100_000),
                                ("fp64", 4096, 1_000_000), ("fp32", 4096, 1_000_000), ("fp32", 2048, 1_000_000),
                                ("fp64", 1000, 100_000)), layout: str = "agc"):
    """Every valid KernelChoice on the replica-bundle layout of a few shapes: the candidates
    behind choose_kernel's table (tests/test_plan_tables.py pins the picks).  layout agc: the
    headline's uneven AGC groups (3 replicas); frc2: FRC s = 1 (4 groups of 2 workers x 2 partitions);
    frc4: FRC / AGC s = 3 (2 groups of 4 workers x 4 partitions); naive: one partition per message."""
    import dataclasses

    import torch

    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import DenseGradPlan, get_precision
    from erasurehead_amd.ops.grad import KernelChoice

    msgs = {"agc": [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2,
            "frc2": [[2 * g, 2 * g + 1] for g in range(4) for _ in range(2)],
            "frc4": [[0, 1, 2, 3]] * 4 + [[4, 5, 6, 7]] * 4,
            "naive": [[p] for p in range(8)]}[layout]
    R = {"agc": 3, "frc2": 2, "frc4": 4, "naive": 1}[layout]
    for prec_name, d, n in shapes:
        prec = get_precision(prec_name)
        rpp = n // 8
        parts = {p: (torch.empty(rpp, prec.ld(d), device="cuda", dtype=prec.storage).uniform_(-1, 1),
                     torch.where(torch.rand(rpp, device="cuda") > 0.5, 1.0, -1.0).to(prec.acc)) for p in range(8)}
        beta = torch.randn(prec.ld(d), device="cuda", dtype=prec.acc) * 0.01
        distinct = 8 * parts[0][0].numel() * parts[0][0].element_size() / 1e12
        cands = [KernelChoice("fused", rows=r, interleave=i) for r in (1, 2, 4) for i in (False, True)]
        cands += [KernelChoice("multi", replicas=R, bundle_rows=b, fold=True, lane_epi=e)
                  for b in (32, 64, 128, 192, 256, 512, 768, 1024) for e in (False, True)]
        cands += [KernelChoice("multi", replicas=R, bundle_rows=b, fold=True, pair=True)
                  for b in (8, 16, 32, 64, 128, 192, 256, 512, 768)]
        cands += [KernelChoice("staged", replicas=R, bundle_rows=b, pair=p, wpr=w)
                  for b in (64, 128, 192, 256, 384, 496, 512, 768, 1024) for p in (False, True) for w in (0, 1)]
        cands += [KernelChoice("wide", interleave=i) for i in (False, True)]
        cands += [KernelChoice("wide", replicas=R, bundle_rows=b) for b in (64, 128, 192, 208, 256, 512, 976, 1968)]
        default = None
        for c in [None] + cands:
            try:
                plan = DenseGradPlan([[(p, 1.0) for p in m] for m in msgs], parts, prec, LOGISTIC, d, choice=c)
            except (ValueError, RuntimeError):
                continue
            G = plan.out_buffer()[0]
            try:
                ms = _time(lambda: plan.run(beta, G), reps=20)
            except RuntimeError:
                continue
            if c is None:
                default = plan.choice
            r = {"kernel": "grad_dense_choice", "layout": layout, "precision": prec_name, "d": d, "n": n,
                 "choice": dataclasses.asdict(plan.choice), "label": plan.choice.label(), "default": c is None,
                 "ms": ms, "distinct_TBps": distinct / ms * 1e3}
            out.append(r)
            print(json.dumps(r), flush=True)
            del plan, G
        del parts
        torch.cuda.empty_cache()


def eval_cases(out):
    """Post-hoc evaluation GEMM (MFMA, loss fused): X [n, 1000] . B[100, 1000]^T, fp64 / fp32."""
    import torch

    from erasurehead_amd._ext import native
    from erasurehead_amd.models.losses import LOGISTIC

    for dt, n in ((torch.float64, 1_000_000), (torch.float32, 1_000_000)):
        d, R = 1000, 100
        X = torch.randn(n, d, device="cuda", dtype=dt)
        y = torch.where(torch.rand(n, device="cuda") > 0.5, 1.0, -1.0).to(dt)
        B = (torch.randn(R, d, device="cuda", dtype=dt) * 0.01).contiguous()
        s = torch.zeros(R, dtype=torch.float64, device="cuda")
        ms = _time(lambda: native().eval_gemm_loss(LOGISTIC, X, n, d, y, B, s, None), reps=10, warm=2)
        flops = 2.0 * n * d * R
        r = {"kernel": "eval_gemm_loss", "dtype": str(dt), "n": n, "d": d, "R": R, "ms": ms,
             "TFLOPs": flops / ms / 1e9, "x_TBps": n * d * X.element_size() / ms / 1e9}
        out.append(r)
        print(json.dumps(r), flush=True)
        del X


UNITS_PROBE = False  # --units-probe


def sparse_cases(out, names=("covtype", "kc_house_data", "amazon-dataset"), ell_only=False, layouts_only=None,
                 rows="both"):
    import torch

    from erasurehead_amd.data.synthetic import REAL_SHAPES, onehot_partitions
    from erasurehead_amd.models.losses import LOGISTIC
    from erasurehead_amd.ops import SparseGradPlan, get_precision

    prec = get_precision("fp64")
    for name in names:
        n, d, f = REAL_SHAPES[name]
        W = 8
        parts_l, _, dd = onehot_partitions(n, d, f, W, seed=1)
        parts = {p: xy for p, xy in enumerate(parts_l)}
        layouts = {"naive": [[(w, 1.0)] for w in range(W)],
                   "s1_replicas": [[(w, 1.0), ((w + 1) % W, 1.0)] for w in range(W)],  # 8 workers, 2 partitions each
                   # FRC / AGC s = 1: groups {2g, 2g + 1} send the sum of both partitions (merged units when small)
                   "frc_s1": [[(w - w % 2, 1.0), (w - w % 2 + 1, 1.0)] for w in range(W)]}
        if layouts_only:
            layouts = {k: v for k, v in layouts.items() if k in layouts_only}
        ells = (True,) if ell_only else ("auto",) if rows == "auto" else (True, False)
        for (layout, msgs), use_ell in [(x, e) for x in layouts.items() for e in ells]:
            plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, dd, device="cuda", use_ell=use_ell)
            beta = torch.randn(prec.ld(dd), device="cuda", dtype=torch.float64) * 0.1
            G = plan.out_buffer()[0]
            if UNITS_PROBE and plan.dst is not None:  # timing probe, not a gradient: each unit's first row only
                plan.dst[:, 1:] = -1
            ms = _time(lambda: plan.run(beta, G))
            kern = ("ell16" if plan.idx16 else "ell32") if plan.ell else "csr"
            r = {"kernel": f"grad_sparse ({kern} rows, CSC{16 if plan.row16 else 32} tiles)", "layout": layout,
                 "units": len(plan.units) if plan.units else None, "identity": bool(plan.identity),
                 "dataset_shape": name, "rows_distinct": plan.nrows, "rows_in_messages": plan.msg_rows,
                 "nnz": int(plan.nnz), "d": dd, "ms": ms, "nnz_per_us": plan.nnz / (ms * 1e3),
                 "stream_bytes": plan.stream_bytes, "TBps": plan.stream_bytes / (ms * 1e9)}
            out.append(r)
            print(json.dumps(r), flush=True)
            del plan
            torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "kernels.jsonl"))
    ap.add_argument("--shapes", default=None, help="--only choices: prec:d:n,... (default: the built-in list)")
    ap.add_argument("--layout", default="agc", choices=["agc", "frc2", "frc4", "naive"],
                    help="--only choices: replica layout")
    ap.add_argument("--only", choices=["dense", "sparse", "scale", "eval", "sweep", "choices"], default=None)
    ap.add_argument("--ds", default="256,1000,2048,4096", help="--only sweep: row widths")
    ap.add_argument("--ns", default="1e5,1e6,4e6", help="--only sweep: row counts")
    ap.add_argument("--precs", default="fp64,fp32", help="--only sweep: precisions")
    ap.add_argument("--sparse-shapes", default="covtype,kc_house_data,amazon-dataset", help="--only sparse: datasets")
    ap.add_argument("--ell-only", action="store_true", help="--only sparse: skip the CSR row pass")
    ap.add_argument("--sparse-layouts", default=None, help="--only sparse: naive,s1_replicas,frc_s1 (default: all)")
    ap.add_argument("--units-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sparse-rows", default="both", choices=["both", "auto"],
                    help="--only sparse: both row passes, or the plan's own choice")
    ap.add_argument("--wg-tiles", type=int, default=0, help="--only sparse: tiles per column-pass workgroup (A/B)")
    ap.add_argument("--row-block", type=int, default=0, help="--only sparse: column-pass sub-block rows (A/B, <= 4096)")
    ap.add_argument("--wg-slots", type=int, default=0, help="--only sparse: workgroup budget of the chip-sized chunks (A/B)")
    ap.add_argument("--no-wg-spans", action="store_true",
                    help="--only sparse: whole 16-tile chunks and the csc_spans launch (A/B of SparseGradPlan.WG_SPANS)")
    a = ap.parse_args()
    global UNITS_PROBE
    UNITS_PROBE = a.units_probe
    if a.row_block:
        from erasurehead_amd.ops import SparseGradPlan

        SparseGradPlan.ROW_BLOCK_ROWS = a.row_block
    if a.no_wg_spans or a.wg_tiles or a.wg_slots:
        from erasurehead_amd.ops import SparseGradPlan

        SparseGradPlan.WG_SPANS = not a.no_wg_spans
        SparseGradPlan.WG_TILES = a.wg_tiles or SparseGradPlan.WG_TILES
        SparseGradPlan.WG_SLOTS = a.wg_slots or SparseGradPlan.WG_SLOTS
    out = []
    if a.only in (None, "dense"):
        dense_cases(out)
    if a.only == "scale":
        scale_cases(out)
    if a.only == "eval":
        eval_cases(out)
    if a.only == "sweep":
        sweep_cases(out, ds=tuple(int(x) for x in a.ds.split(",")), ns=tuple(int(float(x)) for x in a.ns.split(",")),
                    precs=tuple(a.precs.split(",")))
    if a.only == "choices":
        if a.shapes:
            choice_cases(out, [(p, int(d), int(float(n))) for p, d, n in (x.split(":") for x in a.shapes.split(","))],
                         layout=a.layout)
        else:
            choice_cases(out, layout=a.layout)
    if a.only in (None, "sparse"):
        sparse_cases(out, names=tuple(a.sparse_shapes.split(",")), ell_only=a.ell_only,
                     layouts_only=a.sparse_layouts.split(",") if a.sparse_layouts else None, rows=a.sparse_rows)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
