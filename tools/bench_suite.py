"""Secondary benchmark suite: every config BASELINE.json lists, on one MI355X.

    python tools/bench_suite.py [--quick] [--out DIR]

Configs (BASELINE.json "configs"; synthetic stand-ins where the reference used real data,
which is not available offline — same shapes and one-hot structure, see
data/synthetic.py onehot_partitions):
  naive_dense        naive uncoded logistic, synthetic GMM 1e6 x 1e3, W=8
  agc_dense          approximate coding (AGC), same data, W=8 s=2 k=6 (uneven groups)
  cyclic_dense       exact cyclic-MDS (EGC), same data, W=8 s=2
  frc_dense          exact FRC (replication), same data, W=8 s=1
  partialrep_covtype partial replication, covtype-shaped one-hot (396112 x 15509), W=8 s=1 P=4,
                     injected Exp(0.05) delays (forced; the reference only relies on natural stragglers;
                     mean 0.05 s instead of 0.5 s keeps the run short — floors scale linearly)
  avoid_covtype      ignore-stragglers, same data, W=8 s=1, forced delays
  naive_covtype      naive on the same 8-partition covtype-shaped data (the family's loss target)
  agc_covtype        AGC on the covtype-shaped data without delays (sparse kernel throughput)
  ls_kc_house_*      least squares on kc_house-shaped one-hot (17290 x 27654): naive vs AGC with
                     num_collect in {4,5,6,7}, W=8 s=1
  agc_amazon         AGC W=8 s=1 k=6 on amazon-shaped one-hot (26215 x 241915, 45 nnz/row; 1.94 MB
                     messages), and naive on the same data (the family's loss target), both on the same
                     device-driven loop; agc_amazon_instrumented: the same AGC host-driven with HIP-event
                     instrumentation (gradient / combine+update kernel microseconds), its own row.
                     Synthetic stand-in: parity unpinned.

Per config: seconds per round (timed, device-synchronised), time-to-decode (reference
``timeset``), iterations to the COMMON loss target of its data family (the naive run on the same
data: final training loss + 1 %; "-" if never reached or the family has no naive run), the
iterations to the run's own floor (within 1 % of its best loss; not comparable across schemes),
and for delayed runs the deterministic injected-delay floor and the overhead above it
(SURVEY §6).  Writes suite.jsonl and suite.md.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _floor_iters(tl: np.ndarray) -> int:
    floor = float(np.min(tl))
    return int(np.argmax(tl <= floor + 0.01 * abs(floor)))


def _target_iters(tl, target):
    hit = np.nonzero(np.asarray(tl) <= target)[0]
    return int(hit[0]) + 1 if hit.size else None


def run_config(name, cfg_kw, source=None, rounds=100, timed_from=5, delay_floor_kw=None, device_loop="auto",
               instrument=False):
    import torch

    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.engine import Trainer, evaluate
    from erasurehead_amd.parallel.dist import DistEnv
    from erasurehead_amd.utils.delay import delay_floor

    cfg = RunConfig(**cfg_kw, num_itrs=rounds, verbose=False, seed=0, device_loop="off" if instrument else device_loop,
                    instrument=instrument)
    env = DistEnv(device=torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    t0 = time.perf_counter()
    tr = Trainer(cfg, env, source)
    setup = time.perf_counter() - t0
    if torch.cuda.is_available() and tr.local_msgs:
        # ~150 ms of back-to-back gradients first: the clock ramps from idle over ~100 ms of streaming
        # (profiles/round3/clocks), and 100 rounds of ~1 ms would otherwise be timed on the ramp
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.15:
            tr.warmup()
            torch.cuda.synchronize()
    res = tr.run(timed_start=timed_from)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t_ev = time.perf_counter()
    ev = evaluate(tr, res, write=False)
    eval_s = time.perf_counter() - t_ev
    out = {
        "config": name,
        "scheme": tr.key,
        "loss": "least_squares" if tr.loss else "logistic",
        "W": cfg.n_workers, "s": cfg.n_stragglers, "num_collect": cfg.num_collect, "partitions": cfg.partitions,
        "n_rows": cfg.n_rows, "n_cols": cfg.n_cols, "rounds": rounds, "add_delay": cfg.add_delay,
        "sec_per_round": res.timed_seconds / max(1, res.timed_rounds),
        "timeset_mean_ms": 1e3 * float(np.mean(res.timeset[timed_from:])),
        "sum_timeset_s": float(np.sum(res.timeset)),
        "iters_to_loss_floor": _floor_iters(ev.training_loss),
        "final_train_loss": float(ev.training_loss[-1]),
        "train_loss": [float(x) for x in ev.training_loss],
        "final_test_loss": float(ev.testing_loss[-1]),
        "final_auc": float(ev.auc[-1]) if not tr.loss else None,
        "setup_s": setup,
        "native_loop": tr.native_loop,
        "round_loop": tr.device_loop or ("host-native" if tr.native_loop else "host-python"),
        "precision": cfg.precision,
        # replica messages (Trainer.replica_policy): "separate" arithmetic per replica (dense), "encoded"
        # from one gradient per distinct partition (sparse plans), "none" (no partition hosted twice)
        "replicas": tr.replica_policy,
        "message_bytes": int(tr.ld * torch.tensor([], dtype=tr.prec.acc).element_size()),
        "eval_s": eval_s,
        "grad_kernel_us_isolated": tr.time_local_grad(),
    }
    rep = tr.rank_report()
    for k in ("kernel_us", "update_kernel_us", "wait_k_us", "decode_update_us"):
        if k in rep:
            out[k] = rep[k]
    if delay_floor_kw is not None:
        fl = delay_floor(cfg.n_workers, rounds, mean=cfg.delay_mean, **delay_floor_kw)
        out["delay_floor_s"] = fl
        out["overhead_above_floor_ms_per_round"] = 1e3 * (out["sum_timeset_s"] - fl) / rounds
    tr.close()
    del tr
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return out


def run_child(name, a) -> dict:
    """One config in a fresh process (tools/bench_suite.py --only NAME --in-process); its suite row."""
    import subprocess
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        cmd = [sys.executable, os.path.abspath(__file__), "--only", name, "--in-process", "--out", tmp,
               "--device-loop", a.device_loop] + (["--quick"] if a.quick else [])
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
        if out.returncode != 0:
            raise RuntimeError(f"{name}: child exited {out.returncode}: {out.stderr[-2000:]}")
        with open(os.path.join(tmp, "suite.jsonl")) as f:
            return json.loads(f.readline())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="10x smaller problems (plumbing check)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--only", default=None, help="comma-separated config names")
    ap.add_argument("--device-loop", default="auto", choices=["auto", "graph", "stream", "off"])
    ap.add_argument("--in-process", action="store_true",
                    help="run the dense configs in this process too (default: one fresh process each, like bench.py: "
                         "8 GB of X allocated after another config's freed 8 GB streamed up to 9 %% slower)")
    a = ap.parse_args()
    from erasurehead_amd.data.source import ArraySource
    from erasurehead_amd.data.synthetic import REAL_SHAPES, onehot_partitions

    scale = 10 if a.quick else 1
    n_dense = 1_000_000 // scale
    dense = dict(n_procs=9, n_rows=n_dense, n_cols=1000, input_dir="/tmp/eh_suite/", is_real=0, dataset="synthetic",
                 data="synthetic", data_seed=1234, update_rule="AGD")
    configs = []
    # (name, RunConfig kwargs, data source, delay-floor kwargs, instrumented, data family)
    configs.append(("naive_dense", dict(dense, is_coded=0), None, None, False, "dense"))
    configs.append(("agc_dense", dict(dense, is_coded=1, n_stragglers=2, coded_ver=3, num_collect=6,
                                      allow_uneven_groups=True), None, None, False, "dense"))
    configs.append(("cyclic_dense", dict(dense, is_coded=1, n_stragglers=2, coded_ver=0), None, None, False, "dense"))
    configs.append(("frc_dense", dict(dense, is_coded=1, n_stragglers=1, coded_ver=1), None, None, False, "dense"))

    # covtype-shaped one-hot; partial schemes need (P - s) * W partition files.  Sources are built on first
    # use (a dense-only child process never generates the one-hot ones)
    import functools

    n_cov, d_cov, f_cov = REAL_SHAPES["covtype"]
    n_cov //= scale
    W, s, P = 8, 1, 4

    @functools.lru_cache(None)
    def cov_pr():
        cov_parts, cov_test, dc = onehot_partitions(n_cov, d_cov, f_cov, (P - s) * W, seed=3)
        return ArraySource(cov_parts, cov_test, sparse=True), sum(p[0].shape[0] for p in cov_parts), dc

    @functools.lru_cache(None)
    def cov8():
        parts, test, dc = onehot_partitions(n_cov, d_cov, f_cov, W, seed=3)
        return ArraySource(parts, test, sparse=True), sum(p[0].shape[0] for p in parts), dc

    def base_cov(src):
        return dict(n_procs=W + 1, n_rows=src[1], n_cols=src[2], input_dir="/tmp/eh_suite/", is_real=1,
                    dataset="covtype", update_rule="AGD", add_delay=1, force_delay=True, delay_mean=0.05)

    configs.append(("partialrep_covtype", lambda: dict(base_cov(cov_pr()), is_coded=1, n_stragglers=s, partitions=P,
                                                       coded_ver=1),
                    lambda: cov_pr()[0], {"stop_count": W}, False, "covtype_24parts"))
    configs.append(("naive_covtype", lambda: dict(base_cov(cov8()), is_coded=0, add_delay=0, force_delay=False),
                    lambda: cov8()[0], None, False, "covtype"))
    configs.append(("avoid_covtype", lambda: dict(base_cov(cov8()), is_coded=1, n_stragglers=s, coded_ver=2),
                    lambda: cov8()[0], {"stop_count": W - s, "carry": True}, False, "covtype"))
    configs.append(("agc_covtype", lambda: dict(base_cov(cov8()), is_coded=1, n_stragglers=s, coded_ver=3,
                                                num_collect=6, add_delay=0, force_delay=False),
                    lambda: cov8()[0], None, False, "covtype"))

    n_kc, d_kc, f_kc = REAL_SHAPES["kc_house_data"]

    @functools.lru_cache(None)
    def kc():
        parts, test, dk = onehot_partitions(n_kc, d_kc, f_kc, W, seed=5, least_squares=True)
        return ArraySource(parts, test, sparse=True), sum(p[0].shape[0] for p in parts), dk

    def base_kc():
        src = kc()
        return dict(n_procs=W + 1, n_rows=src[1], n_cols=src[2], input_dir="/tmp/eh_suite/", is_real=1,
                    dataset="kc_house_data", update_rule="AGD", loss="least_squares", lr=0.2)

    configs.append(("ls_kc_house_naive", lambda: dict(base_kc(), is_coded=0), lambda: kc()[0], None, False,
                    "kc_house"))
    for k in (4, 5, 6, 7):
        configs.append((f"ls_kc_house_agc_k{k}",
                        functools.partial(lambda k: dict(base_kc(), is_coded=1, n_stragglers=1, coded_ver=3,
                                                         num_collect=k), k),
                        lambda: kc()[0], None, False, "kc_house"))
    n_am, d_am, f_am = REAL_SHAPES["amazon-dataset"]

    @functools.lru_cache(None)
    def am():
        parts, test, da = onehot_partitions(n_am // scale, d_am, f_am, W, seed=21)
        return ArraySource(parts, test, sparse=True), sum(p[0].shape[0] for p in parts), da

    def base_am():
        src = am()
        return dict(n_procs=W + 1, n_rows=src[1], n_cols=src[2], input_dir="/tmp/eh_suite/", is_real=1,
                    dataset="amazon-dataset", update_rule="AGD")

    configs.append(("naive_amazon", lambda: dict(base_am(), is_coded=0), lambda: am()[0], None, False, "amazon"))
    # the AGC / naive pair runs the same (device-driven) loop; the instrumented host-driven run is its own row
    configs.append(("agc_amazon", lambda: dict(base_am(), is_coded=1, n_stragglers=1, coded_ver=3, num_collect=6),
                    lambda: am()[0], None, False, "amazon"))
    configs.append(("agc_amazon_instrumented",
                    lambda: dict(base_am(), is_coded=1, n_stragglers=1, coded_ver=3, num_collect=6),
                    lambda: am()[0], None, True, "amazon"))
    if a.only:
        keep = set(a.only.split(","))
        configs = [c for c in configs if c[0] in keep]
    os.makedirs(a.out, exist_ok=True)
    rows = []
    with open(os.path.join(a.out, "suite.jsonl"), "w") as f:
        for name, kw, src, floor_kw, inst, fam in configs:
            if fam == "dense" and not a.in_process:
                r = run_child(name, a)
            else:
                r = run_config(name, kw() if callable(kw) else kw, src() if callable(src) else src,
                               delay_floor_kw=floor_kw, device_loop=a.device_loop, instrument=inst)
            r["family"] = fam
            rows.append(r)
            f.write(json.dumps(r) + "\n")
            f.flush()
            print(json.dumps(r), flush=True)
    # common target per data family: the naive run's final training loss + 1 %
    targets = {r["family"]: r["final_train_loss"] + 0.01 * abs(r["final_train_loss"])
               for r in rows if r["scheme"] == "naive"}
    for r in rows:
        t = targets.get(r["family"])
        r["loss_target"] = t
        r["iters_to_target"] = _target_iters(r["train_loss"], t) if t is not None else None
    hdr = ("Column `replicas`: how the replica messages of a partition hosted several times are formed -- `separate` "
           "(every replica's own arithmetic from one shared read: the dense plans, the headline), `encoded` (one "
           "gradient per distinct partition, replicas formed by the device encoding: the sparse plans) or `none` (no "
           "partition hosted twice).  Compare AGC against naive within one policy and one loop only.\n\n"
           "| config | scheme | W | s | k | replicas | loop | ms/round | timeset ms | iters to naive target | "
           "iters to own floor | final train loss | AUC | delay floor s | overhead ms/round | msg KB | grad µs | "
           "combine µs | eval s |\n"
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|\n")
    lines = []
    for r in rows:
        tgt = "-" if r["iters_to_target"] is None else str(r["iters_to_target"])
        auc = "%.4f" % r["final_auc"] if r.get("final_auc") is not None else "-"
        fl = "%.2f" % r["delay_floor_s"] if "delay_floor_s" in r else "-"
        ov = "%.3f" % r["overhead_above_floor_ms_per_round"] if "delay_floor_s" in r else "-"
        lines.append(f"| {r['config']} | {r['scheme']} | {r['W']} | {r['s']} | {r['num_collect']} | "
                     f"{r.get('replicas', '-')} | {r['round_loop']} | "
                     f"{1e3 * r['sec_per_round']:.3f} | {r['timeset_mean_ms']:.3f} | {tgt} | {r['iters_to_loss_floor']} | "
                     f"{r['final_train_loss']:.5f} | {auc} | {fl} | {ov} | {r['message_bytes'] / 1024:.0f} | "
                     f"{r.get('kernel_us', r.get('grad_kernel_us_isolated') or 0):.0f} | "
                     f"{r.get('update_kernel_us', float('nan')):.1f} | {r['eval_s']:.3f} |")
    with open(os.path.join(a.out, "suite.jsonl"), "w") as f:  # again, with the targets filled in
        for r in rows:
            f.write(json.dumps(r) + "\n")
    with open(os.path.join(a.out, "suite.md"), "w") as f:
        f.write(hdr + "\n".join(lines) + "\n")
    print(hdr + "\n".join(lines))


if __name__ == "__main__":
    main()
