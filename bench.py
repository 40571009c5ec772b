"""Headline benchmark: AGC logistic regression, synthetic 1e6 x 1e3, 8 workers, s=2, k=6.

Metric (BASELINE.json): "wall-clock sec/iter + iters-to-loss-floor, logistic regression
n_stragglers=2, 1/2/4/8 MI355X".  One *step* = one full training round of approximate
gradient coding: master sends beta to every worker rank over RCCL p2p, every logical
worker computes its (s+1)-replicated gradient with the fused HIP kernel, the master waits
for the stop rule (k = num_collect arrivals or every FRC group covered), decodes, runs
the fused combine+AGD update and drains the straggler tail (ref approximate_coding.py).
The problem is fixed (1e6 x 1e3, W = 8 logical workers) and spread over N GPUs:
strong scaling.  W % (s+1) != 0 for W=8, s=2, so the FRC groups are {0,1,2},{3,4,5},{6,7}
(--allow-uneven-groups extension; the reference would refuse this config).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]   (N>1: launched by torchrun)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

METRIC = "wall-clock sec/iter + iters-to-loss-floor, logistic regression n_stragglers=2, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n-rows", type=int, default=1_000_000)
    ap.add_argument("--n-cols", type=int, default=1000)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--stragglers", type=int, default=2)
    ap.add_argument("--num-collect", type=int, default=6)
    ap.add_argument("--coded-ver", type=int, default=3)
    ap.add_argument("--naive", action="store_true", help="uncoded baseline (is_coded=0), not the headline")
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32", "bf16"])
    ap.add_argument("--update-rule", default="AGD")
    ap.add_argument("--add-delay", type=int, default=0)
    ap.add_argument("--no-floor", action="store_true", help="skip the 100-round iters-to-loss-floor run")
    ap.add_argument("--floor-rounds", type=int, default=100)
    ap.add_argument("--tasks", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--transport", default="auto", choices=["auto", "ipc", "rccl"])
    ap.add_argument("--round-timeout", type=float, default=120.0, help="bounds any hang (a round takes ms)")
    ap.add_argument("--device-loop", default="auto", choices=["auto", "graph", "stream", "off"])
    ap.add_argument("--share-partitions", action="store_true",
                    help="co-located workers stream each distinct partition once (not the headline)")
    return ap.parse_args()


def main() -> int:
    a = parse()
    import torch

    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.engine import Trainer, evaluate
    from erasurehead_amd.parallel.dist import init_distributed

    env = init_distributed("auto")
    if env.world != a.gpus and env.is_master:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={env.world}", file=sys.stderr)

    def make_cfg(rounds: int) -> RunConfig:
        return RunConfig(a.workers + 1, a.n_rows, a.n_cols, "/tmp/erasurehead_bench/", 0, "synthetic",
                         0 if a.naive else 1,
                         a.stragglers, 0, a.coded_ver, a.num_collect, a.add_delay, a.update_rule,
                         num_itrs=rounds, precision=a.precision, data="synthetic", data_seed=1234, seed=0,
                         allow_uneven_groups=True, verbose=False, tasks=a.tasks,
                         transport=a.transport, round_timeout=a.round_timeout,
                         share_partitions=a.share_partitions, device_loop=a.device_loop)

    t_setup = time.perf_counter()
    trainer = Trainer(make_cfg(a.warmup + a.steps), env)
    setup_s = time.perf_counter() - t_setup
    res = trainer.run(timed_start=a.warmup)
    # timed region: barrier + device sync on both sides on every rank; MAX over ranks
    mine = res.timed_seconds if env.is_master else trainer.worker_timed_seconds
    timed = env.allreduce_max(mine)
    transport = trainer.transport
    out = {}
    if env.is_master:
        sec_per_iter = timed / a.steps
        ts = res.timeset[a.warmup:]
        lt = res.loop_time[a.warmup:]
        out = {
            "metric": METRIC,
            "value": sec_per_iter,
            "unit": "s/iter",
            "n_gpus": env.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * sec_per_iter,
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": a.precision,
            "data": "synthetic (on-device GMM of ref generate_data.py; random-init beta)",
            "config": {
                "model": "L2 logistic regression (d=%d)" % a.n_cols,
                "scheme": "naive (uncoded)" if a.naive else {3: "approx (AGC)", 1: "replication (FRC)",
                                                            0: "coded (cyclic MDS)",
                                                            2: "avoidstragg"}.get(a.coded_ver, str(a.coded_ver)),
                "global_batch": a.n_rows,
                "seq_len": None,
                "n_rows": a.n_rows, "n_cols": a.n_cols, "workers": a.workers,
                "n_stragglers": a.stragglers, "num_collect": a.num_collect, "add_delay": a.add_delay,
                "update_rule": a.update_rule,
                "parallelism": f"ps-master + {a.workers} logical workers on {env.world} GPU(s) (dp{env.world})",
                "transport": transport,
            },
            "time_to_decode_ms_median": float(1e3 * np.median(ts)),
            "loop_ms_median": float(1e3 * np.median(lt)),
            # X bytes the rank-0 messages read per round (replicas counted each time) and the bytes of
            # the distinct partitions behind them; co-located replicas share reads through L2
            "x_message_bytes_per_step_rank0": int(getattr(trainer.plan, "bytes_per_round", 0)) or None,
            "x_distinct_bytes_rank0": int(getattr(trainer.plan, "distinct_bytes", 0)) or None,
            "setup_s": setup_s,
            "phases_us": {k: round(v["mean_us"], 1) for k, v in res.phases.items()},
        }
        out["config"]["round_loop"] = {"graph": "device-driven, hipGraph", "stream": "device-driven"}.get(
            trainer.device_loop, "host-driven (native pump)")
        if a.share_partitions:
            out["config"]["share_partitions"] = True
        ref = _ref_cpu_equiv()
        if ref and (a.n_rows, a.n_cols, a.workers, a.stragglers) == (ref["n_rows"], ref["n_cols"], ref["workers"],
                                                                       ref["stragglers"]):
            # reference per-iteration math on 8 host CPU threads (tools/reference_cpu_equiv.py);
            # BASELINE.md publishes no sec/iter, so vs_baseline stays null
            out["ref_cpu_equiv_s_per_iter"] = ref["sec_per_iter_lower_bound"]
            out["speedup_vs_ref_cpu_equiv"] = ref["sec_per_iter_lower_bound"] / sec_per_iter
        bpr = out["x_message_bytes_per_step_rank0"]
        if bpr:
            out["rank0_message_rows_GBps"] = bpr / sec_per_iter / 1e9
        if out["x_distinct_bytes_rank0"]:
            out["rank0_distinct_rows_GBps"] = out["x_distinct_bytes_rank0"] / sec_per_iter / 1e9
    # convergence: iterations to the training-loss floor (100-round run, evaluated with the MFMA eval kernel)
    trainer.close()
    if not a.no_floor:
        del trainer
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
        tr2 = Trainer(make_cfg(a.floor_rounds), env)
        r2 = tr2.run()
        tr2.close()
        if env.is_master:
            tr2.cfg.fix_quirks = True  # evaluate on all partitions
            torch.cuda.synchronize() if torch.cuda.is_available() else None
            t_ev = time.perf_counter()
            ev = evaluate(tr2, r2, write=False)
            out["eval_s"] = time.perf_counter() - t_ev  # 100 betas x (train 1e6 + test 2e5 rows): MFMA GEMM + AUC
            tl = ev.training_loss
            floor = float(np.min(tl))
            thr = floor + 0.01 * abs(floor)
            it = int(np.argmax(tl <= thr))
            out["iters_to_loss_floor"] = it
            out["loss_floor"] = floor
            out["final_train_loss"] = float(tl[-1])
            out["final_test_auc"] = float(ev.auc[-1])
            out["floor_run_wallclock_s"] = float(r2.total_time)
    env.barrier()
    if env.is_master:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    env.shutdown()
    return 0


def _ref_cpu_equiv():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "reference_cpu_equiv.json")
    try:
        with open(path) as f:
            r = json.loads(f.readline())
        r.setdefault("n_rows", 1_000_000)
        return r
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    sys.exit(main())
