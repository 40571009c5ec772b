"""Headline benchmark: AGC logistic regression, synthetic 1e6 x 1e3, 8 workers, s=2, k=6.

Metric (BASELINE.json): "wall-clock sec/iter + iters-to-loss-floor, logistic regression
n_stragglers=2, 1/2/4/8 MI355X".  One *step* = one full training round of approximate
gradient coding: the master pushes beta to every worker rank (IPC mailbox over xGMI),
every logical worker computes its (s+1)-replicated gradient with the fused HIP kernel,
the master waits for the stop rule (k = num_collect arrivals or every FRC group covered),
decodes, runs the fused combine+AGD update and drains the straggler tail
(ref src/approximate_coding.py:136-207).  The problem is fixed (1e6 x 1e3, W = 8 logical
workers) and spread over N GPUs: strong scaling.  W % (s+1) != 0 for W=8, s=2, so the FRC
groups are {0,1,2},{3,4,5},{6,7} (--allow-uneven-groups extension; the reference would
refuse this config, ref src/approximate_coding.py:25-27).

Launch (ref run_approx_coding.sh:47-49 starts every rank from one mpirun command):
  python bench.py --gpus N ...        N > 1 without torchrun: relaunches itself under
                                      torch.distributed.run --nproc-per-node N (before any
                                      GPU call) and exits with its status
  torchrun --nproc-per-node N bench.py --gpus N ...   used as is; WORLD_SIZE must equal N

Reported on rank 0 as ONE JSON line:
  value / ms_per_step     timed rounds (barrier + device sync on both sides, MAX over ranks)
  host_driven_ms_per_step the same rounds driven by the host collector's real wait-for-k
                          path (HIP-event instrumented run; equals the headline path at N > 1)
  hbm_distinct_TBps       distinct X bytes rank 0 streams per round / round time
  fraction_of_rows_used_in_decode   mean over rounds of the training rows whose partitions
                          reach the decoded gradient (AGC < 1; exact codes = 1)
  iters_to_loss_floor     rounds until the AGC training loss reaches the COMMON target
                          loss_target = naive (exact, uncoded GD) 100-round loss + 1 %
  ranks                   per-rank breakdown: hosted workers, transport, kernel / put /
                          wait / decode+update microseconds (Trainer.rank_report)
  straggler_virtual       N = 1: the paper's claim under the reference's straggler model -- naive,
                          AGC with the reference's drain and AGC with the lazy drain under
                          Exp(--straggler-mean-ms) virtual delays: Σtimeset, loop wall-clock, their
                          delay floors and wall-clock to the common loss target (virtual_straggler_block)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

METRIC = "wall-clock sec/iter + iters-to-loss-floor, logistic regression n_stragglers=2, 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clock-warmup-ms", type=float, default=60.0,
                    help="untimed rounds ahead of the warmup rounds, about this long: the GPU's power management "
                         "slows the first ~20 ms of sustained gradient streaming by up to 20 %% (profiles/round3/clocks)")
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
    ap.add_argument("--delay-mode", default="exp", choices=["exp", "fixed", "none"])
    ap.add_argument("--delay-mean", type=float, default=0.5)
    ap.add_argument("--fixed-stragglers", type=int, nargs="*", default=[])
    ap.add_argument("--fixed-sleep", type=float, default=0.5)
    ap.add_argument("--delay-on", default="collector", choices=["collector", "worker"],
                    help="injected delays as virtual arrival times or physically late worker ranks")
    ap.add_argument("--slow-ranks", nargs="*", default=[], metavar="RANK:FACTOR",
                    help="physically slow GPUs: the rank runs its gradient FACTOR times per round")
    ap.add_argument("--shard", default="partition", choices=["partition", "message"],
                    help="N > 1 placement: partition shards (default here: fastest, but a physically slow "
                         "GPU delays every message with a shard on it) or whole messages round-robin "
                         "(the reference topology and the training default: a slow GPU erases its own workers)")
    ap.add_argument("--no-integrity", action="store_true", help="untagged IPC messages (A/B of the tag cost)")
    ap.add_argument("--no-floor", action="store_true", help="skip the 100-round convergence runs")
    ap.add_argument("--no-breakdown", action="store_true", help="skip the instrumented host-driven run")
    ap.add_argument("--floor-rounds", type=int, default=100)
    ap.add_argument("--tasks", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--transport", default="auto", choices=["auto", "ipc", "rccl", "loopback"])
    ap.add_argument("--round-timeout", type=float, default=30.0,
                    help="bounds any hang (a round takes ms; a gone rank is found within a few of these)")
    ap.add_argument("--subrun-timeout", type=float, default=20.0,
                    help="round timeout of every run after the headline (a failed sub-run is found within a few of "
                         "them and recorded in subrun_failures; the headline keeps --round-timeout)")
    ap.add_argument("--device-loop", default="auto", choices=["auto", "graph", "stream", "off"])
    ap.add_argument("--tie-break", default="permute", choices=["permute", "worker"])
    ap.add_argument("--preflight", type=int, default=1000,
                    help="N > 1: put -> flag round trips per worker/master pair before the timed rounds (0: off)")
    ap.add_argument("--selfcheck", type=int, default=30,
                    help="N > 1: integrity-tagged rounds on the headline's executor before timing (first_contact)")
    ap.add_argument("--selfcheck-timeout", type=float, default=10.0,
                    help="first_contact: round timeout of the check run (worker beta waits: 2.5x + 5 s)")
    ap.add_argument("--no-single-ref", dest="single_ref", action="store_false",
                    help="N > 1: skip rank 0's single-GPU run of the same config (the scaling denominator)")
    ap.add_argument("--share-partitions", action="store_true",
                    help="co-located workers stream each distinct partition once (not the headline)")
    ap.add_argument("--drain", default=None, choices=["all", "carry", "lazy"],
                    help="straggler tail (default: the scheme's reference behaviour; AGC drains)")
    ap.add_argument("--late-ms", type=float, default=5.0,
                    help="N > 1 straggler sub-run: the last rank is physically late by this much every round")
    ap.add_argument("--straggler-steps", type=int, default=40, help="timed rounds of each straggler sub-run")
    ap.add_argument("--straggler-mean-ms", type=float, default=5.0,
                    help="N = 1 straggler block: mean of the Exp virtual delays (the reference's 0.5 s scaled "
                         "down 100x; every delay floor scales linearly in it)")
    ap.add_argument("--slab-mode", type=int, default=None, help=argparse.SUPPRESS)  # A/B of the slab reduction form
    ap.add_argument("--mfma-stream", type=int, default=None, help=argparse.SUPPRESS)  # A/B of the bf16 MFMA stream
    ap.add_argument("--no-straggler", action="store_true",
                    help="skip the straggler runs (N = 1: the virtual-delay block; N > 1: the reference-topology "
                         "and physically-late-rank sub-runs)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch(gpus: int, argv, script: str = None) -> int:
    """Start N ranks of this script under torch.distributed.run as a CHILD process (never exec:
    nothing here has touched the GPU, and the children own it) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", script or os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if int(env.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:  # erasurehead_amd/__init__.py: per-peer p2p streams
        env["GPU_MAX_HW_QUEUES"] = "16"
    print(f"[bench] launching {gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return relaunch(a.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"error: --gpus {a.gpus} but WORLD_SIZE={world}: the measurement would not be the one "
              f"labelled; launch with --nproc-per-node {a.gpus} or drop torchrun", file=sys.stderr)
        return 2

    import torch

    from erasurehead_amd.cli import parse_slow_ranks
    from erasurehead_amd.codes.schemes import Arrival
    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.engine import Trainer, evaluate
    from erasurehead_amd.parallel.dist import init_distributed
    from erasurehead_amd.parallel.transport import TransportError

    env = init_distributed("auto")
    if a.slab_mode is not None and torch.cuda.is_available():
        from erasurehead_amd._ext import native

        native().set_slab_reduce_mode(a.slab_mode)
    if a.mfma_stream is not None and torch.cuda.is_available():
        from erasurehead_amd._ext import native

        native().set_mfma_stream(int(a.mfma_stream))

    def make_cfg(rounds: int, naive: bool = a.naive, ver: int = a.coded_ver, **kw) -> RunConfig:
        opts = dict(add_delay=a.add_delay, num_itrs=rounds, precision=a.precision, data="synthetic", data_seed=1234,
                    seed=0, allow_uneven_groups=True, verbose=False, tasks=a.tasks, transport=a.transport,
                    round_timeout=a.round_timeout, share_partitions=a.share_partitions, device_loop=a.device_loop,
                    tie_break=a.tie_break, shard=a.shard, delay_mode=a.delay_mode, delay_mean=a.delay_mean,
                    fixed_stragglers=a.fixed_stragglers, fixed_sleep=a.fixed_sleep, delay_on=a.delay_on,
                    slow_ranks=parse_slow_ranks(a.slow_ranks), integrity=not a.no_integrity, drain=a.drain)
        opts.update(kw)
        add_delay = opts.pop("add_delay")
        return RunConfig(a.workers + 1, a.n_rows, a.n_cols, "/tmp/erasurehead_bench/", 0, "synthetic",
                         0 if naive else 1, a.stragglers, 0, ver, a.num_collect, add_delay, a.update_rule,
                         **opts)

    def free(tr):
        tr.close()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    # ---- 1. headline: timed rounds --------------------------------------------------------------
    # Untimed clock warm-up: rounds of the same work ahead of the W warmup rounds, no idle gap before the
    # timed ones.  The first ~20 ms of sustained streaming after setup run up to 20 % slow while the
    # power controller settles (per-call kernel trace, profiles/round3/clocks); like the reference's
    # discarded warm-up gradient (ref src/naive.py:39-44), nothing of it is timed or reported as a step.
    esize = {"fp64": 8, "fp32": 4, "bf16": 2}[a.precision]
    est_round_ms = max(0.02, a.n_rows * a.n_cols * esize / world / 6e9)  # distinct rows at ~6 TB/s
    clock_rounds = min(1000, int(np.ceil(a.clock_warmup_ms / est_round_ms))) if a.clock_warmup_ms > 0 else 0
    w0 = clock_rounds + a.warmup  # first timed round
    # N > 1: the job checks the exact path its headline will take before anything is timed (preflight
    # round trips per pair, then a bounded integrity-tagged run), stepping down arbiter -> native pump ->
    # RCCL p2p on any failure, in this process (first_contact)
    # test hook ERASUREHEAD_SABOTAGE=subrun:<spec>: ERASUREHEAD_SABOTAGE=<spec> from the first run after the
    # headline on (the containment of the sub-runs below)
    late_sabotage = None
    if os.environ.get("ERASUREHEAD_SABOTAGE", "").startswith("subrun:"):
        late_sabotage = os.environ.pop("ERASUREHEAD_SABOTAGE").split(":", 1)[1]
    contact = first_contact(a, make_cfg, env, free, Trainer, TransportError) if env.world > 1 else None
    t_setup = time.perf_counter()
    trainer = Trainer(make_cfg(w0 + a.steps), env)
    setup_s = time.perf_counter() - t_setup
    res, why = trainer.run_contained(timed_start=w0)
    while why is not None:  # the headline itself failed after a clean first contact: one rung down and again
        step = step_down(a, env, trainer, why)  # (raises once nothing is left below)
        if env.is_master:
            print(f"[bench] WARNING: headline run failed ({why}); rebuilding: {step}", file=sys.stderr, flush=True)
        free(trainer)
        contact = dict(contact or {})
        contact.setdefault("headline_failures", []).append({"failure": why, "step_down": step})
        trainer = Trainer(make_cfg(w0 + a.steps), env)
        res, why = trainer.run_contained(timed_start=w0)
    mine = res.timed_seconds if env.is_master else trainer.worker_timed_seconds
    timed = env.allreduce_max(mine)
    sch = trainer.scheme
    out = {}
    if env.is_master:
        sec_per_iter = timed / a.steps
        ts = res.timeset[w0:]
        lt = res.loop_time[w0:]
        n_gpu_dev = torch.cuda.device_count() if torch.cuda.is_available() else 0
        out = {
            "metric": METRIC,
            "value": sec_per_iter,
            "unit": "s/iter",
            "n_gpus": env.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "clock_warmup_rounds": clock_rounds,
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
                "parallelism": f"ps-master + {a.workers} logical workers on {env.world} GPU rank(s) (dp{env.world})",
                "transport": trainer.transport,
                "tie_break": a.tie_break,
                # replica messages: every replica's own arithmetic ("separate", the headline) or one
                # gradient per distinct partition encoded into the replicas ("encoded": --share-partitions)
                "replicas": trainer.replica_policy,
            },
            "time_to_decode_ms_median": float(1e3 * np.median(ts)),
            "loop_ms_median": float(1e3 * np.median(lt)),
            # X bytes rank 0's messages read per round (replicas counted each time) and the distinct
            # partitions behind them; co-located replicas share those reads (LDS-staged bundles)
            "x_message_bytes_per_step_rank0": int(getattr(trainer.plan, "bytes_per_round", 0)) or None,
            "x_distinct_bytes_rank0": int(getattr(trainer.plan, "distinct_bytes", 0)) or None,
            "setup_s": setup_s,
            "phases_us": {k: round(v["mean_us"], 1) for k, v in res.phases.items()},
            # rank -> the (worker, partition) shards it computes ("w3" = worker 3's whole message)
            "placement": {str(r): [f"w{u.worker}" + (f":p{u.segments[0][0]}" if u.n_shards > 1 else "")
                                   + (":part1" if u.part else "")
                                   for u, o in zip(trainer.shards, trainer.owner) if o == r]
                          for r in range(env.world)},
            "shard": trainer.shard_mode,
            # what a physically slow GPU does to the stop rule under this placement (parallel/placement.py)
            "straggler_tolerance": ("per worker rank: a slow GPU erases only its own workers' messages"
                                    if trainer.shard_mode == "message" or env.world == 1 else
                                    "none across ranks: every replica of a partition is on one rank, a slow GPU "
                                    "delays every message with a shard there (virtual delays unaffected)"),
        }
        if a.delay_on == "worker" or a.slow_ranks:
            out["config"]["delay_on"] = a.delay_on
            out["config"]["slow_ranks"] = parse_slow_ranks(a.slow_ranks)
        # what the first multi-GPU contact will run, and why (first_contact; README "First contact")
        out["release_form"] = trainer.release_form
        out["release_reason"] = trainer.release_reason
        out["device_map"] = {str(r): b for r, b in enumerate(trainer.device_map)}
        if contact is not None:
            out["first_contact"] = contact
            if contact.get("preflight") is not None:
                out["peer_preflight"] = contact["preflight"]
            if contact.get("preflight_failure") is not None:
                out["peer_preflight_failure"] = contact["preflight_failure"]
                out["fallback_preflight"] = contact.get("fallback_preflight")
                out["fallback_mechanism"] = ("loopback: device copies through IPC staging rings + shared counters "
                                             "(the mailbox's mechanism), checked by fallback_preflight before timing"
                                             if trainer.transport == "loopback" else "RCCL p2p (ncclSend / ncclRecv)")
        if n_gpu_dev and env.world > n_gpu_dev:
            out["config"]["ranks_per_gpu"] = env.world / n_gpu_dev  # rehearsal: ranks time-share GPUs
        out["config"]["round_loop"] = {"graph": "device-driven, hipGraph", "stream": "device-driven",
                                          "arbiter": "device-driven (arbiter kernel polls the workers)"}.get(
            trainer.device_loop, "host-driven (native pump)" if trainer.native_loop else "host-driven (python)")
        out["config"]["round_loop_reason"] = trainer.loop_reason
        out["config"]["release_form"] = trainer.release_form
        if a.share_partitions:
            out["config"]["share_partitions"] = True
        ref = _ref_cpu_equiv()
        if ref and (a.n_rows, a.n_cols, a.workers, a.stragglers) == (ref["n_rows"], ref["n_cols"], ref["workers"],
                                                                       ref["stragglers"]):
            # reference per-iteration math on 8 host CPU threads (tools/reference_cpu_equiv.py);
            # BASELINE.md publishes no sec/iter, so vs_baseline stays null
            out["ref_cpu_equiv_s_per_iter"] = ref["sec_per_iter_lower_bound"]
            out["speedup_vs_ref_cpu_equiv"] = ref["sec_per_iter_lower_bound"] / sec_per_iter
        if out["x_distinct_bytes_rank0"]:
            out["hbm_distinct_TBps"] = out["x_distinct_bytes_rank0"] / sec_per_iter / 1e12
        out["fraction_of_rows_used_in_decode"] = decode_row_fraction(sch, res.arrivals[w0:], Arrival)
    reports = env.gather_objects(trainer.rank_report())
    trainer_shard = trainer.shard_mode
    kernel_iso = None
    for r in range(env.world):  # one rank at a time: ranks may share a GPU (rehearsals)
        if r == env.rank and trainer.local_msgs:
            kernel_iso = trainer.time_local_grad()
        env.barrier()
    kernel_iso = env.gather_objects(kernel_iso)
    free(trainer)
    del trainer, res

    # Every run after the headline is contained (Trainer.run_contained: one verdict on every rank): a failure
    # is recorded in `subrun_failures` and the collective runs after it are skipped on every rank alike, so a
    # sub-run that breaks on new hardware never costs the headline line.
    failures = {}
    a.round_timeout = min(a.round_timeout, a.subrun_timeout)  # make_cfg reads it at every call
    if late_sabotage:
        os.environ["ERASUREHEAD_SABOTAGE"] = late_sabotage

    class _SubRunFailed(Exception):
        pass

    def contained(name: str, tr_, **kw):
        res_, why_ = tr_.run_contained(**kw)
        if why_:
            failures[name] = why_
            if env.is_master:
                print(f"[bench] WARNING: {name} run failed ({why_}); the later sub-runs are skipped", file=sys.stderr,
                      flush=True)
        return res_, why_ is None

    # ---- 2. the same rounds host-driven, instrumented: real wait-for-k path + per-rank breakdown -----
    if not a.no_breakdown:
        headline = reports
        # N > 1: device records too, for the worker half of the round chain (worker_round_start_latency)
        tr = Trainer(make_cfg(w0 + a.steps, device_loop="off", instrument=True, device_records=env.world > 1), env)
        r, ok = contained("breakdown", tr, timed_start=w0)
        if ok:
            t = env.allreduce_max(r.timed_seconds if env.is_master else tr.worker_timed_seconds)
            reports = env.gather_objects(tr.rank_report())
            if env.world > 1:
                lat = worker_round_start_latency(env.gather_objects(tr.device_records), w0)
                if env.is_master:
                    for rep in reports:
                        if rep["rank"] in lat:
                            rep["beta_to_round_start_us"] = lat[rep["rank"]]
            if env.is_master:  # the headline run's device-side master ticks (arbiter: poll / update / release)
                for rep, h in zip(reports, headline):
                    rep.update({f"headline_{k}": v for k, v in h.items()
                                if k.startswith("arbiter_") or k in ("device_round_us", "round_loop")})
            if env.is_master:
                out["host_driven_ms_per_step"] = 1e3 * t / a.steps
                out["host_driven_instrumented"] = True
        free(tr)
        del tr, r

    if env.is_master:
        for rep, k in zip(reports, kernel_iso):
            if k is not None:
                rep["kernel_us_isolated"] = round(k, 1)
        out["ranks"] = reports

    # ---- 2b. N > 1: the reference topology and a physically late rank -------------------------------
    # The headline places partition shards (bandwidth: each GPU streams its partitions once), whose
    # replicas of a partition share one rank, so a slow GPU stalls every message with a shard there.
    # The reference runs one worker per process (ref run_approx_coding.sh:47-49,
    # src/approximate_coding.py:47-53): message placement.  On it, one rank is made late by --late-ms
    # every round (a device spin after its gradient, before its put: ref src/naive.py:141-148), and
    # AGC with a lazy drain (no wait for the tail, stale rounds skipped on the late rank) is timed
    # against naive (which must wait for every worker), each with and without the straggler.
    if env.world > 1 and not a.no_straggler and not failures:
        S, W = a.straggler_steps, a.workers
        late_rank = env.world - 1
        late_workers = [w for w in range(W) if w % env.world == late_rank]  # parallel/placement.py place_spread
        keys = ("rank", "workers", "round_loop", "kernel_us", "wait_k_us", "beta_wait_us", "stale_rounds_skipped",
                "stale_arrivals", "stale_skipped_virtual", "arbiter_poll_us")

        def sub_run(naive: bool, late: bool, warm: int = a.warmup, steps: int = S, **kw):
            extra = dict(shard="message", drain=kw.pop("drain", None), **kw)
            if late:
                extra.update(add_delay=1, delay_mode="fixed", delay_on="worker", fixed_sleep=a.late_ms / 1e3,
                             fixed_stragglers=[w + 1 for w in late_workers], force_delay=True)
            else:
                extra.update(add_delay=0)
            tr_s = Trainer(make_cfg(warm + steps, naive=naive, **extra), env)
            r_s, ok_s = contained(f"{'naive' if naive else 'scheme'}_{'late' if late else 'on_time'}_{extra['shard']}",
                                  tr_s, timed_start=warm)
            if not ok_s:
                free(tr_s)
                raise _SubRunFailed()
            t_s = env.allreduce_max(r_s.timed_seconds if env.is_master else tr_s.worker_timed_seconds)
            reps = env.gather_objects(tr_s.rank_report())
            rec = None
            if env.is_master:
                lt = np.asarray(r_s.loop_time[warm:])
                rec = {"ms_per_step": 1e3 * t_s / steps, "steps": steps, "round_ms_mean": float(1e3 * np.mean(lt)),
                       "round_ms_median": float(1e3 * np.median(lt)), "drain": tr_s.drain_mode,
                       "ranks": [{k: x[k] for k in keys if k in x} for x in reps]}
            free(tr_s)
            return rec

        try:
            topo = sub_run(a.naive, False, warm=w0, steps=a.steps)  # the headline's warm-up and step count
            straggler = {
                "late_rank": late_rank, "late_workers": late_workers, "late_ms": a.late_ms, "placement": "message",
                "steps": S, "agc_lazy": sub_run(False, True, drain="lazy"),
                "agc_lazy_no_straggler": sub_run(False, False, drain="lazy"),
                "naive": sub_run(True, True), "naive_no_straggler": sub_run(True, False)}
        except _SubRunFailed:
            topo = straggler = None
        except Exception as e:  # noqa: BLE001 -- e.g. a transport that failed to build: its peers fail with it
            failures["straggler_setup"] = f"rank {env.rank}: {type(e).__name__}: {e}"
            topo = straggler = None
        # one view of what failed on every rank (a construction error is raised on each side of its pair)
        seen = env.gather_objects(dict(failures))  # (the list on rank 0, None elsewhere)
        merged = env.broadcast_object({k: v for f in seen for k, v in f.items()} if env.is_master else None, 0)
        failures.update(merged)
        if failures:
            topo = straggler = None
        if env.is_master and topo is not None and straggler is not None:
            out["message_placement_ms_per_step"] = topo["ms_per_step"]
            out["message_placement"] = topo
            # the straggler-tolerant co-headline: the reference topology (one worker's s+1 partitions per
            # rank, ref run_approx_coding.sh:47-49, src/approximate_coding.py:47-53), where a slow GPU
            # erases only its own workers -- `value` uses the bandwidth placement (--shard)
            out["value_tolerant"] = topo["ms_per_step"] / 1e3
            out["value_tolerant_placement"] = "message"
            for name in ("agc_lazy", "naive"):  # the master's round period: late vs on time
                straggler[f"{name}_round_slowdown"] = (straggler[name]["round_ms_mean"]
                                                      / straggler[f"{name}_no_straggler"]["round_ms_mean"])
            straggler["definition"] = ("round_ms_*: mean master round (beta(i) out -> beta(i+1) out) over the timed "
                                       "rounds; ms_per_step: fenced wall-clock / steps (includes the late rank's "
                                       "last in-flight round)")
            out["straggler"] = straggler

    # ---- 2c. N > 1: the same problem on rank 0's GPU alone, in this job (the scaling denominator) --------
    if env.world > 1 and a.single_ref and not failures:
        single = single_gpu_reference(a, make_cfg, env, free, Trainer, clock_rounds)
        if env.is_master and isinstance(single, str):  # rank 0's solo run failed: recorded, not collective
            out["single_gpu_reference_failure"] = single
        elif env.is_master:
            out["single_gpu_s_per_iter"] = single
            out["single_gpu_definition"] = ("the headline config on rank 0's GPU alone (world 1, every message "
                                            "local), timed in this job right after the N-rank runs")
            out["scaling_efficiency"] = single / (env.world * out["value"])
            if "value_tolerant" in out:
                out["scaling_efficiency_tolerant"] = single / (env.world * out["value_tolerant"])
            out["scaling_placements"] = {"value": f"{trainer_shard} (--shard)",
                                         "value_tolerant": "message (the reference topology)"}

    # ---- 3. convergence: naive (exact GD) sets the common loss target, then the scheme -------------
    if not a.no_floor and not failures:
        curves = {}
        for name, naive in (("naive", True), ("scheme", a.naive)):
            if name == "scheme" and a.naive:
                curves["scheme"] = curves["naive"]
                continue
            tr2 = Trainer(make_cfg(a.floor_rounds, naive=naive), env)
            r2, ok2 = contained(f"floor_{name}", tr2)
            free(tr2)
            if not ok2:
                break
            if env.is_master:
                tr2.cfg.fix_quirks = True  # evaluate on every partition
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                t_ev = time.perf_counter()
                ev = evaluate(tr2, r2, write=False)
                curves[name] = (ev, r2, time.perf_counter() - t_ev)
            del tr2, r2
        if env.is_master and "scheme" in curves:
            ev_n, r_n, _ = curves["naive"]
            ev, r2, eval_s = curves["scheme"]
            target = float(ev_n.training_loss[-1]) * 1.01
            tl = ev.training_loss
            hit = np.nonzero(tl <= target)[0]
            hit_n = np.nonzero(ev_n.training_loss <= target)[0]
            out["eval_s"] = eval_s  # 100 betas x (train 1e6 + test 2e5 rows): MFMA GEMM + AUC
            out["loss_target"] = target
            out["loss_target_definition"] = "naive (exact uncoded GD) training loss after %d rounds + 1%%" % (
                a.floor_rounds)
            out["iters_to_loss_floor"] = int(hit[0]) + 1 if hit.size else None
            out["naive_iters_to_loss_floor"] = int(hit_n[0]) + 1 if hit_n.size else None
            out["seconds_to_loss_floor"] = float(np.sum(r2.loop_time[: hit[0] + 1])) if hit.size else None
            out["final_train_loss"] = float(tl[-1])
            out["naive_final_train_loss"] = float(ev_n.training_loss[-1])
            out["final_test_auc"] = float(ev.auc[-1])
            out["floor_run_wallclock_s"] = float(r2.total_time)

    # ---- 4. N = 1: the paper's claim under the reference straggler model ----------------------------
    # The reference's delay model (Exp per worker per round, seeded by the round index, after compute
    # and before the send: ref src/approximate_coding.py:198-205) with its mean scaled from 0.5 s to
    # --straggler-mean-ms, applied as virtual arrival times by the native collector (the GPU never
    # sleeps).  naive (waits for every worker), AGC with the reference's Waitall drain (ref :182-183)
    # and AGC with the lazy drain (no wait for the tail, a worker still busy skips the stale round: the
    # replacement of the reference's send Cancel, ref src/coded.py:178-180) run one after another, each
    # for --floor-rounds rounds, and are compared on wall-clock to the common loss target.
    if env.world == 1 and not a.no_straggler and not a.no_floor and not failures:
        try:  # one process: nothing collective inside, so a failure here is this rank's alone
            blk = virtual_straggler_block(a, make_cfg, env, free, Trainer, evaluate,
                                          out.get("ms_per_step", 0.0) / 1e3 if env.is_master else 0.0)
            out["straggler_virtual"] = blk
        except Exception as e:  # noqa: BLE001 -- recorded in the JSON, the headline line still prints
            failures["straggler_virtual"] = f"{type(e).__name__}: {e}"
            print(f"[bench] WARNING: straggler_virtual failed ({e})", file=sys.stderr, flush=True)
    env.barrier()
    if env.is_master and failures:
        out["subrun_failures"] = failures
    if env.is_master:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if failures and env.world > 1:
        # a contained failure can leave receives posted on the process group that nothing will match
        # (gloo cannot cancel them), and its teardown would wait on them: the line is out, leave now
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    env.shutdown()
    return 0


def worker_round_start_latency(records, first: int) -> dict:
    """The worker half of the round chain, per worker rank: median over rounds >= ``first`` of the time
    from the master's beta(i) put (the stamp right after its put kernels) to the worker's round i start on
    its own stream (the stamp right behind its beta wait), both GPU clocks mapped to the host clock
    (Trainer device_records; accurate to the clocks' calibration, a few microseconds).  {} on workers."""
    if not records or records[0] is None or records[0].get("clock") is None:
        return {}
    m = records[0]
    bp = np.asarray(m["beta_put"], dtype=np.float64)
    _, k0, t0, hz0 = m["clock"]
    out = {}
    for x in records[1:]:
        if not x or x.get("clock") is None:
            continue
        rows = np.asarray(x["rounds"], dtype=np.float64)
        _, k1, t1, hz1 = x["clock"]
        lat = [(t1 + (rows[i][9] - k1) / hz1) - (t0 + (bp[i][1] - k0) / hz0)
               for i in range(first, min(len(bp), len(rows))) if bp[i][1] >= 0 and rows[i][9] >= 0]
        if lat:
            out[int(x["rank"])] = round(1e6 * float(np.median(lat)), 2)
    return out


def single_gpu_reference(a, make_cfg, env, free, Trainer, clock_rounds: int):
    """N > 1: rank 0 runs the headline configuration by itself (a world-1 Trainer on its own GPU: every
    message local, the single-process device loop) for --steps timed rounds after the same warm-up,
    while the other ranks wait at a barrier.  Returns its s/iter on rank 0 (None elsewhere): the
    denominator of the job's own scaling efficiencies, measured on the same node in the same job (a failed
    solo run returns its reason instead)."""
    from erasurehead_amd.parallel.dist import DistEnv

    env.barrier()
    sec = None
    if env.is_master:
        solo = DistEnv(rank=0, world=1, local_rank=env.local_rank, device=env.device, backend="none")
        w0 = clock_rounds + a.warmup
        try:  # rank 0 alone: whatever fails here must still reach the barrier the others wait at
            tr = Trainer(make_cfg(w0 + a.steps), solo)
            r, why = tr.run_contained(timed_start=w0)  # world 1: a verdict of this rank alone
            sec = r.timed_seconds / a.steps if why is None else why
            free(tr)
            del tr, r
        except Exception as e:  # noqa: BLE001 -- recorded as single_gpu_reference_failure
            sec = f"{type(e).__name__}: {e}"
    env.barrier()
    return sec


def step_down(a, env, trainer, why: str) -> str:
    """One rung down the N > 1 executor ladder after ``trainer``'s run failed collectively (every rank
    calls it with the same trainer state): arbiter -> native pump on the same transport (for the rest
    of the job: ERASUREHEAD_DEVICE_MASTER=off), IPC mailbox -> RCCL p2p (loopback where ranks share a
    GPU, which RCCL refuses).  Raises when nothing is left below."""
    if trainer.loop == "arbiter":
        os.environ["ERASUREHEAD_DEVICE_MASTER"] = "off"
        return "arbiter -> native pump (ERASUREHEAD_DEVICE_MASTER=off for the rest of the job)"
    if trainer.transport == "ipc" and a.transport != "ipc" and not os.environ.get("ERASUREHEAD_NO_FALLBACK"):
        a.transport = "rccl" if env.backend == "nccl" else "loopback"
        return f"ipc -> {a.transport} (native pump)"
    raise RuntimeError(f"first contact: the {trainer.loop} loop over {trainer.transport} failed and no path is "
                       f"left below it: {why}")


def first_contact(a, make_cfg, env, free, Trainer, TransportError) -> dict:
    """N > 1, before the headline trainer exists: check the path it will take, in this process.

    1. --preflight put -> flag round trips per master/worker pair over the IPC mailbox (device clock,
       payload checked both ways; IpcTransport.preflight), plus RCCL p2p round trips for comparison.
    2. --selfcheck rounds of the real problem on the executor the headline will select (the arbiter
       where ranks own their GPUs), every message and beta integrity-tagged, every wait bounded by
       --selfcheck-timeout (Trainer.run_contained: a failure on any rank becomes one verdict that
       every rank holds, with the job still collectively consistent).
    Any failure steps one rung down (step_down) and checks again: arbiter -> native pump -> RCCL p2p.
    Nothing re-execs.  Returns the record bench.py reports as ``first_contact``: the device map and
    release form, the preflight, and one entry per rung tried (loop, transport, verdict, seconds).
    Test hook ERASUREHEAD_SABOTAGE=firstcontact:<spec>: ERASUREHEAD_SABOTAGE=<spec> for the first rung only."""
    rec = {"rounds": a.selfcheck, "round_timeout_s": a.selfcheck_timeout, "ladder": []}
    once = None
    if os.environ.get("ERASUREHEAD_SABOTAGE", "").startswith("firstcontact:"):
        once = os.environ.pop("ERASUREHEAD_SABOTAGE").split(":", 1)[1]
    while True:
        if once:
            os.environ["ERASUREHEAD_SABOTAGE"] = once
        tr = Trainer(make_cfg(max(1, a.selfcheck), round_timeout=a.selfcheck_timeout, integrity=True), env)
        rec.setdefault("device_map", {str(r): b for r, b in enumerate(tr.device_map)})
        rec.setdefault("release_form", tr.release_form)
        rec.setdefault("release_reason", tr.release_reason)
        if tr.transport == "ipc" and a.preflight > 0 and "preflight" not in rec:
            try:
                rec["preflight"] = tr.preflight(a.preflight)
            except TransportError as e:
                # every rank raised the same verdict: the mailbox lost a payload or a signal
                rec["preflight"], rec["preflight_failure"] = None, str(e)
                if a.transport == "ipc" or os.environ.get("ERASUREHEAD_NO_FALLBACK"):
                    raise
                a.transport = "rccl" if env.backend == "nccl" else "loopback"
                if env.is_master:
                    print(f"[bench] WARNING: {e}; rebuilding on {a.transport}", file=sys.stderr, flush=True)
                rec["ladder"].append({"transport": "ipc", "ok": False, "failure": str(e), "stage": "preflight",
                                      "step_down": f"ipc -> {a.transport}"})
                free(tr)
                continue
        if tr.transport != "ipc" and "fallback_preflight" not in rec and hasattr(tr.tx, "preflight") \
                and rec.get("preflight_failure"):
            # loopback runs over the same IPC mappings as the mailbox whose check failed: it proves itself
            rec["fallback_preflight"] = tr.tx.preflight(min(200, max(1, a.preflight)))
        tr.native_loop  # noqa: B018 -- selects tr.loop / tr.loop_reason from this run's facts
        step = {"transport": tr.transport, "round_loop": tr.loop, "reason": tr.loop_reason,
                "release_form": tr.release_form}
        t0 = time.perf_counter()
        _, why = tr.run_contained()
        step.update(ok=why is None, seconds=round(time.perf_counter() - t0, 3),
                    round_loop_ran=tr.device_loop or ("native pump" if tr.native_loop else "python"))
        if once:
            os.environ.pop("ERASUREHEAD_SABOTAGE", None)
            once = None
        if why is not None:
            step["failure"] = why
            step["step_down"] = step_down(a, env, tr, why)
            if env.is_master:
                print(f"[bench] WARNING: first contact failed on {tr.loop} over {tr.transport}: {why}; "
                      f"{step['step_down']}", file=sys.stderr, flush=True)
        rec["ladder"].append(step)
        free(tr)
        if why is None:
            rec["round_loop"], rec["transport"] = step["round_loop"], step["transport"]
            return rec


STRAGGLER_RUNS = (("naive", True, None), ("agc_drain", False, "all"), ("agc_lazy", False, "lazy"))


def virtual_straggler_block(a, make_cfg, env, free, Trainer, evaluate, compute_s: float) -> dict:
    """Run naive / AGC drain / AGC lazy under Exp(--straggler-mean-ms) virtual delays (section 4 of
    main) and summarise them (straggler_summary); None on ranks other than the master."""
    from erasurehead_amd.utils.delay import schedule_floors

    mean = a.straggler_mean_ms / 1e3
    R, W = a.floor_rounds, a.workers
    delays = np.stack([np.random.RandomState(i).exponential(mean, W) for i in range(R)])  # ref src/naive.py:146
    runs = {}
    for name, naive, drain in STRAGGLER_RUNS:
        tr = Trainer(make_cfg(R, naive=naive, ver=3, add_delay=1, delay_mode="exp", delay_mean=mean,
                              delay_on="collector", drain=drain), env)
        r = tr.run()
        free(tr)
        if not env.is_master:
            continue
        groups = list(tr.scheme.group_of)
        rule, k = ("all", W) if naive else ("frc", a.num_collect)
        fl_dec, fl_loop = schedule_floors(delays, rule, k, groups, drain=tr.drain_mode)
        _, model_loop = schedule_floors(delays, rule, k, groups, drain=tr.drain_mode, compute=compute_s)
        tr.cfg.fix_quirks = True  # training loss over every partition
        ev = evaluate(tr, r, write=False)
        runs[name] = {
            "drain": tr.drain_mode,
            "round_loop": tr.device_loop or ("native pump" if tr.native_loop else "python"),
            "timeset": [float(x) for x in r.timeset], "loop_time": [float(x) for x in r.loop_time],
            "train_loss": [float(x) for x in ev.training_loss], "final_test_auc": float(ev.auc[-1]),
            "floor_timeset_s": fl_dec, "floor_loop_s": fl_loop, "model_loop_s": model_loop,
            "run_wallclock_s": float(r.total_time),
            "stale_skipped": int(tr.rank_stats.get("stale_skipped_virtual", 0) or 0),
            "used_workers_per_round": float(np.mean([(np.asarray(x) >= 0).sum() for x in r.worker_timeset])),
        }
        del tr, r
    return straggler_summary(runs, R, mean) if env.is_master else None


def straggler_summary(runs: dict, rounds: int, mean_s: float) -> dict:
    """The straggler block's JSON: per run Σtimeset, loop wall-clock, their zero-compute delay floors,
    overheads, iterations / Σtimeset / wall-clock to the common target (naive's final training loss
    + 1 %), and the headline comparison: AGC-lazy wall-clock to target against naive's."""
    target = float(runs["naive"]["train_loss"][-1]) * 1.01
    out = {"delay_model": f"Exp(mean {1e3 * mean_s:g} ms) per worker per round, seed = round (the reference's "
                          f"0.5 s mean scaled down; virtual arrival times on the collector's clock)",
           "delay_mean_s": mean_s, "rounds": rounds, "loss_target": target,
           "loss_target_definition": "naive (exact uncoded GD) training loss after %d rounds + 1%%" % rounds,
           "floor_definition": "zero-compute replay of the same delays under the run's stop rule and drain "
                               "(utils/delay.schedule_floors); model_loop_s adds the headline round time as "
                               "every worker's compute"}
    for name, r in runs.items():
        tl = np.asarray(r["train_loss"])
        hit = np.nonzero(tl <= target)[0]
        cum_ts, cum_lp = np.cumsum(r["timeset"]), np.cumsum(r["loop_time"])
        sum_ts, sum_lp = float(cum_ts[-1]), float(cum_lp[-1])
        out[name] = {
            "drain": r["drain"], "round_loop": r["round_loop"],
            "sum_timeset_s": sum_ts, "loop_wallclock_s": sum_lp, "run_wallclock_s": r["run_wallclock_s"],
            "floor_timeset_s": r["floor_timeset_s"], "floor_loop_s": r["floor_loop_s"],
            "model_loop_s": r["model_loop_s"],
            "overhead_ms_per_round": 1e3 * (sum_ts - r["floor_timeset_s"]) / rounds,
            "loop_overhead_ms_per_round": 1e3 * (sum_lp - r["floor_loop_s"]) / rounds,
            "iters_to_target": int(hit[0]) + 1 if hit.size else None,
            "timeset_s_to_target": float(cum_ts[hit[0]]) if hit.size else None,
            "wallclock_s_to_target": float(cum_lp[hit[0]]) if hit.size else None,
            "final_train_loss": float(tl[-1]), "final_test_auc": r["final_test_auc"],
            "stale_skipped": r["stale_skipped"], "used_workers_per_round": r["used_workers_per_round"],
        }
    base = out["naive"]["wallclock_s_to_target"]
    for name in runs:
        w = out[name]["wallclock_s_to_target"]
        out[name]["speedup_to_target_vs_naive"] = base / w if base and w else None
    lazy = out.get("agc_lazy", {}).get("wallclock_s_to_target")
    out["agc_lazy_beats_naive_to_target"] = bool(lazy is not None and base is not None and lazy < base)
    return out


def decode_row_fraction(scheme, arrivals_log, Arrival) -> float:
    """Mean over rounds of the fraction of partitions (= of training rows: equal-sized partitions)
    that reach the decoded gradient.  AGC covers fewer groups than it has (ref
    src/approximate_coding.py:144-158); exact codes always cover everything."""
    seg = {(m.worker, m.part): [p for p, _ in m.segments] for m in scheme.messages}
    n = scheme.n_partition_files
    fr = []
    for arr in arrivals_log:
        used = scheme.decode([Arrival(*x) for x in arr])
        parts = {p for key in used for p in seg[key]}
        fr.append(len(parts) / n)
    return float(np.mean(fr)) if fr else None


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
