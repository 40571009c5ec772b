"""The generic straggler-tolerant training engine (L4), one loop for every scheme.

Reference skeleton (ref src/naive.py:11-211, repeated in all seven engine files):
load shard -> warm-up gradient -> pre-post receives -> Barrier -> per round {master:
Isend beta to all, Waitany until the stop rule, decode, GD/AGD update, record times;
worker: Wait beta, gradient, optional delay, Isend g} -> Barrier -> master evaluates
every stored beta and writes results/*.dat.

MI355X design:
  * one process per GPU; logical workers are placed on ranks (parallel/placement.py) and
    each rank computes ALL its workers' messages with one fused kernel launch per round
    (ops/grad.py), reading its resident partitions from HBM exactly once;
  * rank 0 is also the master: local messages are probed with a HIP event behind the
    gradient kernel, remote messages with a HIP event behind the RCCL receive on the
    per-peer stream; the native collector decides arrival order / the stop rule with the
    GIL released (parallel/collector.py);
  * decode coefficients are solved on the host in fp64 (codes/), then one
    ``combine_update`` launch forms g and updates beta/u/betaset/worker-beta on the GPU;
  * worker ranks never block their host: receive, kernel and sends are stream-ordered,
    ring buffers are protected by device-side event waits;
  * every buffer is per (round mod K) — no aliasing of beta or message buffers across
    rounds (the reference's latent races, SURVEY §5.2, cannot happen);
  * the injected straggler delay is, by default, a virtual arrival time on the master's
    clock (utils/delay.py, --delay-on collector: the GPUs never sleep); with --delay-on worker
    a worker rank is physically late instead (a device spin between its gradient and its
    put, like the reference's time.sleep) and --slow-ranks makes a GPU really slower;
  * the straggler tail after the stop rule (``drain``): "all" waits for every message before
    the next beta (the reference's Waitall, FRC/AGC), "carry" does not wait and late workers
    deliver every round in order (the reference's other schemes), "lazy" does not wait and a
    worker still busy when the next beta is out skips the stale round (csrc/kernels/common.h
    gate_closed; the collector models the same skip for virtual delays) — the replacement of
    the reference's send Cancel (ref src/coded.py:178-180).
"""
from __future__ import annotations

import collections
import math
import os
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .._ext import native as native_ext
from .loops import LoopInputs, release_override, select_release_form, select_round_loop
from ..codes.schemes import Arrival, Scheme, SchemeError, make_scheme, scheme_key
from ..config import RunConfig
from ..data import io as dio
from ..data.source import DataSource, FileSource, SyntheticSource
from ..models.losses import LEAST_SQUARES, LOGISTIC, UpdateRule
from ..ops.grad import DenseGradPlan, SharedGradPlan, SparseGradPlan
from ..ops.precision import get_precision
from ..ops.update import combine_update
from ..parallel.collector import ArrivalCollector
from ..parallel.dist import DistEnv
from ..parallel.placement import make_shards, place_spread, place_units

# Cost of a replica's message rows whose HBM reads a co-located replica already streams, relative
# to a distinct row (dense fp64 on MI355X with the LDS-staged bundles: (1.56 - 1.29) ms for 14 GB
# of replica rows against 1.29 ms for 8 GB of distinct rows; FRC s = 1 gives the same 0.11,
# docs/PERF_NOTES.md).
REPLICA_WEIGHT_DENSE = 0.12
# Sparse plans stream every distinct partition once and encode the replicas (ops/grad.py
# SparseGradPlan): a further replica costs one encode row, next to nothing.
REPLICA_WEIGHT_SPARSE = 0.02
from ..parallel.transport import make_transport

P2P_TRANSPORTS = ("rccl", "loopback", "rccl-self")  # stream-ordered p2p (csrc/runtime/comm.h)
from ..utils import report
from ..utils.delay import DelayModel
from ..utils.tracing import PhaseTimer

@dataclass
class TrainResult:
    scheme: str
    betaset: np.ndarray  # [R, d] beta after each round (fp64)
    timeset: np.ndarray  # [R] time-to-decode per round (reference semantics)
    worker_timeset: np.ndarray  # [R, W]
    loop_time: np.ndarray  # [R] true per-round wall-clock incl. drain
    total_time: float
    timed_seconds: Optional[float] = None
    timed_rounds: int = 0
    timeouts: int = 0
    phases: Dict[str, Dict[str, float]] = field(default_factory=dict)
    arrivals: List[List[Tuple[int, int, float]]] = field(default_factory=list)


class ContainedFailure(RuntimeError):
    """A rank's round loop failed, and the rank has since drained its device and joined the run's
    closing barrier (Trainer.run(contain=True)): the job is collectively consistent again."""


def _sabotage_exit(rank: int) -> Optional[Tuple[str, int]]:
    """Test hook ERASUREHEAD_SABOTAGE=exit:<rank>:<round> (that worker rank exits before that round),
    hang:<rank>:<round> (it stops there and never sends again, alive until the job is torn down) or
    raise:<rank>:<round> (its round loop raises there: Trainer.run(contain=True) must contain it)."""
    spec = os.environ.get("ERASUREHEAD_SABOTAGE", "")
    parts = spec.split(":")
    if len(parts) == 3 and parts[0] in ("exit", "hang", "raise") and int(parts[1]) == rank:
        return parts[0], int(parts[2])
    return None


def _mean_us(ms, a0: int = 0) -> Optional[float]:
    """Mean (microseconds) of the non-negative millisecond entries from round a0 on; None if none."""
    v = [x for x in list(ms)[a0:] if x is not None and x >= 0]
    return 1e3 * float(np.mean(v)) if v else None


class Trainer:
    def __init__(self, cfg: RunConfig, env: Optional[DistEnv] = None, source: Optional[DataSource] = None,
                 scheme: Optional[Scheme] = None):
        self.cfg = cfg
        if env is None:
            from ..parallel.dist import init_distributed

            env = init_distributed("auto")
        self.env = env
        self.timer = PhaseTimer()
        self.device_loop: Optional[str] = None  # set by the native master loop when rounds ran device-driven
        self.rank_stats: Dict[str, float] = {}  # per-rank breakdown of the last run (rank_report)
        self._setup_scheme(scheme, source)
        warm = self._start_eval_warmup()
        self._setup_data(source)
        self._setup_buffers()
        if warm is not None:
            warm.join()

    # ------------------------------------------------------------------------------ setup
    def _start_eval_warmup(self):
        """Master on a GPU, logistic runs that will be evaluated: load the AUC path's code objects on a
        side thread while the data is generated / loaded (ops/eval.warm_auc; 0.6 s cold)."""
        if not (self.env.is_master and self.env.gpu and self.cfg.evaluate and self.loss == LOGISTIC):
            return None
        import threading

        from ..ops.eval import warm_auc

        dev = self.env.device

        def run():
            with torch.cuda.device(dev):
                warm_auc(dev)

        t = threading.Thread(target=run, name="eh-eval-warmup", daemon=True)
        t.start()
        return t

    def _setup_scheme(self, scheme: Optional[Scheme], source: Optional[DataSource] = None):
        cfg, env = self.cfg, self.env
        W = cfg.n_workers
        if W < 1:
            raise SchemeError("n_procs must be >= 2 (one master + at least one worker)")
        self.key = scheme_key(cfg.is_coded, cfg.partitions, cfg.coded_ver)
        if scheme is None:
            rng = np.random.RandomState(cfg.seed) if cfg.seed is not None else None
            B = None
            if env.is_master or env.world == 1:
                B0 = self._checkpoint_B(cfg.resume) if cfg.resume else None  # a resumed run keeps its code
                scheme = make_scheme(self.key, W, cfg.n_stragglers, cfg.n_rows, cfg.num_collect, cfg.partitions,
                                     cfg.allow_uneven_groups, rng if B0 is None else None, B0)
                B = scheme.B
            B = env.broadcast_object(B, 0) if env.world > 1 else B
            if not env.is_master:
                scheme = make_scheme(self.key, W, cfg.n_stragglers, cfg.n_rows, cfg.num_collect, cfg.partitions,
                                     cfg.allow_uneven_groups, None, B)
        self.scheme = scheme
        if cfg.loss == "auto":
            self.loss = LEAST_SQUARES if (cfg.dataset == "kc_house_data" and scheme.has_linear) else LOGISTIC
        else:
            self.loss = LEAST_SQUARES if cfg.loss == "least_squares" else LOGISTIC
        self.rule_kind, self.rule_k = scheme.rule()
        self.update = UpdateRule("AGD" if scheme.fixed_agd else cfg.update_rule, cfg.alpha_value, cfg.n_rows,
                                 scheme.grad_scale())
        self.drain_mode = cfg.drain or ("all" if scheme.drain else "carry")
        self.drain = self.drain_mode == "all"
        self.skip_stale = self.drain_mode == "lazy"
        inject = cfg.add_delay == 1 and (scheme.has_delay or cfg.force_delay)
        mode = "none"
        if inject:
            mode = cfg.delay_mode if cfg.delay_mode in ("exp", "fixed") else "none"
        self.delay = DelayModel(W, mode, cfg.delay_mean, [w - 1 for w in cfg.fixed_stragglers], cfg.fixed_sleep,
                                [w - 1 for w in cfg.kill_workers])
        # placement (parallel/placement.py): whole messages dealt round-robin over the ranks (the
        # default: the reference's one-worker-per-process topology, a slow GPU erases only its own
        # workers), or with partition shards (benchmark opt-in) one shard per (message, partition)
        # placed sharing-aware: each partition's replicas live on one rank and stream once.
        rows = scheme.rows_per_partition
        sparse = source.is_sparse if source is not None else bool(cfg.is_real)
        if cfg.share_partitions:
            replica_weight = 0.0
        elif env.gpu and not sparse:
            replica_weight = REPLICA_WEIGHT_DENSE
        elif env.gpu:
            replica_weight = REPLICA_WEIGHT_SPARSE
        else:
            replica_weight = 1.0
        self.shard_mode = cfg.shard if cfg.shard != "auto" else "message"
        self.shards = make_shards(scheme.messages, self.shard_mode)
        parts = [[(p, rows) for p, _ in u.segments] for u in self.shards]
        # --dedicated-master: the worker ranks are 1..world-1, rank 0 only runs the master (the reference
        # topology); otherwise rank 0 hosts workers too
        dedicated = bool(cfg.dedicated_master) and env.world > 1
        ranks = env.world - 1 if dedicated else env.world
        if self.shard_mode == "partition":
            self.owner = place_units(parts, ranks, replica_weight)
        else:
            self.owner = place_spread([u.worker for u in self.shards], ranks)
        if dedicated:
            self.owner = [o + 1 for o in self.owner]
        self.by_rank = {r: sorted({u.worker for u, o in zip(self.shards, self.owner) if o == r})
                        for r in range(env.world)}
        self.local_msgs = [u for u, o in zip(self.shards, self.owner) if o == env.rank]
        self.remote_msgs = {r: [u for u, o in zip(self.shards, self.owner) if o == r]
                            for r in range(1, env.world)} if env.is_master else {}
        self.n_shards = {(u.worker, u.part): u.n_shards for u in self.shards}
        # physically late worker ranks (--delay-on worker): a worker rank sleeps / spins after its
        # compute and before its send; the master's collector then sees real arrival times for
        # remote messages (virtual delay 0; dead workers stay virtual erasures) and keeps the
        # virtual per-worker delay only for the logical workers co-located with it on rank 0
        self.physical = cfg.delay_on == "worker" and env.world > 1 and self.delay.mode != "none"
        self.repeat = int(cfg.slow_ranks.get(env.rank, 1))  # --slow-ranks: gradient launches per round

    def _setup_data(self, source: Optional[DataSource]):
        cfg, sch = self.cfg, self.scheme
        self.prec = get_precision(cfg.precision)
        if source is None:
            if cfg.data == "synthetic":
                source = SyntheticSource(cfg.n_rows, cfg.n_cols, sch.n_partition_files, cfg.data_seed)
            else:
                data_dir = dio.dataset_dir(cfg.input_dir, cfg.is_real, cfg.dataset, cfg.n_rows, cfg.n_cols)
                data_dir = data_dir + sch.data_subdir()
                source = FileSource(data_dir, cfg.is_real, sch.rows_per_partition, cfg.n_cols)
        self.source = source
        self.d = cfg.n_cols
        self.ld = self.prec.ld(self.d)
        dev = self.env.device
        needed = sorted({p for m in self.local_msgs for p, _ in m.segments})
        if not source.is_sparse and self.env.gpu:
            self._check_hbm(len(needed) * sch.rows_per_partition * self.ld * self.prec.storage_bytes)
        t0 = time.perf_counter()
        parts = {p: source.partition(p, self.prec, dev) for p in needed}
        self.load_seconds = time.perf_counter() - t0
        segs = [m.segments for m in self.local_msgs]

        def make_plan(messages):
            if source.is_sparse:
                return SparseGradPlan(messages, parts, self.prec, self.loss, self.d, device=dev)
            kw = {"target_tasks": cfg.tasks} if cfg.tasks else {}
            return DenseGradPlan(messages, parts, self.prec, self.loss, self.d, **kw)

        if cfg.share_partitions and SharedGradPlan.worthwhile(segs, lambda p: parts[p][0].shape[0]):
            self.plan = SharedGradPlan(segs, make_plan)
        else:
            self.plan = make_plan(segs)
        self._parts = parts

    def _check_hbm(self, need_bytes: int) -> None:
        """Fail early (and say what to change) when this rank's resident partitions cannot fit."""
        free, total = torch.cuda.mem_get_info(self.env.device)
        if need_bytes > 0.92 * free:
            raise MemoryError(
                f"rank {self.env.rank}: its logical workers need {need_bytes / 2**30:.1f} GiB of resident "
                f"partitions but only {free / 2**30:.1f} of {total / 2**30:.1f} GiB HBM are free; launch more GPU "
                f"ranks (torchrun --nproc-per-node) or use --precision fp32/bf16")

    def _setup_buffers(self):
        cfg, env = self.cfg, self.env
        R, ld, acc, dev = cfg.num_itrs, self.ld, self.prec.acc, env.device
        es = torch.tensor([], dtype=acc).element_size()
        n_loc = len(self.local_msgs)
        n_rem = sum(len(v) for v in self.remote_msgs.values())
        per_round = max(1, (n_loc + n_rem) * ld * es)
        K = int(max(2, min(R, (4 << 30) // per_round)))  # <= 4 GiB of message ring (288 GB HBM)
        self.K = int(env.broadcast_object(K, 0)) if env.world > 1 else K  # the mailbox ring is shared: one K
        self.G = torch.zeros((self.K, max(1, n_loc), ld), dtype=acc, device=dev)
        self.n_loc = n_loc
        remote_counts = {r: len(v) for r, v in self.remote_msgs.items() if v} if env.is_master else {}
        self._choose_release_form()  # before the transport: its handshake puts already use the form
        self.tx = make_transport(cfg.transport, env, R, self.K, ld, acc, n_loc, remote_counts, cfg.round_timeout) \
            if env.world > 1 else None
        if env.is_master:
            self.rem_slot = {}
            for r in sorted(self.remote_msgs):
                for jj, m in enumerate(self.remote_msgs[r]):
                    self.rem_slot[(m.worker, m.part, m.shard)] = self.tx.row0[r] + jj
            self.Rbuf = self.tx.make_rbuf() if self.tx is not None else None
            self.beta = torch.zeros(ld, dtype=torch.float64, device=dev)
            self.u = torch.zeros(ld, dtype=torch.float64, device=dev)
            self.hist = torch.zeros((R, ld), dtype=torch.float64, device=dev)
            self.beta_in = torch.zeros((R + 1, ld), dtype=acc, device=dev)
            self.loc_index = {(m.worker, m.part, m.shard): j for j, m in enumerate(self.local_msgs)}
        if env.gpu:
            self.cs = torch.cuda.current_stream(dev)
            self.loc_ev = [torch.cuda.Event() for _ in range(self.K)]
            if env.is_master:
                self.upd_ev = torch.cuda.Event()

    def _choose_release_form(self) -> None:
        """Collective on GPU ranks: gather every rank's GPU (PCI bus id) and set this process's release
        form for every later put / signal / arbiter launch (engine/loops.py select_release_form; the
        native default is strict).  ERASUREHEAD_FAKE_DEVICE_MAP=<id>,<id>,... (one per rank) stands in
        for the bus ids, so a one-GPU box can exercise the cross-device selection."""
        env = self.env
        self.device_map: List[str] = []
        self.release_form, self.release_reason = "n/a", "CPU ranks: no device puts"
        if not env.gpu:
            return
        C = native_ext()
        dev = env.device.index if env.device.index is not None else torch.cuda.current_device()
        mine = C.pci_bus_id(dev)
        buses = env.broadcast_object(env.gather_objects(mine), 0) if env.world > 1 else [mine]
        fake = [x.strip() for x in os.environ.get("ERASUREHEAD_FAKE_DEVICE_MAP", "").split(",") if x.strip()]
        if fake and len(fake) == env.world:
            buses = [f"fake:{x}" for x in fake]
        self.device_map = list(buses)
        self.release_form, self.release_reason = select_release_form(self.device_map, release_override())
        C.set_release_form(self.release_form == "strict")

    def preflight(self, iters: int = 1000) -> Optional[List[dict]]:
        """Collective: per-pair put -> flag round trips over the IPC mailbox (IpcTransport.preflight);
        None when there is no IPC transport."""
        if self.tx is None or not hasattr(self.tx, "preflight"):
            return None
        recs = self.tx.preflight(iters)
        # ranks with their own GPUs: the RCCL point-to-point path (the IPC fallback) measured per pair too
        if recs is not None and self.env.backend == "nccl" and self.env.device.type == "cuda":
            from ..parallel.transport import rccl_p2p_preflight

            try:  # informational: a failure is recorded, the run goes on over IPC
                rc = rccl_p2p_preflight(self.env, self.ld, self.prec.acc, iters=min(200, iters))
            except Exception as e:  # noqa: BLE001
                rc = {r: {"rccl_error": f"{type(e).__name__}: {e}"[:300]} for r in range(1, self.env.world)}
            rc = self.env.broadcast_object(rc, 0)
            for rec in recs:
                rec.update(rc.get(rec["rank"], {}))
        return recs

    @property
    def transport(self) -> str:
        return self.tx.name if self.tx is not None else "local"

    @property
    def replica_policy(self) -> str:
        """How this rank's plan forms the replica messages of a partition it hosts several times:
        "separate" -- every replica does its own arithmetic from the shared read (dense plans, the
        headline: ref src/approximate_coding.py:185-196 computes each worker's message by itself);
        "encoded" -- each distinct partition's gradient is computed once with coefficient 1 and the
        replicas are formed by the device encoding (sparse plans, --share-partitions); "none" -- no
        partition is hosted twice (naive, ignore-stragglers, one message per rank)."""
        plan = getattr(self, "plan", None)
        counts = collections.Counter(p for m in self.local_msgs for p, _ in m.segments)
        if not counts or max(counts.values()) < 2:
            return "none"
        if isinstance(plan, (SharedGradPlan, SparseGradPlan)):
            return "encoded"
        return "separate"

    # --------------------------------------------------------------------------- helpers
    def _init_beta(self):
        """beta_0: randn (naive/replication/approx) or zeros (ref §2.2 'Per-scheme beta init')."""
        d = self.d
        if self.scheme.init_zero:
            b0 = np.zeros(d)
        elif self.cfg.seed is not None:
            b0 = np.random.RandomState(self.cfg.seed + 1).randn(d)
        else:
            b0 = np.random.randn(d)
        self.beta.zero_()
        self.beta[:d] = torch.from_numpy(b0).to(self.beta.device)
        self.u.zero_()
        self.beta_in[0].zero_()
        self.beta_in[0, :d] = self.beta[:d].to(self.beta_in.dtype)
        self.beta0 = b0

    def _sync(self):
        if self.env.gpu:
            torch.cuda.synchronize(self.env.device)

    def warmup(self):
        """Discarded warm-up gradient (ref src/naive.py:39-44); also loads the kernels."""
        beta = torch.zeros(self.ld, dtype=self.prec.acc, device=self.env.device)
        if self.local_msgs:
            self.plan.run(beta, self.G[0])
        self._sync()

    def time_local_grad(self, reps: int = 5) -> Optional[float]:
        """Mean microseconds of this rank's gradient launch run on its own (no transport, no
        other rank's traffic); HIP events on a GPU, host time on the CPU."""
        if not self.local_msgs:
            return None
        beta = torch.zeros(self.ld, dtype=self.prec.acc, device=self.env.device)
        beta[: self.d] = 1e-3
        self.plan.run(beta, self.G[0])
        if self.env.gpu:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                self.plan.run(beta, self.G[0])
            e1.record()
            e1.synchronize()
            return 1e3 * e0.elapsed_time(e1) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            self.plan.run(beta, self.G[0])
        return 1e6 * (time.perf_counter() - t0) / reps

    # ------------------------------------------------------------------------------ run
    def run(self, timed_start: Optional[int] = None, log=None, contain: bool = False) -> Optional[TrainResult]:
        """Train for cfg.num_itrs rounds; returns the master's TrainResult (None on workers).

        timed_start: if set, all ranks synchronise (device sync + barrier) before that round
        and after the last one, and the result carries the timed wall-clock (bench.py).
        contain: a failure inside the round loop (a timeout, an integrity-tag verdict, a device
        round that did not decode) does not leave the job split across collectives: the failing
        rank drains its device (bounded), joins the barriers its loop had not reached yet (the timed
        fences and the closing barrier, counted), and raises :class:`ContainedFailure`.  Every rank
        then stands at the same point, so the caller can agree on a verdict (:meth:`run_contained`)
        and rebuild.  Not with cfg.verify_beta (its gather sits between the loops' barriers).
        """
        log = log or report.log
        cfg, env = self.cfg, self.env
        self.warmup()
        start = 0
        if env.is_master:
            self._init_beta()
            if cfg.resume:
                start = self._restore(cfg.resume)
            for line in self.scheme.setup_lines():
                if cfg.verbose:
                    log(line)
        start = env.broadcast_object(start, 0)
        env.barrier()
        self.loop, self.loop_reason = select_round_loop(self.loop_inputs(start))
        self.device_records = None
        # physically late ranks: every rank's GPU clock against the host clock, so the master's collector
        # orders their messages by when they landed (collector.h "Device times")
        self._clocks = None
        if env.gpu and env.world > 1 and self.loop != "python" and (self.physical or cfg.device_records):
            C = native_ext()
            dev = env.device.index if env.device.index is not None else torch.cuda.current_device()
            self._clocks = env.broadcast_object(env.gather_objects((env.rank, *C.device_clock(dev))), 0)
        native_loop = self.native_loop
        if self.skip_stale and self.loop == "python" and self.tx is not None and self.tx.name in P2P_TRANSPORTS:
            # the Python round loop receives beta in stream order (no look-ahead), so a p2p worker cannot
            # tell that a round is stale before computing it: the run switches to the carry drain -- the
            # master's collector included, so the books and the rank report say what ran
            why = (f"drain lazy -> carry: in the Python round loop over {self.tx.name} the workers cannot skip "
                   f"stale rounds (beta arrives in stream order, no look-ahead)")
            if env.is_master:
                print(f"[erasurehead] WARNING: {why}", file=sys.stderr, flush=True)
            self.rank_stats["drain_downgraded"] = why
            self.drain_mode, self.skip_stale = "carry", False
        self._coll_done = 0
        contain = contain and not cfg.verify_beta
        try:
            if env.is_master:
                res = (self._master_loop_native if native_loop else self._master_loop)(timed_start, log, start)
            else:
                res = (self._worker_loop_native if native_loop else self._worker_loop)(timed_start, start)
        except BaseException as e:
            if self.tx is not None:  # release queued p2p work on peers that will not answer
                self.tx.abort()
            if contain and isinstance(e, Exception) and not isinstance(e, ContainedFailure):
                self._contain_failure(e, self._loop_collectives(timed_start, start) - self._coll_done)
                raise ContainedFailure(f"rank {env.rank}: {type(e).__name__}: {e}") from e
            raise
        return res

    def _contain_failure(self, e: Exception, barriers: int, drain_s: float = 60.0) -> None:
        """run(contain=True) after a failure inside a round loop: wait (bounded) for this rank's device
        work to drain -- the pumps have released their queued waits (WorkerPump stop_queued, the
        arbiter's abort word) -- then call the ``barriers`` barriers the loop had left.  A device that
        does not drain cannot be recovered in this process: the original error is re-raised unchanged."""
        import threading

        print(f"[erasurehead] rank {self.env.rank}: round loop failed ({type(e).__name__}: {str(e)[:300]}); "
              f"draining the device and joining the closing barrier", file=sys.stderr, flush=True)
        if self.env.gpu:
            done = threading.Event()

            def drain():
                torch.cuda.synchronize(self.env.device)
                done.set()

            threading.Thread(target=drain, name="eh-contain-drain", daemon=True).start()
            if not done.wait(drain_s):
                raise e
        for _ in range(max(0, barriers)):
            self.env.barrier()

    def run_contained(self, timed_start: Optional[int] = None, log=None) -> Tuple[Optional[TrainResult], Optional[str]]:
        """Collective.  run(contain=True) on every rank, then one verdict every rank agrees on:
        (result, None) after a clean run (result None on workers), or (None, reasons) when any rank's
        round loop failed -- the reasons of every failing rank, joined."""
        res, err = None, None
        try:
            res = self.run(timed_start, log, contain=True)
        except ContainedFailure as e:
            err = str(e)
        if self.env.world > 1:
            errs = self.env.gather_objects(err)
            verdict = self.env.broadcast_object("; ".join(x for x in errs if x) if self.env.is_master else None, 0)
        else:
            verdict = err
        if verdict:
            return None, verdict
        if res is not None and not bool(np.all(np.isfinite(res.betaset))):
            verdict = "the trajectory has non-finite entries"
        if self.env.world > 1:
            verdict = self.env.broadcast_object(verdict if self.env.is_master else None, 0)
        return (None, verdict) if verdict else (res, None)

    def loop_inputs(self, start: int = 0, blocker: str = "") -> LoopInputs:
        """This run's facts for engine/loops.py select_round_loop (the same on every rank)."""
        cfg, sch, R = self.cfg, self.scheme, self.cfg.num_itrs
        W, s = cfg.n_workers, sch.n_stragglers
        table = sch.decode_kind in (3, 4)
        tx = self.tx
        if self.env.world > 1:
            d = self.delay_table()[start:]
            r = self._remote_delays(d) if d.size else d
            local = sorted({u.worker for u, o in zip(self.shards, self.owner) if o == 0})
            remote = sorted({u.worker for u, o in zip(self.shards, self.owner) if o != 0})
            virtual = bool(d.size) and (bool(np.any(d[:, local] != 0)) or bool(np.any(r[:, remote] != 0)))
        else:
            d = self.delay_table()[start:]
            virtual = bool(d.size) and bool(np.any(d != 0))
        return LoopInputs(
            gpu=bool(self.env.gpu), world=self.env.world,
            transport="local" if tx is None else ("gloo" if not self.env.gpu else tx.name),
            virtual_delay=virtual, physical_delay=bool(self.physical or self.cfg.slow_ranks),
            drain=self.drain_mode, instrument=bool(cfg.instrument), checkpoint=bool(cfg.checkpoint_every),
            resume=bool(start), verify_beta=bool(cfg.verify_beta), native_loop=bool(cfg.native_loop),
            device_loop=cfg.device_loop, device_master=os.environ.get("ERASUREHEAD_DEVICE_MASTER", "auto"),
            shared_gpu=bool(tx is not None and self._shared_gpu(tx)), has_local=bool(self.local_msgs),
            table_w64=table and W > 64, table_ondemand=table and math.comb(W, s) > 20000, blocker=blocker)

    def delay_table(self) -> np.ndarray:
        """[R, W] injected delay of every logical worker in every round (utils/delay.py)."""
        R, W = self.cfg.num_itrs, self.cfg.n_workers
        return np.stack([self.delay.delays(i) for i in range(R)]) if R else np.zeros((0, W))

    @property
    def native_loop(self) -> bool:
        """Run rounds in the C++ executors (engine/loops.py: every master loop but "python"; a worker
        rank without messages only waits for beta, which the Python loop does as well)."""
        if not hasattr(self, "loop"):
            self.loop, self.loop_reason = select_round_loop(self.loop_inputs())
        if self.loop == "python":
            return False
        return self.n_loc > 0 or self.env.is_master

    def _final_drain(self, col) -> bool:
        """After the last round: wait until every message of every round has arrived (dead workers
        excepted), bounded by the round timeout or the longest virtual lag the delays can carry.  A
        message that never lands means a worker rank is gone: the transport is aborted (its queued
        receives released) before anything synchronises the device, and the run fails with that reason."""
        d = self.delay_table()
        fin = np.where(np.isfinite(d), d, 0.0) if d.size else d
        lag = float(np.sum(np.max(fin, axis=1))) if fin.size else 0.0
        ok = col.drain(self.cfg.num_itrs - 1, max(float(self.cfg.round_timeout), min(600.0, lag + 10.0)))
        if not ok and self.tx is not None:
            why = f"rank 0: {col.c.pending_upto(self.cfg.num_itrs - 1)} messages never arrived; aborting the transport"
            print(f"[erasurehead] WARNING: {why}", file=sys.stderr, flush=True)
            self.rank_stats["aborted"] = why
            self.tx.abort()
            # the device is drained now (the abort released the queued receives); a rank that is gone
            # cannot join the run's closing collectives, so the run fails here, by name
            self._sync()
            raise RuntimeError(why)
        return ok

    def _timed_fence(self):
        self._sync()
        self._coll_done += 1
        self.env.barrier()
        return time.perf_counter()

    def _closing_barrier(self):
        """The barrier every round loop ends with (counted: run(contain=True) replays what is left)."""
        self._coll_done += 1
        self.env.barrier()

    def _loop_collectives(self, timed_start: Optional[int], start: int) -> int:
        """Barriers a round loop calls on its success path, in order: the timed fences around the timed
        rounds (the opening one only when the timed start is inside the run) and the closing barrier.
        The same count on every rank and in every loop (the race check's gather is outside contain)."""
        n = 1
        if timed_start is not None:
            n += 1 + int(start <= timed_start < self.cfg.num_itrs)
        return n

    def _master_loop(self, timed_start, log, start: int = 0) -> TrainResult:
        cfg, env, sch = self.cfg, self.env, self.scheme
        R, W, K = cfg.num_itrs, cfg.n_workers, self.K
        eta = cfg.eta()
        col = ArrivalCollector(W, sch.group_of, sch.n_groups, env.gpu, cfg.tie_seed_value)
        col.set_shards(self.n_shards)
        col.set_skip_stale(self.skip_stale)
        if self.tx is not None and hasattr(self.tx, "check_queue_budget") and env.gpu:
            self.rank_stats.update(self.tx.check_queue_budget(len(self.tx.ps)))  # its per-peer streams
        timeset = np.zeros(R)
        loop_time = np.zeros(R)
        worker_timeset = np.zeros((R, W))
        arrivals_log: List = [[] for _ in range(start)]
        upd_events: List = []
        delay_table = self.delay_table()
        remote_table = self._remote_delays(delay_table)
        views: Dict[Tuple[int, int, int], torch.Tensor] = {}  # (slot, worker, part) -> message row
        if start:
            timeset[:start] = self._restored["timeset"]
            worker_timeset[:start] = self._restored["worker_timeset"]
        timeouts = 0
        t_timed0 = t_timed1 = None
        if cfg.verbose:
            log(sch.banner(cfg.add_delay))
        orig_start = time.perf_counter()
        for i in range(start, R):
            if timed_start is not None and i == timed_start:
                t_timed0 = self._timed_fence()
            if cfg.verbose and i % 10 == 0:
                log(report.iteration_tick(i))
            slot = i % K
            if i >= K and not col.wait_seen(i - K, cfg.round_timeout):  # ring slot reuse: round i-K landed
                raise TimeoutError(f"round {i}: messages of round {i - K} still in flight after "
                                   f"{cfg.round_timeout}s; cannot reuse mailbox slot {i % K}")
            t_start = col.now()
            col.begin_round(i, t_start, self.rule_kind, self.rule_k)
            delays = delay_table[i]
            with self.timer.phase("send_beta"):
                self._send_beta(i)
            with self.timer.phase("local_grad"):
                if self.local_msgs:
                    for _ in range(self.repeat):  # --slow-ranks: a slower GPU
                        self.plan.run(self.beta_in[i], self.G[slot])
                    if env.gpu:
                        ev = self.loc_ev[slot]
                        ev.record(self.cs)
                        for m in self.local_msgs:
                            col.add_event(m.worker, m.part, i, ev, delays[m.worker])
                    else:  # one compute call finished every local message: they are seen together
                        t_done = col.now()
                        for m in self.local_msgs:
                            col.add_work(m.worker, m.part, i, None, delays[m.worker], t_seen=t_done)
            with self.timer.phase("post_recv"):
                self._post_recvs(i, slot, col, remote_table[i])
            with self.timer.phase("wait_k"):
                arrivals, ok = col.wait(cfg.round_timeout)
            if not ok:
                timeouts += 1
            with self.timer.phase("decode_update"):
                used = sch.decode(arrivals)
                msgs, coefs = [], []
                for (w, part), c in sorted(used.items()):
                    for k in range(self.n_shards[(w, part)]):  # a message = the sum of its shards
                        key = (w, part, k)
                        v = views.get((slot, key))
                        if v is None:
                            v = self.G[slot, self.loc_index[key]] if key in self.loc_index else \
                                self.Rbuf[slot, self.rem_slot[key]]
                            views[(slot, key)] = v
                        if key not in self.loc_index:
                            self.tx.before_read(slot, self.rem_slot[key])
                        msgs.append(v)
                        coefs.append(c)
                decay, gm, l2, theta, code = self.update.coeffs(i, float(eta[i]))
                if env.gpu and not cfg.sync_update:
                    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    ev0.record(self.cs)
                combine_update(msgs, coefs, self.beta, self.u, self.d, decay, gm, l2, theta, code,
                               hist=self.hist[i], beta_w=self.beta_in[i + 1])
                if env.gpu:
                    if cfg.sync_update:
                        self.upd_ev.record(self.cs)
                        self.upd_ev.synchronize()
                    else:  # no host round trip: the next round's sends are stream-ordered behind it
                        ev1.record(self.cs)
                        upd_events.append((i, ev0, ev1))
            timeset[i] = col.now() - t_start
            worker_timeset[i] = sch.worker_times(arrivals)
            arrivals_log.append([(a.worker, a.part, a.t_rel) for a in arrivals])
            if self.drain:
                with self.timer.phase("drain"):
                    col.drain(i, cfg.round_timeout)
            loop_time[i] = col.now() - t_start
            if cfg.checkpoint_every and (i + 1) % cfg.checkpoint_every == 0:
                self._checkpoint(i + 1, timeset, worker_timeset)
        if self.skip_stale:  # whatever a late worker still has queued is stale now
            col.c.end_run(col.now())
            if self.tx is not None:
                self.tx.release_workers(R + 1)
        if timed_start is not None:  # rounds complete on every rank at the fence (see the native loop)
            t_timed1 = self._timed_fence()
        self._final_drain(col)
        self.rank_stats.update(stale_skipped_virtual=col.skipped, stale_arrivals=col.stale_arrivals)
        col.close()
        if cfg.verify_beta and env.world > 1:
            self._verify_beta_checksums(start)
        if upd_events:
            torch.cuda.synchronize(env.device)
            for i, ev0, ev1 in upd_events:  # + the update kernel's own duration (reference: decode + update)
                timeset[i] += 1e-3 * ev0.elapsed_time(ev1)
        self._sync()
        self._closing_barrier()
        total = time.perf_counter() - orig_start
        a0 = (timed_start or start) - start
        self.rank_stats.update({f"{k}_us": float(1e6 * np.mean(v[a0:])) for k, v in self.timer.t.items()
                                if len(v) > a0})
        res = TrainResult(self.key, self.hist[:, : self.d].double().cpu().numpy(), timeset, worker_timeset, loop_time,
                          total, timeouts=timeouts, phases=self.timer.summary(), arrivals=arrivals_log)
        if t_timed0 is not None:
            res.timed_seconds = t_timed1 - t_timed0
            res.timed_rounds = R - timed_start
        return res

    def rank_report(self) -> Dict[str, object]:
        """This rank's share of the job and where its round time went (bench.py per-rank breakdown).

        Times are means over the timed rounds, in microseconds: ``kernel_us`` the local gradient
        launch (HIP events; cfg.instrument), ``beta_put_us`` / ``msg_put_us`` the put+signal
        launches (a worker with ``fused_put`` issues its message put + signal from the final
        reduction kernel, so ``kernel_us`` includes it and ``msg_put_us`` is ~0), ``beta_wait_us`` a worker's host wait for beta, ``wait_k_us`` the master's wait
        for the stop rule, ``decode_update_us`` its host decode + combine/update enqueue and
        ``update_kernel_us`` the combine+update kernel itself.
        """
        env = self.env
        role = ("master+workers" if self.local_msgs else "master") if env.is_master else "workers"
        rep: Dict[str, object] = {"rank": env.rank, "role": role, "device": str(env.device),
                                  "transport": self.transport,
                                  "round_loop": self.device_loop or ("native pump" if self.native_loop else "python"),
                                  "loop_reason": getattr(self, "loop_reason", None),
                                  "drain": self.drain_mode,
                                  "release_form": getattr(self, "release_form", None),
                                  "replicas": self.replica_policy,
                                  "workers": sorted({int(m.worker) for m in self.local_msgs}),
                                  "messages": len(self.local_msgs),
                                  "partitions": len({p for m in self.local_msgs for p, _ in m.segments})}
        rep.update({k: (round(float(v), 2) if isinstance(v, (int, float)) and not isinstance(v, bool) else v)
                    for k, v in self.rank_stats.items() if v is not None})
        kern = self._kernel_label()
        if kern:
            rep["grad_kernel"] = kern
        if self.tx is not None and self.tx.name in P2P_TRANSPORTS:
            from .. import HW_QUEUES

            rep["hw_queues"] = int(HW_QUEUES)  # what HIP started with, not the (possibly later) environment
        if self.tx is not None and self.tx.fallback_reason:
            rep["transport_fallback"] = self.tx.fallback_reason
        if self.tx is not None and env.is_master and self.tx.pairs:
            rep["peer_access"] = [{k: x[k] for k in ("rank", "same_gpu", "master_to_rank", "rank_to_master")}
                                  for x in self.tx.pairs]
        return rep

    def _kernel_label(self) -> Optional[str]:
        """Which gradient kernel this rank's plan launches (bench.py per-rank breakdown)."""
        plan = getattr(self, "plan", None)
        inner = getattr(plan, "inner", plan)  # SharedPlan wraps a dense plan
        if inner is None or not hasattr(inner, "choice"):
            return type(plan).__name__ if plan is not None else None
        if getattr(inner, "device", None) is not None and inner.device.type != "cuda":
            return "torch reference path (CPU)"
        return inner.choice.label()

    def _master_loop_native(self, timed_start, log, start: int = 0) -> TrainResult:
        """Master rounds in csrc/runtime/engine.cpp (MasterPump); Python only keeps the books."""
        cfg, env, sch = self.cfg, self.env, self.scheme
        R, W, K = cfg.num_itrs, cfg.n_workers, self.K
        C = native_ext()
        col = ArrivalCollector(W, sch.group_of, sch.n_groups, True, cfg.tie_seed_value)
        col.set_shards(self.n_shards)
        dev = env.device.index if env.device.index is not None else torch.cuda.current_device()
        pump = C.MasterPump(col.c, W, R, K, self.d, self.ld, dev, float(cfg.round_timeout))
        pump.set_skip_stale(self.skip_stale)
        pump.set_state(self.beta, self.u, self.hist, self.beta_in)
        if self.local_msgs:
            pump.set_local(self.plan.native_launcher(), self.G, [(m.worker, m.part) for m in self.local_msgs])
        tx = self.tx
        if tx is not None and tx.name != "ipc":  # RCCL / loopback p2p: receives + events, no IPC counters
            pump.set_comm(tx.comm, tx.sender_rows(), list(range(1, env.world)))
            self.rank_stats.update(tx.check_queue_budget(int(pump.comm_streams)))
            rem = [(m.worker, m.part, self.rem_slot[(m.worker, m.part, m.shard)], 0, r)
                   for r in sorted(self.remote_msgs) for m in self.remote_msgs[r]]
            pump.set_remote(self.Rbuf, rem)
        elif tx is not None:
            rem = [(m.worker, m.part, self.rem_slot[(m.worker, m.part, m.shard)], tx.flags.host_addr(env.world + r), r)
                   for r in sorted(self.remote_msgs) for m in self.remote_msgs[r]]
            pump.set_remote(self.Rbuf, rem)
            # every message / beta carries a (round, rank, checksum) tag that the receiver checks
            pump.set_integrity(tx.mbox_tags_addr(), tx.inbox_tag_off, bool(cfg.integrity))
            pump.set_puts([(tx.inbox_remote[r].data_ptr(), tx.flags.dev_addr(r)) for r in range(1, env.world)],
                          tx.counters)
            srcs = [(tx.flags.host_addr(env.world + r), tx.flags.dev_addr(env.world + r))
                    for r in sorted(self.remote_msgs) if self.remote_msgs[r]]
            pump.set_sources(srcs)
            if self._device_waits(tx):  # drain on the device: beta(i+1) leaves as the last message lands
                self.rank_stats["device_drain"] = bool(pump.set_drain_flags(srcs))
        eta = cfg.eta()
        co = [self.update.coeffs(i, float(eta[i])) for i in range(R)]
        delay_table = self.delay_table()
        pump.set_schedule([c[0] for c in co], [c[1] for c in co], [c[2] for c in co], [c[3] for c in co],
                          co[0][4] if co else 0, [float(x) for x in delay_table.ravel()], self.rule_kind,
                          self.rule_k, bool(self.drain))
        if self.physical:  # remote messages are really late: the collector applies no virtual delay to them
            pump.set_remote_delays([float(x) for x in self._remote_delays(delay_table).ravel()])
        if self._clocks and tx is not None and (self.physical or cfg.device_records):
            ring = (tx.flags.host_addr(tx.stamp_base), tx.K) if tx.name == "ipc" else (0, 1)
            pump.set_device_times([tuple(c) for c in self._clocks if c[0] != 0], *ring)
        if cfg.device_records:
            pump.set_records(True)
        pump.set_repeat(self.repeat)
        # device-driven local rounds: combine + update inside the slab reduction (off: separate launches)
        pump.set_fused_update(bool(getattr(self, "fused_update", True)))
        pump.set_decode(sch.decode_kind, list(sch.group_of), sch.n_groups)
        pump.set_timing(bool(cfg.instrument))
        table_decoded = sch.decode_kind in (3, 4)
        if table_decoded and math.comb(W, sch.n_stragglers) <= 20000:  # else filled on demand below
            for mask, a in sch.decode_table().items():
                pump.add_table(mask, [float(x) for x in a])
        timeset, loop_time, worker_timeset = np.zeros(R), np.zeros(R), np.zeros((R, W))
        arrivals_log: List = [[] for _ in range(start)]
        if start:
            timeset[:start] = self._restored["timeset"]
            worker_timeset[:start] = self._restored["worker_timeset"]
        timeouts = 0
        t_timed0 = t_timed1 = None
        if cfg.verbose:
            log(sch.banner(cfg.add_delay))
        orig_start = time.perf_counter()
        if self.loop == "arbiter":  # the pump's structural limits (engine/loops.py: blocker)
            why = pump.device_blocker(start, R)
            if why:
                if os.environ.get("ERASUREHEAD_DEVICE_MASTER", "auto") == "on":
                    raise RuntimeError(f"ERASUREHEAD_DEVICE_MASTER=on, but the rounds cannot run on the device: {why}")
                self.loop, self.loop_reason = select_round_loop(self.loop_inputs(start, blocker=why))
        device_mode = self.loop if self.loop in ("graph", "stream") else None
        arb_mode = self.loop == "arbiter"
        if arb_mode:
            # every round on the device: the master's gradient, then csrc/kernels/arbiter.hip polls the
            # workers' counters, decodes, updates and releases the next beta; the host only reads back
            cuts = [start] + ([timed_start] if timed_start is not None and start < timed_start < R else []) + [R]
            deadline = min(float(cfg.round_timeout), 60.0)
            for a, b in zip(cuts[:-1], cuts[1:]):
                if timed_start is not None and a == timed_start:
                    t_timed0 = self._timed_fence()
                pump.run_device(a, b, deadline)
            pump.finish_run()  # lazy drain: a late worker's queued rounds are stale now
            if timed_start is not None:
                t_timed1 = self._timed_fence()
            for i, (status, arr, tdec, tend, detail, tstop, (tjoin, tdecoded)) in zip(range(start, R),
                                                                                     pump.device_log(start, R)):
                if status:
                    why = detail or {1: f"a worker rank's message did not arrive within {deadline:.0f} s",
                                 2: "the arrivals could not be decoded on the device",
                                 3: "an earlier round failed"}.get(status, f"status {status}")
                    raise RuntimeError(f"device-driven round {i}: {why}")
                if tstop >= 0:  # arbiter ticks: poll until the stop rule, combine + checks, drain + release
                    self.timer.add("arbiter_poll", tstop)
                    self.timer.add("arbiter_update", tdec - tstop)
                    self.timer.add("arbiter_join", tjoin - tstop)  # the update's parts: barrier + acquire,
                    self.timer.add("arbiter_decode", tdecoded - tjoin)  # decode (thread 0),
                    self.timer.add("arbiter_combine", tdec - tdecoded)  # combine + update + beta puts
                    self.timer.add("arbiter_release", tend - tdec)
                arrivals = [Arrival(w, p, t) for (w, p, t) in arr]
                timeset[i], loop_time[i] = tdec, tend
                worker_timeset[i] = sch.worker_times(arrivals)
                arrivals_log.append([(a.worker, a.part, a.t_rel) for a in arrivals])
                self.timer.add("device_round", tend)
            pump.check_integrity()  # the segments' tail checks (device_log synchronised the stream)
            self.device_loop = "arbiter"
        if device_mode:
            stamps = torch.zeros(R + 1, dtype=torch.int64, device=env.device)
            hz = pump.stamp_hz()
            cuts = [start] + ([timed_start] if timed_start is not None and start < timed_start < R else []) + [R]
            for a, b in zip(cuts[:-1], cuts[1:]):
                if timed_start is not None and a == timed_start:
                    t_timed0 = self._timed_fence()
                if cfg.verbose:
                    for i in range(a, b):
                        if i % 10 == 0:
                            log(report.iteration_tick(i))
                arrs = pump.run_local(a, b, device_mode == "graph", stamps)
                arrivals_log.extend(arrs)
            if timed_start is not None:  # the rounds are done: stop the clock before the host bookkeeping
                t_timed1 = self._timed_fence()
            self._sync()
            st = stamps.cpu().numpy().astype(np.float64)
            for i in range(start, R):
                dt = (st[i + 1] - st[i]) / hz  # device time: round i's gradients + the previous update
                timeset[i] = loop_time[i] = dt
                arrivals = [Arrival(w, p, dt) for (w, p, _t) in arrivals_log[i]]
                arrivals_log[i] = [(a.worker, a.part, a.t_rel) for a in arrivals]
                worker_timeset[i] = sch.worker_times(arrivals)
                self.timer.add("device_round", dt)
            self.device_loop = device_mode
        begun = device_mode is not None or arb_mode
        for i in range(start, start if (device_mode or arb_mode) else R):
            if not begun:
                if timed_start is not None and i == timed_start:
                    t_timed0 = self._timed_fence()
                pump.begin(i)
            if cfg.verbose and i % 10 == 0:
                log(report.iteration_tick(i))
            fence_next = timed_start is not None and i + 1 == timed_start
            publish = i + 1 < R and not fence_next
            status, arr, t0, tdec, tend, twait = pump.finish(i, publish)
            arrivals = [Arrival(w, p, t) for (w, p, t) in arr]
            if status == 2:  # completion pattern not in the table yet (timed-out round or a large C(W, s))
                used = sch.decode(arrivals)
                timed_out = len(sch.completed_workers(arrivals)) < self.rule_k
                if table_decoded and not timed_out:
                    mask = sum(1 << w for w in sch.completed_workers(arrivals))
                    coefs = [0.0] * W
                    for (w, p), c in used.items():
                        if p == 0:
                            coefs[w] = float(c)
                    pump.add_table(mask, coefs)
                status, arr, t0, tdec, tend, _ = pump.resolve(i, [(w, p, float(c)) for (w, p), c in used.items()],
                                                              publish)
                timeouts += int(timed_out)
            elif status == 1:
                timeouts += 1
            begun = publish
            self.timer.add("wait_k", twait - t0)
            self.timer.add("decode_update", tdec - twait)
            self.timer.add("drain", tend - tdec)
            timeset[i] = tdec - t0
            loop_time[i] = tend - t0
            worker_timeset[i] = sch.worker_times(arrivals)
            arrivals_log.append([(a.worker, a.part, a.t_rel) for a in arrivals])
            if cfg.checkpoint_every and (i + 1) % cfg.checkpoint_every == 0:
                self._checkpoint(i + 1, timeset, worker_timeset)
        if not device_mode and not arb_mode:
            pump.finish_run()  # lazy drain: a late worker's queued rounds are stale now
        if timed_start is not None and not device_mode and not arb_mode:
            # every rank's rounds are complete once all ranks pass the fence (workers' puts have landed
            # before their barrier); the straggler drain and bookkeeping below are not round time
            t_timed1 = self._timed_fence()
        self._final_drain(col)
        upd = pump.update_ms()
        pump.final_check()  # the last round's mailbox rows (earlier rounds were checked as the run went)
        cut = int(pump.check_rows_cut())
        if cut:  # decodes of more mailbox rows than one check list holds: the rest went unchecked
            why = f"{cut} decoded mailbox rows were past a round's integrity check list and went unchecked"
            print(f"[erasurehead] WARNING: {why}", file=sys.stderr, flush=True)
            self.rank_stats["integrity_unchecked_rows"] = cut
        if not device_mode and not arb_mode:
            timeset[start:] += 1e-3 * np.asarray(upd[start:])
        a0 = timed_start if timed_start is not None else start
        if cfg.instrument:
            put_ms, ker_ms = pump.timing_ms()
            self.rank_stats.update(beta_put_us=_mean_us(put_ms, a0), kernel_us=_mean_us(ker_ms, a0))
        if self.drain_mode != "all":
            self.rank_stats.update(stale_skipped_virtual=col.skipped, stale_arrivals=col.stale_arrivals)
        self.rank_stats.update(update_kernel_us=_mean_us(upd, a0),
                               **{f"{k}_us": float(1e6 * np.mean(v[a0 - start:]))
                                  for k, v in self.timer.t.items() if len(v) > a0 - start})
        if cfg.device_records:
            self.device_records = {"rank": 0, "clock": self._clocks[0] if self._clocks else None,
                                   "beta_put": pump.records().numpy(), "probes": list(pump.probe_log())}
        col.close()
        self._sync()
        self._closing_barrier()
        total = time.perf_counter() - orig_start
        res = TrainResult(self.key, self.hist[:, : self.d].double().cpu().numpy(), timeset, worker_timeset, loop_time,
                          total, timeouts=timeouts, phases=self.timer.summary(), arrivals=arrivals_log)
        if t_timed0 is not None:
            res.timed_seconds = t_timed1 - t_timed0
            res.timed_rounds = R - timed_start
        del pump
        return res

    @staticmethod
    def _shared_gpu(tx) -> bool:
        """Some ranks time-share one GPU (the IPC topology check compares PCI bus ids; other
        transports: never known to share, RCCL refuses it)."""
        pairs = getattr(tx, "pairs", None) or []
        if getattr(tx, "name", "") != "ipc" or not pairs:
            return False
        buses = [p.get("master_bus") for p in pairs[:1]] + [p.get("bus") for p in pairs]
        return len(set(buses)) < len(buses)

    @classmethod
    def _device_waits(cls, tx) -> bool:
        """Stream-side waits on the shared flags (hipStreamWaitValue64): a worker's wait for beta and
        the master's drain before the next beta.  On when every rank has its GPU to itself; ranks
        time-sharing one GPU keep host waits (a queued wait competes with the other ranks' kernels
        there: profiles/round2/s1_worker_wait/).  ERASUREHEAD_WORKER_WAIT=host|device|auto."""
        mode = os.environ.get("ERASUREHEAD_WORKER_WAIT", "auto")
        if getattr(tx, "name", "") != "ipc" or mode == "host":
            return False
        return mode == "device" or (mode == "auto" and not cls._shared_gpu(tx))

    def _worker_loop_native(self, timed_start, start: int = 0) -> None:
        """Worker rounds in csrc/runtime/engine.cpp (WorkerPump) over the IPC mailbox."""
        cfg, env, tx = self.cfg, self.env, self.tx
        R, K = cfg.num_itrs, self.K
        C = native_ext()
        dev = env.device.index if env.device.index is not None else torch.cuda.current_device()
        w = env.world
        dwait = self._device_waits(tx)
        # a worker waits for beta longer than the master's worst round (stop rule + drain, each up to
        # round_timeout), so only a master that is really gone makes it give up
        wait_limit = 2.5 * float(cfg.round_timeout) + 5.0
        if tx.name != "ipc":  # RCCL / loopback p2p: recv(beta) -> gradient -> send, stream-ordered
            pump = C.WorkerPump(self.plan.native_launcher(), tx.inbox, self.G, self.n_loc, tx.comm, K, dev, wait_limit)
        else:
            pump = C.WorkerPump(self.plan.native_launcher(), tx.inbox, self.G, self.n_loc, tx.rremote.ptr,
                                tx.mbox_rows, tx.my_row0, tx.flags.host_addr(env.rank), tx.flags.dev_addr(w + env.rank),
                                tx.counters, K, dev, wait_limit, tx.flags.dev_addr(env.rank) if dwait else 0)
            tagged = pump.set_integrity(tx.mbox_tags_addr(), tx.inbox_tags_addr(), env.rank, bool(cfg.integrity))
            if cfg.integrity and not tagged:  # more message rows than one tagged put holds: loud, recorded
                why = f"rank {env.rank} hosts {self.n_loc} message rows (> 1024 per tagged put): its puts are untagged"
                print(f"[erasurehead] WARNING: {why}", file=sys.stderr, flush=True)
                self.rank_stats["integrity_off"] = why
        pump.set_timing(bool(cfg.instrument))
        pump.set_repeat(self.repeat)
        if tx.name == "ipc":  # landing stamps of this rank's puts, read by the master's collector
            pump.set_stamp_ring(tx.flags.dev_addr(tx.stamp_base + 2 * env.rank * tx.K), tx.K)
        if cfg.device_records:
            pump.set_records(True)
        if self.physical:
            pump.set_delays(self._rank_delays())
        if self.skip_stale and tx.name == "ipc" and self.n_loc:  # stale-round gates read the beta counter
            pump.set_skip_stale(tx.flags.dev_addr(env.rank))
        elif self.skip_stale and tx.name != "ipc":  # p2p: beta received a round ahead, gates from its counter;
            pump.set_skip_stale_comm()  # the end-of-run beta(R) goes to every rank that sends messages
        self.rank_stats["fused_put"] = bool(pump.fused_put)
        self.rank_stats["device_wait"] = bool(pump.device_wait)
        cut = timed_start if timed_start is not None and start <= timed_start < R else None
        segments = [(start, cut), (cut, R)] if cut is not None else [(start, R)]
        gone = _sabotage_exit(env.rank)  # test hook: this worker rank dies / hangs / fails after that round
        if gone is not None:
            pump.run(start, min(R, gone[1]))
            torch.cuda.synchronize(env.device)
            if gone[0] == "raise":
                raise RuntimeError(f"test hook: rank {env.rank} fails at round {gone[1]}")
            if gone[0] == "exit":
                os._exit(0)
            while True:  # silent from here on: the master's drain must give up on it
                time.sleep(1.0)
        t0 = None
        for k, (a, b) in enumerate(segments):
            if k == 1:
                t0 = self._timed_fence()
            bad = pump.run(a, b)
            if bad >= 0:
                raise TimeoutError(f"rank {env.rank}: beta of round {bad} did not arrive within {cfg.round_timeout}s")
        tx.finish()
        if timed_start is not None:
            self.worker_timed_seconds = self._timed_fence() - (t0 if t0 is not None else time.perf_counter())
        self._sync()
        a0 = cut if cut is not None else start
        wait_s, ker_ms, put_ms = pump.timing()
        if cfg.device_records:
            self.device_records = {"rank": env.rank, "clock": self._clocks[env.rank] if self._clocks else None,
                                   "rounds": pump.records().numpy(), "delay_ticks": None}
        self.rank_stats.update(beta_wait_us=_mean_us([1e3 * x if x >= 0 else -1.0 for x in wait_s], a0))
        if pump.skip_stale:
            self.skipped_rounds = list(pump.skipped_rounds())
            self.rank_stats["stale_rounds_skipped"] = len(self.skipped_rounds)
        if cfg.instrument:
            self.rank_stats.update(kernel_us=_mean_us(ker_ms, a0), msg_put_us=_mean_us(put_ms, a0))
        try:
            self._closing_barrier()
        except RuntimeError as e:  # a peer rank is gone (gloo: connection reset): this rank's rounds are done,
            # the master names the lost messages and fails the run (its final drain times out)
            print(f"rank {env.rank}: final barrier failed, a peer rank is gone ({e}); "
                  f"this worker's {R - start} rounds completed", file=sys.stderr, flush=True)
        del pump
        return None

    def _verify_beta_checksums(self, start: int) -> None:
        """Race detector: every worker's beta, before and after its gradient read it,
        must equal the beta the master published for that round."""
        R = self.cfg.num_itrs
        want = self.beta_in[:R].double().sum(1).cpu().numpy()
        got = self.env.gather_objects(None)
        for r in range(1, self.env.world):
            sums = got[r]
            for i in range(start, R):
                if not (sums[i, 0] == want[i] and sums[i, 1] == want[i]):
                    raise RuntimeError(f"beta race detected: rank {r} round {i}: master {want[i]!r}, worker "
                                       f"before/after gradient {sums[i, 0]!r}/{sums[i, 1]!r}")

    def _remote_delays(self, delay_table: np.ndarray) -> np.ndarray:
        """Virtual delays the master's collector applies to REMOTE messages: the injected ones, or
        with physically late worker ranks (--delay-on worker) none but the dead workers'."""
        if not self.physical:
            return delay_table
        return np.where(np.isinf(delay_table), np.inf, 0.0)

    def _rank_delays(self) -> List[float]:
        """Worker rank: seconds it is physically late in every round (0 unless --delay-on worker)."""
        R = self.cfg.num_itrs
        if not self.physical:
            return [0.0] * R
        return [self.delay.rank_delay(i, self.by_rank[self.env.rank]) for i in range(R)]

    def _send_beta(self, i: int):
        if self.tx is not None:
            self.tx.send_beta(i, self.beta_in[i])

    def _post_recvs(self, i: int, slot: int, col: ArrivalCollector, delays):
        if self.tx is not None:
            self.tx.post_recvs(i, slot, col, self.Rbuf, self.remote_msgs, delays, self.physical)

    def _worker_loop(self, timed_start, start: int = 0) -> None:
        cfg, env, tx = self.cfg, self.env, self.tx
        R, K, n = cfg.num_itrs, self.K, self.n_loc
        late = self._rank_delays()
        t0 = None
        bsum = torch.full((R, 2), float("nan"), dtype=torch.float64, device=env.device) if cfg.verify_beta else None
        self.skipped_rounds = []
        gone = _sabotage_exit(env.rank)
        for i in range(start, R):
            if gone is not None and gone[0] == "raise" and i == gone[1]:
                raise RuntimeError(f"test hook: rank {env.rank} fails at round {i}")
            if timed_start is not None and i == timed_start:
                t0 = self._timed_fence()
            slot = i % K
            with self.timer.phase("recv_beta"):
                b = tx.recv_beta(i)
            if bsum is not None:
                bsum[i, 0] = b.double().sum()
            stale = bool(n) and self.skip_stale and tx.stale(i)  # beta(i+1) is already out
            if stale:
                self.skipped_rounds.append(i)
            if n and not stale:
                with self.timer.phase("local_grad"):
                    for _ in range(self.repeat):  # --slow-ranks: a slower GPU
                        self.plan.run(b, self.G[slot])
                if late[i] > 0:  # --delay-on worker: after compute, before the send (ref src/naive.py:141-148)
                    self._sync()
                    time.sleep(late[i])
                with self.timer.phase("send_msgs"):
                    tx.send_msgs(i, self.G[slot, :n])
            if bsum is not None:  # beta must be unchanged after the gradient read it
                bsum[i, 1] = b.double().sum()
        if self.skip_stale and n:
            tx.rounds_done(R)  # every round put or skipped: the master's collector can drain
            self.rank_stats["stale_rounds_skipped"] = len(self.skipped_rounds)
        tx.finish()
        if timed_start is not None:  # same collective order as the master: fence, then the race check
            self.worker_timed_seconds = self._timed_fence() - t0
        if bsum is not None:
            env.gather_objects(bsum.cpu().numpy())
        a0 = (timed_start or 0) - start
        self.rank_stats.update({f"{k}_us": float(1e6 * np.mean(v[a0:])) for k, v in self.timer.t.items()
                                if len(v) > a0})
        self._sync()
        self._closing_barrier()
        return None

    def close(self) -> None:
        """Release transport resources (IPC mappings, shared flags); collective."""
        if self.tx is not None:
            self.env.barrier()
            self.tx.close()
            self.tx = None

    # ------------------------------------------------------------------- checkpointing
    def _restore(self, path: str) -> int:
        """Resume the master from a checkpoint written by :meth:`_checkpoint`; returns the next round.

        Loaded with ``weights_only=True`` (tensors and plain containers only).  The injected
        delays are seeded by the round index (utils/delay.py) and the cyclic code B is
        restored from the checkpoint (:meth:`_checkpoint_B`), so a resumed run draws the same
        delays and decodes with the same code as an uninterrupted one.  What is NOT carried
        over is the virtual lag a straggler carries between rounds in schemes without a drain
        (cyclic, avoidstragg, partial_*): the collector's finish times are wall-clock instants
        of the interrupted process, so the first resumed round starts every worker fresh.
        """
        st = torch.load(path, map_location="cpu", weights_only=True)
        if st.get("scheme") != self.key:
            raise ValueError(f"checkpoint {path} is for scheme {st.get('scheme')!r}, not {self.key!r}")
        nxt = int(st["next_round"])
        if not 0 < nxt <= self.cfg.num_itrs:
            raise ValueError(f"checkpoint next_round {nxt} outside (0, {self.cfg.num_itrs}]")
        ld = self.ld
        if st["beta"].numel() != ld:
            raise ValueError("checkpoint beta has a different feature dimension")
        dev = self.beta.device
        self.beta.copy_(st["beta"].to(dev))
        self.u.copy_(st["u"].to(dev))
        self.hist[:nxt].copy_(st["hist"].to(dev))
        self.beta_in[nxt].copy_(self.beta.to(self.beta_in.dtype))
        self._restored = {"timeset": st["timeset"].numpy(), "worker_timeset": st["worker_timeset"].numpy()}
        return nxt

    @staticmethod
    def _checkpoint_B(path: str) -> Optional[np.ndarray]:
        st = torch.load(path, map_location="cpu", weights_only=True)
        B = st.get("B")
        return None if B is None else B.numpy().astype(np.float64)

    def _checkpoint(self, next_round: int, timeset, worker_timeset):
        path = self.cfg.checkpoint_path or os.path.join(self.cfg.input_dir, "checkpoint.pt")
        state = {"next_round": next_round, "beta": self.beta.cpu(), "u": self.u.cpu(),
                 "hist": self.hist[:next_round].cpu(), "timeset": torch.from_numpy(timeset[:next_round].copy()),
                 "worker_timeset": torch.from_numpy(worker_timeset[:next_round].copy()), "scheme": self.key}
        if getattr(self.scheme, "B", None) is not None:
            state["B"] = torch.from_numpy(np.ascontiguousarray(self.scheme.B, dtype=np.float64))
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
