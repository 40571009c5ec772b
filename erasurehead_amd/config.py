"""Run configuration: the reference's 13 positional arguments + hard-coded constants + extensions.

Positional CLI (ref main.py:20-27):
  n_procs n_rows n_cols input_dir is_real dataset is_coded n_stragglers partitions coded_ver
  num_collect add_delay update_rule
Constants (ref main.py:31-53): num_itrs = 100, alpha = 1/n_rows, eta_i = 10.0 for every round.

Everything past the 13 positionals is an opt-in extension (``--flags`` in cli.py); the
defaults reproduce the reference, including its quirks, unless
``fix_quirks`` is set.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np


@dataclass
class RunConfig:
    n_procs: int
    n_rows: int
    n_cols: int
    input_dir: str
    is_real: int = 0
    dataset: str = "synthetic"
    is_coded: int = 0
    n_stragglers: int = 0
    partitions: int = 0
    coded_ver: int = 0
    num_collect: int = 0
    add_delay: int = 0
    update_rule: str = "GD"

    # ---- reference constants (ref main.py:31-46) ----------------------------------
    num_itrs: int = 100
    alpha: Optional[float] = None  # default 1 / n_rows
    lr: float = 10.0  # learning_rate_schedule = lr * ones(num_itrs)
    lr_schedule: Optional[List[float]] = None
    lr_kind: str = "const"  # const (ref default) | invscaling | exponential (ref main.py:40-46, commented there)
    lr_t0: float = 90.0  # invscaling: eta_i = lr * t0 / (i + t0), i = 1..R
    lr_decay: float = 0.98  # exponential: eta_i = lr * decay**i, i = 1..R (the regression schedule)

    # ---- extensions -----------------------------------------------------------------
    precision: str = "fp64"  # fp64 | fp32 | bf16 worker compute (master state always fp64)
    loss: str = "auto"  # auto (reference dispatch) | logistic | least_squares
    seed: Optional[int] = None  # beta_0 / B matrix seed (reference: unseeded)
    data: str = "files"  # files | synthetic (on-device generator, no files)
    data_seed: int = 0
    allow_uneven_groups: bool = False  # FRC with W % (s+1) != 0
    # straggler tail after the stop rule (engine/trainer.py): None = the scheme's reference behaviour
    # ("all" for FRC/AGC, ref src/approximate_coding.py:182-183; "carry" for the rest, which never
    # Waitall); "all" | "carry" | "lazy" (no wait + stale-round skipping on the workers)
    drain: Optional[str] = None
    delay_mode: str = "exp"  # exp (reference) | fixed | none
    # where an injected delay happens: "collector" (a virtual arrival time on the master's clock, the
    # GPUs never idle) or "worker" (the worker rank is physically late: its messages leave after a
    # device spin / host sleep, after compute and before the send, like the reference's time.sleep)
    delay_on: str = "collector"
    # rank -> factor: that rank runs its gradient `factor` times per round (a physically slower GPU)
    slow_ranks: Dict[int, int] = field(default_factory=dict)
    delay_mean: float = 0.5
    fixed_stragglers: List[int] = field(default_factory=list)  # 1-based worker ids (fixed mode)
    fixed_sleep: float = 0.5
    kill_workers: List[int] = field(default_factory=list)  # 1-based ids that never arrive
    force_delay: bool = False  # inject delays even where the reference does not
    round_timeout: float = 600.0  # master waits at most this long per round (dead worker -> erasure)
    fix_quirks: bool = False
    save_linear: bool = False  # reference comments the linear-model outputs out
    full_precision_outputs: bool = False
    evaluate: bool = True
    verbose: bool = True
    checkpoint_every: int = 0
    checkpoint_path: Optional[str] = None
    resume: Optional[str] = None
    trace: bool = False
    tasks: int = 0  # override gradient-kernel workgroup count
    verify_beta: bool = False  # race detector: workers checksum beta before/after use (Python loop)
    native_loop: bool = True  # GPU rounds in the C++ executors (csrc/runtime/engine.cpp)
    sync_update: bool = False  # host waits for every round's update kernel (else timed by HIP events)
    transport: str = "auto"  # auto | ipc | rccl | gloo (parallel/transport.py)
    device_loop: str = "auto"  # auto|graph|stream|off: device-driven rounds when eligible (trainer._device_loop_mode)
    share_partitions: bool = False  # co-located workers: distinct partitions once + device encode (ops/grad.py)
    # simultaneous arrivals (add_delay = 0, or one kernel finishing several local workers): "permute"
    # orders them by a per-round permutation seeded by (tie_seed, round) (csrc/runtime/collector.h,
    # tie model); "worker" keeps worker-id order (AGC then stops on the same k workers every round)
    tie_break: str = "permute"
    tie_seed: int = 0
    # placement unit: "message" (a logical worker's whole message on one rank), "partition" (one
    # shard per (message, partition): each partition's replicas on one rank; parallel/placement.py)
    # or "auto" (partition when there are several ranks)
    shard: str = "auto"
    instrument: bool = False  # per-round HIP-event timing of puts / gradient launches (Trainer.rank_report)
    # IPC messages carry (round, rank, checksum) tags that the receiver verifies (csrc/kernels/integrity.h)
    integrity: bool = True
    # the reference topology's master: rank 0 runs the master only and hosts no logical worker (worker
    # w on rank 1 + w mod (world - 1); ref main.py:16-18, run_approx_coding.sh:47-49).  Default: rank 0
    # hosts workers too (one process per GPU, no GPU idles)
    dedicated_master: bool = False
    # per-round device records of every rank (beta put / message put / spin / gate stamps on the GPU
    # clocks) and the master's probe log, kept as Trainer.device_records (tests/lazy_check.py)
    device_records: bool = False

    def __post_init__(self):
        self.update_rule = str(self.update_rule)
        if self.update_rule not in ("GD", "AGD"):
            raise ValueError("update_rule must be GD or AGD")  # ref src/naive.py:13 assert
        self.input_dir = self.input_dir if self.input_dir.endswith("/") else self.input_dir + "/"
        if self.tie_break not in ("permute", "worker"):
            raise ValueError("tie_break must be permute or worker")
        if self.delay_mode == "worker":  # shorthand: the reference's Exp delays, slept on the worker rank
            self.delay_mode, self.delay_on = "exp", "worker"
        if self.delay_on not in ("collector", "worker"):
            raise ValueError("delay_on must be collector or worker")
        if self.drain not in (None, "all", "carry", "lazy"):
            raise ValueError("drain must be all, carry or lazy")
        if any(int(f) < 1 for f in self.slow_ranks.values()):
            raise ValueError("slow rank factors must be integers >= 1")

    @property
    def tie_seed_value(self) -> int:
        return int(self.tie_seed) if self.tie_break == "permute" else -1

    @property
    def n_workers(self) -> int:
        return self.n_procs - 1

    @property
    def alpha_value(self) -> float:
        return 1.0 / self.n_rows if self.alpha is None else self.alpha

    def eta(self) -> np.ndarray:
        if self.lr_schedule is not None:
            s = np.asarray(self.lr_schedule, dtype=np.float64)
            if len(s) < self.num_itrs:
                raise ValueError("lr_schedule shorter than num_itrs")
            return s
        i = np.arange(1, self.num_itrs + 1, dtype=np.float64)
        if self.lr_kind == "const":
            return self.lr * np.ones(self.num_itrs)
        if self.lr_kind == "invscaling":
            return self.lr * self.lr_t0 / (i + self.lr_t0)
        if self.lr_kind == "exponential":
            return self.lr * self.lr_decay ** i
        raise ValueError(f"unknown lr schedule {self.lr_kind!r}")
