"""Gradient-coding schemes: data placement, stop rule, decode, naming.

One object per scheme replaces the reference's seven monolithic engine files
(ref src/naive.py, coded.py, replication.py, approximate_coding.py, avoidstragg.py,
partial_replication.py, partial_coded.py).  Each scheme answers four questions the
generic engine (:mod:`erasurehead_amd.engine.trainer`) asks:

  * placement — which data partitions (and label-encoding coefficients) every logical
    worker holds, split into one or two *messages* per round (``part`` 0 = the main /
    coded message sent with tag i, ``part`` 1 = the uncoded "first part" the partial
    schemes send with tag 2R+i, ref src/partial_replication.py:219-227);
  * stop rule — when the master stops waiting (kind + k, see csrc/runtime/collector.h);
  * decode — the fp64 coefficient of every arrived message in the gradient sum;
  * reporting — banner strings and result file names, reference quirks included.

Replication (FRC exact, "EGC" in the README) and approximate coding (AGC) are the
same placement; AGC only adds the ``num_collect`` early stop (the two
reference files differ in 4 lines), so both are :class:`FRC` here.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .cyclic import DecodeCache, make_cyclic_B

# stop-rule kinds (must match csrc/runtime/collector.h)
RULE_ALL, RULE_COUNT, RULE_FRC, RULE_PARTIAL_FRC, RULE_PARTIAL_COUNT = range(5)
# host decode kinds of the native master executor (must match csrc/runtime/engine.cpp DecodeKind)
DEC_SUM, DEC_FIRST_PER_GROUP, DEC_PARTIAL_FRC, DEC_TABLE, DEC_PARTIAL_TABLE = range(5)


class SchemeError(ValueError):
    """Configuration the reference rejects (it prints a message and exits)."""


@dataclass
class Message:
    worker: int  # 0-based logical worker id (reference rank - 1)
    part: int  # 0 main/coded message, 1 uncoded first part (partial schemes)
    segments: List[Tuple[int, float]]  # (0-based partition index, label coefficient)


@dataclass
class Arrival:
    worker: int
    part: int
    t_rel: float


@dataclass
class Scheme:
    key: str
    n_workers: int
    n_stragglers: int
    n_samples: int
    num_collect: int = 0
    n_partitions: int = 0  # partial schemes: partitions per worker (P)
    allow_uneven: bool = False
    rng: Optional[np.random.RandomState] = None
    messages: List[Message] = field(default_factory=list)
    group_of: List[int] = field(default_factory=list)
    n_groups: int = 1
    B: Optional[np.ndarray] = None

    # ---- static properties (overridden) -----------------------------------------
    drain = False  # master Waitall()s the straggler tail before the next round
    has_delay = True  # reference injects the Exp(0.5) delay
    init_zero = False  # beta_0 = zeros (else randn)
    fixed_agd = False  # reference hard-codes AGD regardless of the CLI update rule
    has_linear = False  # reference has a least-squares variant
    needs_B = False
    decode_kind = DEC_SUM
    logs_eval_loading = False  # naive/coded print ">> Loaded j" per dense training partition (ref naive.py:160-164)

    def __post_init__(self):
        if self.n_workers < 1:
            raise SchemeError("need at least one worker")
        if self.n_stragglers < 0:
            raise SchemeError("n_stragglers must be >= 0")
        self._build()

    def _check_s(self):
        if not 0 <= self.n_stragglers < self.n_workers:
            raise SchemeError(f"n_stragglers must be in [0, W), got {self.n_stragglers} with W={self.n_workers}")

    # ---- to implement -----------------------------------------------------------
    def _build(self):
        raise NotImplementedError

    def rule(self) -> Tuple[int, int]:
        raise NotImplementedError

    def decode(self, arrivals: Sequence[Arrival]) -> Dict[Tuple[int, int], float]:
        raise NotImplementedError

    # ---- shared helpers ---------------------------------------------------------
    @property
    def rows_per_partition(self) -> int:
        return self.n_samples // self.n_partition_files

    @property
    def n_partition_files(self) -> int:
        return self.n_workers

    def data_subdir(self) -> str:
        return f"{self.n_workers}/"

    def grad_scale(self) -> float:
        """Multiplier on eta/n (avoidstragg rescales by W/(W-s))."""
        return 1.0

    def messages_of(self, worker: int) -> List[Message]:
        return [m for m in self.messages if m.worker == worker]

    def completed_workers(self, arrivals: Sequence[Arrival]) -> List[int]:
        """Workers whose main message arrived before the stop (the reference's completed_workers)."""
        return sorted({a.worker for a in arrivals if a.part == 0})

    def worker_times(self, arrivals: Sequence[Arrival]) -> np.ndarray:
        """worker_timeset row: arrival time per worker, -1 if not completed (ref src/coded.py:171-173)."""
        row = np.zeros(self.n_workers)
        for a in arrivals:
            row[a.worker] = a.t_rel
        if self.marks_unused:
            done = set(self.completed_workers(arrivals))
            for w in range(self.n_workers):
                if w not in done:
                    row[w] = -1.0
        return row

    marks_unused = True

    def banner(self, add_delay: int) -> str:
        raise NotImplementedError

    def setup_lines(self) -> List[str]:
        return []

    def output_names(self, fix_quirks: bool = False) -> Optional[Dict[str, str]]:
        raise NotImplementedError

    def describe(self) -> str:
        return f"{self.key}(W={self.n_workers}, s={self.n_stragglers})"

    def decode_table(self) -> Dict[int, np.ndarray]:
        """Completion bitmask -> W decode coefficients (table-decoded schemes only).

        Every pattern the stop rule can produce on time (exactly W - s completed main
        messages) is solved up front in fp64 (the reference's getA, ref src/util.py:85-103);
        any other pattern (a round that timed out) is solved on demand by :meth:`decode`.
        """
        import itertools

        W, s = self.n_workers, self.n_stragglers
        out = {}
        for done in itertools.combinations(range(W), W - s):
            mask = 0
            for w in done:
                mask |= 1 << w
            out[mask] = self._decoder(done)
        return out


def _names(prefix: str, train_prefix: Optional[str] = None) -> Dict[str, str]:
    return {
        "training_loss": (train_prefix or prefix) + "training_loss.dat",
        "testing_loss": prefix + "testing_loss.dat",
        "auc": prefix + "auc.dat",
        "timeset": prefix + "timeset.dat",
        "worker_timeset": prefix + "worker_timeset.dat",
    }


class Naive(Scheme):
    """Uncoded data-parallel GD: wait for all W (ref src/naive.py:11-211)."""

    has_linear = True
    marks_unused = False
    logs_eval_loading = True

    def _build(self):
        self.messages = [Message(w, 0, [(w, 1.0)]) for w in range(self.n_workers)]
        self.group_of = list(range(self.n_workers))
        self.n_groups = self.n_workers

    def rule(self):
        return RULE_ALL, self.n_workers

    def decode(self, arrivals):
        return {(a.worker, 0): 1.0 for a in arrivals if a.part == 0}

    def banner(self, add_delay):
        return "---- Starting Naive Iterations ----"

    def output_names(self, fix_quirks=False):
        return _names("naive_acc_")


class Cyclic(Scheme):
    """Exact cyclic-MDS gradient code, wait for W-s (ref src/coded.py:12-257)."""

    init_zero = True
    needs_B = True
    decode_kind = DEC_TABLE
    logs_eval_loading = True

    def _build(self):
        self._check_s()
        W, s = self.n_workers, self.n_stragglers
        if self.B is None:
            self.B = make_cyclic_B(W, s, self.rng)
        self._decoder = DecodeCache(self.B)
        self.messages = [
            Message(w, 0, [((w + i) % W, float(self.B[w, (w + i) % W])) for i in range(s + 1)]) for w in range(W)
        ]
        self.group_of = list(range(W))
        self.n_groups = W

    def set_B(self, B: np.ndarray):
        self.B = np.asarray(B, dtype=np.float64)
        self._build()

    def rule(self):
        return RULE_COUNT, self.n_workers - self.n_stragglers

    def decode(self, arrivals):
        done = self.completed_workers(arrivals)
        a = self._decoder(done)
        return {(w, 0): float(a[w]) for w in done}

    def banner(self, add_delay):
        return "---- Starting Coded Iterations for " + str(self.n_stragglers) + " stragglers ----"

    def output_names(self, fix_quirks=False):
        return _names("coded_acc_%d_" % self.n_stragglers)


class FRC(Scheme):
    """Fractional repetition code; with num_collect < W it is approximate gradient coding.

    Placement (ref src/approximate_coding.py:47-53): group a = w // (s+1), position
    b = w % (s+1), partitions (s+1) a + (b + i) % (s+1).  Stop (ref :144): collect until
    ``num_collect`` workers arrived or every group is covered; the first arrival of each
    group is summed (ref :150-158), uncovered groups contribute zero (inexact gradient).
    The master drains the straggler tail every round (ref :182-183).

    ``allow_uneven`` (extension, off by default): when W % (s+1) != 0 the last group
    simply has W % (s+1) members; the reference exits instead (ref :25-27).
    """

    drain = True
    has_linear = True
    approx = False
    decode_kind = DEC_FIRST_PER_GROUP

    def _build(self):
        self._check_s()
        W, s = self.n_workers, self.n_stragglers
        size = s + 1
        if W % size and not self.allow_uneven:
            raise SchemeError("Error: n_workers must be multiple of n_stragglers+1!")
        self.group_of = [w // size for w in range(W)]
        self.n_groups = (W + size - 1) // size
        self.messages = []
        for w in range(W):
            g = w // size
            first = g * size
            gsize = min(size, W - first)
            b = w - first
            parts = [first + (b + i) % gsize for i in range(gsize)]
            self.messages.append(Message(w, 0, [(p, 1.0) for p in parts]))
        if not self.approx:
            self.num_collect = W

    def rule(self):
        k = self.num_collect if self.num_collect > 0 else self.n_workers
        return RULE_FRC, k

    def decode(self, arrivals):
        used = {}
        covered = set()
        for a in arrivals:  # arrival order
            if a.part != 0:
                continue
            g = self.group_of[a.worker]
            if g not in covered:
                covered.add(g)
                used[(a.worker, 0)] = 1.0
        return used

    def banner(self, add_delay):
        kind = "Approx Coding" if self.approx else "Replication"
        return ("---- Starting " + kind + " Iterations for " + str(self.n_stragglers) + " stragglers"
                + "simulated delay " + str(add_delay) + "-------")

    def output_names(self, fix_quirks=False):
        if self.approx and fix_quirks:
            return _names("approx_acc_%d_%d_" % (self.n_stragglers, self.num_collect))
        return _names("replication_acc_%d_" % self.n_stragglers)  # AGC collides (ref :259-263)


class Replication(FRC):
    """Exact FRC ("EGC" in the README; ref src/replication.py:14-265)."""


class Approx(FRC):
    """Approximate gradient coding = FRC + early stop (ref src/approximate_coding.py:14-266)."""

    approx = True


class AvoidStragg(Scheme):
    """Ignore the s slowest and rescale (ref src/avoidstragg.py:11-209)."""

    init_zero = True
    fixed_agd = True
    has_delay = False

    def _build(self):
        self._check_s()
        self.messages = [Message(w, 0, [(w, 1.0)]) for w in range(self.n_workers)]
        self.group_of = list(range(self.n_workers))
        self.n_groups = self.n_workers

    def rule(self):
        return RULE_COUNT, self.n_workers - self.n_stragglers

    def grad_scale(self):
        W, s = self.n_workers, self.n_stragglers
        return W / (W - s)  # eta / (n (W-s)/W)  (ref :116)

    def decode(self, arrivals):
        return {(a.worker, 0): 1.0 for a in arrivals if a.part == 0}

    def banner(self, add_delay):
        return "---- Starting AvoidStragg Iterations with " + str(self.n_stragglers) + " stragglers ----"

    def output_names(self, fix_quirks=False):
        return _names("avoidstragg_acc_%d_" % self.n_stragglers)


class _Partial(Scheme):
    """Uncoded private part + coded/replicated shared part, two messages per round."""

    init_zero = True
    fixed_agd = True
    has_delay = False

    @property
    def n_separate(self) -> int:
        return self.n_partitions - self.n_stragglers - 1

    @property
    def n_partition_files(self) -> int:
        return (self.n_partitions - self.n_stragglers) * self.n_workers

    def data_subdir(self) -> str:
        return f"partial/{self.n_partition_files}/"

    def setup_lines(self):
        P, s = self.n_partitions, self.n_stragglers
        return ["Stragglers are allowed to be atmost %.2f times slower" % (P * 1.0 / (P - s - 1))]

    def _separate(self, w: int) -> List[Tuple[int, float]]:
        ns = self.n_separate
        return [(i + ns * w, 1.0) for i in range(ns)]

    def _check(self):
        self._check_s()
        if self.n_partitions <= self.n_stragglers + 1:
            raise SchemeError("partial schemes need partitions > n_stragglers + 1")


class PartialReplication(_Partial):
    """ref src/partial_replication.py:11-286 (first part all W + FRC second part)."""

    decode_kind = DEC_PARTIAL_FRC

    def _build(self):
        self._check()
        W, s = self.n_workers, self.n_stragglers
        size = s + 1
        if W % size and not self.allow_uneven:
            raise SchemeError("Error: n_workers must be multiple of n_stragglers+1!")
        ns = self.n_separate
        self.group_of = [w // size for w in range(W)]
        self.n_groups = (W + size - 1) // size
        self.messages = []
        for w in range(W):
            a = w // size
            gsize = min(size, W - a * size)
            shared = [(ns * W + a * size + b, 1.0) for b in range(gsize)]
            self.messages.append(Message(w, 1, self._separate(w)))
            self.messages.append(Message(w, 0, shared))

    def rule(self):
        return RULE_PARTIAL_FRC, self.n_workers

    def decode(self, arrivals):
        used = {}
        covered = set()
        for a in arrivals:
            if a.part == 1:
                used[(a.worker, 1)] = 1.0
            else:
                g = self.group_of[a.worker]
                if g not in covered:
                    covered.add(g)
                    used[(a.worker, 0)] = 1.0
        return used

    def banner(self, add_delay):
        return "---- Starting Partial Replication Iterations for " + str(self.n_stragglers) + " stragglers ----"

    def output_names(self, fix_quirks=False):
        return _names("partialreplication_%d_%d_" % (self.n_stragglers, self.n_partitions))


class PartialCoded(_Partial):
    """ref src/partial_coded.py:12-293 (first part all W + cyclic-coded second part)."""

    needs_B = True
    decode_kind = DEC_PARTIAL_TABLE

    def _build(self):
        self._check()
        W, s = self.n_workers, self.n_stragglers
        if self.B is None:
            self.B = make_cyclic_B(W, s, self.rng)
        self._decoder = DecodeCache(self.B)
        ns = self.n_separate
        self.group_of = list(range(W))
        self.n_groups = W
        self.messages = []
        for w in range(W):
            coded = [(ns * W + (w + j) % W, float(self.B[w, (w + j) % W])) for j in range(s + 1)]
            self.messages.append(Message(w, 1, self._separate(w)))
            self.messages.append(Message(w, 0, coded))

    def set_B(self, B: np.ndarray):
        self.B = np.asarray(B, dtype=np.float64)
        self._build()

    def rule(self):
        return RULE_PARTIAL_COUNT, self.n_workers - self.n_stragglers

    def decode(self, arrivals):
        used = {(a.worker, 1): 1.0 for a in arrivals if a.part == 1}
        done = self.completed_workers(arrivals)
        a = self._decoder(done)
        for w in done:
            used[(w, 0)] = float(a[w])
        return used

    def banner(self, add_delay):
        return "---- Starting Partial Coded Iterations for " + str(self.n_stragglers) + " stragglers ----"

    def output_names(self, fix_quirks=False):
        s, P = self.n_stragglers, self.n_partitions
        train = None if fix_quirks else "partialreplication_%d_%d_" % (s, P)  # ref :286 quirk
        return _names("partialcoded_%d_%d_" % (s, P), train)


SCHEMES = {
    "naive": Naive,
    "coded": Cyclic,
    "replication": Replication,
    "avoidstragg": AvoidStragg,
    "approx": Approx,
    "partial_replication": PartialReplication,
    "partial_coded": PartialCoded,
}


def scheme_key(is_coded: int, partitions: int, coded_ver: int) -> str:
    """Dispatch table of ref main.py:62-92."""
    if not is_coded:
        return "naive"
    if partitions:
        if coded_ver == 1:
            return "partial_replication"
        if coded_ver == 0:
            return "partial_coded"
        raise SchemeError(f"partial schemes need coded_ver 0 or 1, got {coded_ver}")
    table = {0: "coded", 1: "replication", 2: "avoidstragg", 3: "approx"}
    if coded_ver not in table:
        raise SchemeError(f"unknown coded_ver {coded_ver}")
    return table[coded_ver]


def make_scheme(key: str, n_workers: int, n_stragglers: int, n_samples: int, num_collect: int = 0,
                n_partitions: int = 0, allow_uneven: bool = False,
                rng: Optional[np.random.RandomState] = None, B: Optional[np.ndarray] = None) -> Scheme:
    return SCHEMES[key](key=key, n_workers=n_workers, n_stragglers=n_stragglers, n_samples=n_samples,
                        num_collect=num_collect, n_partitions=n_partitions, allow_uneven=allow_uneven, rng=rng, B=B)
