"""Straggler / fault injection model.

Reference (ref src/naive.py:141-148, also coded/replication/approximate_coding):
    if add_delay == 1:
        np.random.seed(seed=i); artificial_delays = np.random.exponential(0.5, n_workers)
        time.sleep(artificial_delays[rank-1])          # after compute, before the send
Every worker seeds with the round index, so all draw the same vector: the pattern is
deterministic.  ``RandomState(i).exponential`` reproduces that stream exactly.

Extra modes (opt-in): ``fixed`` (the commented variant at ref src/naive.py:143-145: a
fixed set of workers sleeps ``fixed_sleep``), ``kill`` (workers that never arrive: the
master's round timeout turns them into erasures instead of hanging).
The delay is applied as a virtual arrival time by the native collector (see
csrc/runtime/collector.h) so the GPUs never idle in ``sleep``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List

import numpy as np


@dataclass
class DelayModel:
    n_workers: int
    mode: str = "none"  # none | exp | fixed
    mean: float = 0.5
    fixed_workers: List[int] = field(default_factory=list)  # 0-based
    fixed_sleep: float = 0.5
    dead: List[int] = field(default_factory=list)  # 0-based

    def delays(self, i: int) -> np.ndarray:
        """Delay (seconds) of every worker in round i."""
        W = self.n_workers
        if self.mode == "exp":
            d = np.random.RandomState(seed=i).exponential(self.mean, W)
        elif self.mode == "fixed":
            d = np.zeros(W)
            d[list(self.fixed_workers)] = self.fixed_sleep
        else:
            d = np.zeros(W)
        for w in self.dead:
            d[w] = math.inf
        return d

    # ---- physically late worker ranks (--delay-on worker) -------------------------------------
    # A worker rank is one process on one GPU: it sends all of its messages together, after
    # compute, so it is late by the LARGEST delay among the logical workers it hosts (with one
    # logical worker per rank, --shard message with ranks = workers, this is exactly the
    # reference's per-worker sleep).  Dead workers (inf) stay virtual erasures on the master.
    # The master's own co-located workers keep their per-worker delay on the collector's clock.
    def rank_delay(self, i: int, workers) -> float:
        """Seconds worker rank hosting `workers` (logical worker ids) sleeps in round i."""
        d = self.delays(i)
        vals = [float(d[w]) for w in workers if math.isfinite(d[w])]
        return max(vals) if vals else 0.0

    def equivalent(self, i: int, hosts) -> np.ndarray:
        """Per-worker delay of round i that the virtual collector model needs to reproduce the
        physical schedule: hosts = {rank: logical workers with messages (or shards) on it}.  A
        worker's message is complete when its last shard lands, i.e. at the max over its ranks."""
        d = self.delays(i)
        out = np.zeros_like(d)
        for r, ws in hosts.items():
            dr = self.rank_delay(i, ws) if r != 0 else None
            for w in ws:
                v = d[w] if (r == 0 or not math.isfinite(d[w])) else dr
                out[w] = max(out[w], v)
        return out


def delay_floor(n_workers: int, rounds: int, stop_count=None, groups=None, k=None, mean=0.5,
                carry: bool = False) -> float:
    """Sum over rounds of the injected delay the master must wait for.

    stop_count: wait for the `stop_count`-th smallest delay (naive: W, cyclic: W-s).
    groups/k:   FRC/AGC rule — stop at k arrivals or when every group is covered.
    carry:      schemes that do not drain (cyclic, avoidstragg): a straggler still busy with
                round i-1 starts round i late (the collector's
                ready = max(t_start, finish(w, i-1)) + delay), so the floor is the exact
                zero-compute replay of that timeline instead of the per-round order statistic.
    """
    if carry:
        return _carried_floor(n_workers, rounds, stop_count, groups, k, mean)
    tot = 0.0
    for i in range(rounds):
        d = np.random.RandomState(seed=i).exponential(mean, n_workers)
        order = np.argsort(d, kind="stable")
        if groups is None:
            tot += float(np.sort(d)[stop_count - 1])
            continue
        covered = set()
        cnt = 0
        t = 0.0
        n_groups = len(set(groups))
        for w in order:
            t = d[w]
            cnt += 1
            covered.add(groups[w])
            if cnt >= k or len(covered) >= n_groups:
                break
        tot += float(t)
    return tot


def schedule(delays: np.ndarray, rule: str, k: int, groups, drain: str = "lazy", compute: float = 0.0,
             margin: float = 0.0):
    """Event model of the master's rounds under ``drain`` with per-round worker delays [R, W].

    The master publishes beta(i) at t_i (t_0 = 0) and decides round i when the stop rule holds over
    the arrivals sorted by time (rule: "all" | "count" (k arrivals) | "frc" (k arrivals or every
    group covered)); decode and update take no time, so t_{i+1} = that stop time, or, with drain
    "all", the last arrival.  Worker w, free from F_w on (its previous put), starts round i at
    s = max(t_i, F_w) and its message lands at s + compute + d[i, w]:
      * "all" / "carry": every round runs (carry: lag crosses rounds, the reference's no-Waitall
        schemes, the collector's carried finish);
      * "lazy": a worker not free before t_{i+1} skips round i (its gate finds beta(i+1) out:
        csrc/kernels/common.h gate_closed, the collector's stale-round skipping).
    Returns (arrivals, separated): arrivals[i] = worker ids in arrival order up to the stop (the
    decode's inputs), separated[i] = every event the round's outcome depends on (arrival order near
    the stop, a busy worker's start against t_{i+1}) is more than ``margin`` apart -- the rounds a
    physical run with timing noise below the margin must reproduce exactly.
    """
    out, sep, _, _ = _run_schedule(delays, rule, k, groups, drain, compute, margin)
    return out, sep


def schedule_floors(delays: np.ndarray, rule: str, k: int, groups, drain: str = "lazy", compute: float = 0.0):
    """(Σ time-to-decode, Σ round length) in seconds of :func:`schedule`'s event model: the floors of a
    run's Σtimeset and of its loop wall-clock under ``drain`` (zero compute: the injected delays alone).
    drain "all": a round lasts until its last arrival, its decode happens at the stop; "carry" / "lazy":
    the next beta leaves at the stop, so both sums are equal."""
    _, _, dec, rnd = _run_schedule(delays, rule, k, groups, drain, compute, 0.0)
    return float(np.sum(dec)), float(np.sum(rnd))


def _run_schedule(delays, rule, k, groups, drain, compute, margin):
    delays = np.asarray(delays, dtype=np.float64)
    R, W = delays.shape
    n_groups = len(set(groups))
    F = np.full(W, -np.inf)
    t = 0.0
    out, sep, dec, rnd = [], [], [], []
    for i in range(R):
        s = np.maximum(t, F)
        a = s + compute + delays[i]
        order = sorted(range(W), key=lambda w: (a[w], w))
        got, cov = [], set()
        t_stop = np.inf
        for w in order:
            if not np.isfinite(a[w]):
                break
            got.append(w)
            cov.add(groups[w])
            if (rule == "all" and len(got) == W) or (rule == "count" and len(got) >= k) or \
                    (rule == "frc" and (len(got) >= k or len(cov) == n_groups)):
                t_stop = a[w]
                break
        t_next = t_stop if drain != "all" else float(np.max(a[np.isfinite(a)]))
        ok = True
        fin = np.sort(a[np.isfinite(a)])
        if margin > 0 and fin.size > 1:
            # the order up to (and one past) the stop must be unambiguous
            near = fin[: min(len(fin), len(got) + 1)]
            ok = bool(np.all(np.diff(near) > margin))
        for w in range(W):
            runs = drain != "lazy" or F[w] <= t or s[w] < t_next  # free at t_i: it starts at once
            if drain == "lazy" and margin > 0 and F[w] > t and abs(s[w] - t_next) <= margin:
                ok = False  # a busy worker's skip decision is within the noise
            if runs:
                F[w] = a[w]
        out.append(got)
        sep.append(ok)
        dec.append(t_stop - t)
        rnd.append(t_next - t)
        t = t_next
    return out, sep, dec, rnd


def _carried_floor(n_workers, rounds, stop_count, groups, k, mean) -> float:
    finish = np.zeros(n_workers)  # virtual finish of every worker's latest message
    t = 0.0  # start of the current round (= decode of the previous one, zero compute)
    tot = 0.0
    n_groups = len(set(groups)) if groups is not None else 0
    for i in range(rounds):
        d = np.random.RandomState(seed=i).exponential(mean, n_workers)
        ready = np.maximum(t, finish) + d
        finish = ready
        order = np.argsort(ready, kind="stable")
        if groups is None:
            t_stop = float(ready[order[stop_count - 1]])
        else:
            covered, cnt = set(), 0
            for w in order:
                t_stop = float(ready[w])
                cnt += 1
                covered.add(groups[w])
                if cnt >= k or len(covered) >= n_groups:
                    break
        tot += t_stop - t
        t = t_stop
    return tot
