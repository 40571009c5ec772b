"""Check a lazy-drain run of the CPU / gloo Python loop (host sleeps, no device clock) against the
event model of utils/delay.py ``schedule``, replayed ALONG THE OBSERVED TRAJECTORY.  The GPU runs are
checked against the ranks' own device records instead (tests/lazy_check.py), with no model.

A physical run has timing noise, so a free-running model drifts away from it after the first
close call.  Here the model is re-anchored every round: the master's observed round starts t_i
(cumulative loop times) and the worker ranks' observed skip decisions drive it, and only the
decisions the model can call with a margin are compared:

  * the decode's inputs of round i -- the set of arrivals up to the stop and, for FRC / AGC, the
    first arrival of every group -- on rounds whose stop boundary and within-group order are more
    than ``margin`` apart;
  * every worker rank's skip decision (skip iff still busy when beta(i+1) was out) where its
    start and t_{i+1} are more than ``margin`` apart.
"""
import numpy as np


def replay_along(delays, t, ran, rule, k, groups, margin):
    """delays [R, W]; t [R + 1] observed round starts (t[0] = 0); ran[i][w] = observed (True: ran,
    False: skipped) or None (the model decides: the master's own virtual workers)."""
    delays = np.asarray(delays, dtype=np.float64)
    R, W = delays.shape
    n_groups = len(set(groups))
    F = np.full(W, -np.inf)
    out = []
    for i in range(R):
        s = np.maximum(t[i], F)
        model_runs = (F <= t[i]) | (s < t[i + 1])
        ambiguous = (F > t[i]) & (np.abs(s - t[i + 1]) <= margin)
        runs = np.array([model_runs[w] if ran[i][w] is None else bool(ran[i][w]) for w in range(W)])
        a = np.where(runs, s + delays[i], np.inf)
        order = sorted(range(W), key=lambda w: (a[w], w))
        got, cov, m = [], set(), None
        for idx, w in enumerate(order):
            if not np.isfinite(a[w]):
                break
            got.append(w)
            cov.add(groups[w])
            if (rule == "all" and len(got) == W) or (rule == "count" and len(got) >= k) or \
                    (rule == "frc" and (len(got) >= k or len(cov) == n_groups)):
                m = idx
                break
        sep = m is not None and (m + 1 >= W or not np.isfinite(a[order[m + 1]])
                                 or a[order[m + 1]] - a[order[m]] > margin)
        if sep and rule == "frc":
            for g in set(groups):
                mem = sorted((a[w] for w in got if groups[w] == g))
                if len(mem) >= 2 and mem[1] - mem[0] <= margin:
                    sep = False
        out.append({"pred": got, "sep": bool(sep), "model_runs": model_runs, "ambiguous": ambiguous, "runs": runs})
        F[runs] = a[runs]
    return out


def decode_key(workers, rule, groups):
    """What the decode depends on: the arrived set (its membership drives the stop rule and the workers'
    times), and for FRC / AGC also the first arrival of each covered group -- the order of a covered
    group's later members against another group's first arrival does not enter the decode, so only that
    ordering is relaxed, never the membership."""
    if rule != "frc":
        return (sorted(workers), None)
    first = {}
    for w in workers:
        first.setdefault(groups[w], w)
    return (sorted(workers), sorted(first.items()))


def check_lazy(arrivals, loop_time, delays, rule, k, groups, margin, skipped_by_worker=None, local=()):
    """arrivals[i] = observed worker ids in arrival order; skipped_by_worker = {w: rounds its rank
    skipped} for the workers on physically late ranks (the others are modelled).  Returns (rounds
    compared, skip decisions compared)."""
    R, W = np.asarray(delays).shape
    t = np.concatenate([[0.0], np.cumsum(np.asarray(loop_time, dtype=np.float64)[:R])])
    ran = [[None] * W for _ in range(R)]
    if skipped_by_worker is not None:
        for w, sk in skipped_by_worker.items():
            if w in local:
                continue
            for i in range(R):
                ran[i][w] = i not in set(sk)
    rounds = replay_along(delays, t, ran, rule, k, groups, margin)
    n_rounds = n_skips = 0
    for i, r in enumerate(rounds):
        if r["sep"]:
            assert decode_key(list(arrivals[i]), rule, groups) == decode_key(r["pred"], rule, groups), \
                (i, list(arrivals[i]), r["pred"], t[i], np.asarray(delays)[i])
            n_rounds += 1
        for w in range(W):
            if ran[i][w] is not None and not r["ambiguous"][w]:
                assert bool(ran[i][w]) == bool(r["model_runs"][w]), (i, w, ran[i][w], t[i], t[i + 1])
                n_skips += 1
    return n_rounds, n_skips
