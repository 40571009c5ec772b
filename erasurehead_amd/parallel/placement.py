"""Logical-worker -> process placement.

The reference maps worker w to MPI rank w+1 on its own host.  On an MI355X node the
number of GPUs N and the number of logical workers W are independent: a GPU with 288 GB
of HBM can hold many workers' replicated shards, so every rank hosts a set of logical
workers and computes all of their messages in one kernel launch per round.

Assignment (deterministic on every rank): `place_workers` is longest-processing-time greedy
on each worker's rows-per-round (the coded schemes replicate data unevenly, e.g. FRC with a
short last group).  `place_workers_shared` refines it for GPUs, where workers that read the
same partitions share HBM reads (LDS-staged bundles / interleaved dispatch), so keeping an FRC group or
cyclic neighbours together costs less than their message rows suggest.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple


def place_workers(costs: Sequence[float], world: int) -> List[int]:
    """owner[w] in [0, world) minimising the max per-rank cost (LPT greedy)."""
    W = len(costs)
    if world <= 0:
        raise ValueError("world must be >= 1")
    if world == 1:
        return [0] * W
    if W % world == 0 and len(set(costs)) == 1:
        per = W // world
        return [w // per for w in range(W)]
    load = [0.0] * world
    owner = [0] * W
    for w in sorted(range(W), key=lambda w: (-costs[w], w)):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[w] = r
        load[r] += costs[w]
    return owner


def rank_cost(workers: Sequence[int], parts: Sequence[Sequence[Tuple[int, int]]], replica_weight: float) -> float:
    """Estimated per-round work of one rank hosting `workers`.

    parts[w] = [(partition, rows), ...] read by worker w's messages.  Rows of a partition read
    by several co-located messages are streamed from HBM once (LDS-staged replica bundles, or
    replica tasks co-scheduled on one XCD: ops/grad.py); each further message over them costs
    `replica_weight` of a distinct row (measured ≈ 0.12 for dense fp64 on MI355X with the staged
    bundles, 0.25 with the interleaved dispatch, 1 where nothing is shared, 0 with
    --share-partitions).
    """
    distinct: Dict[int, int] = {}
    total = 0
    for w in workers:
        for p, n in parts[w]:
            distinct[p] = n
            total += n
    d = sum(distinct.values())
    return d + replica_weight * (total - d)


def place_workers_shared(parts: Sequence[Sequence[Tuple[int, int]]], world: int,
                         replica_weight: float) -> List[int]:
    """owner[w] minimising (max rank cost, idle ranks, total cost) with the sharing-aware cost model.

    Starts from the LPT placement on message rows and improves it by single-worker moves and
    pairwise swaps (first improvement, fixed scan order): deterministic on every rank.  With
    replica_weight = 1 nothing is shared and the result balances message rows like LPT.
    """
    W = len(parts)
    if world <= 1:
        return [0] * W
    owner = place_workers([float(sum(n for _, n in parts[w])) for w in range(W)], world)

    def costs(own):
        by = workers_by_rank(own, world)
        return [rank_cost(by[r], parts, replica_weight) for r in range(world)]

    def key(c):  # (slowest rank, idle GPUs, total work): never leave a GPU idle for nothing
        return (round(max(c), 9), sum(1 for x in c if x == 0), round(sum(c), 9))

    best = key(costs(owner))
    improved = True
    while improved:
        improved = False
        for w in range(W):
            for r in range(world):
                if r == owner[w]:
                    continue
                trial = list(owner)
                trial[w] = r
                k = key(costs(trial))
                if k < best:
                    owner, best, improved = trial, k, True
        for a in range(W):
            for b in range(a + 1, W):
                if owner[a] == owner[b]:
                    continue
                trial = list(owner)
                trial[a], trial[b] = owner[b], owner[a]
                k = key(costs(trial))
                if k < best:
                    owner, best, improved = trial, k, True
    return owner


def workers_by_rank(owner: Sequence[int], world: int) -> Dict[int, List[int]]:
    out: Dict[int, List[int]] = {r: [] for r in range(world)}
    for w, r in enumerate(owner):
        out[r].append(w)
    return out
