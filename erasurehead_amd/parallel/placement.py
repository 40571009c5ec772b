"""Logical-worker -> process placement.

The reference maps worker w to MPI rank w+1 on its own host.  On an MI355X node the
number of GPUs N and the number of logical workers W are independent: a GPU with 288 GB
of HBM can hold many workers' replicated shards, so every rank hosts a set of logical
workers and computes all of their messages in one kernel launch per round.

Assignment: longest-processing-time greedy on each worker's rows-per-round (the coded
schemes replicate data unevenly, e.g. FRC with a short last group), ties broken by
worker id, so per-GPU work is balanced and deterministic on every rank.
"""
from __future__ import annotations

from typing import Dict, List, Sequence


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


def workers_by_rank(owner: Sequence[int], world: int) -> Dict[int, List[int]]:
    out: Dict[int, List[int]] = {r: [] for r in range(world)}
    for w, r in enumerate(owner):
        out[r].append(w)
    return out
