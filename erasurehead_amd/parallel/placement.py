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

Two placements of multi-rank runs, a deliberate trade-off:

* ``message`` (default for training): whole messages dealt round-robin over the ranks
  (``place_spread``), the reference's one-worker-per-process topology.  A slow or dead GPU
  erases only its own workers' messages, which the gradient code tolerates.
* ``partition`` (benchmark opt-in): a logical message (worker, part) reads s+1 partitions.
  Placing whole messages caps strong scaling — at W = 8 on 8 GPUs every GPU still streams its
  worker's 3 partitions per round.  ``make_shards(messages, "partition")`` splits every message
  into one shard per partition; ``place_units`` then keeps the shards of one partition (all its
  replicas) together, so each GPU streams its partitions once and computes every replica's
  segment gradient from those rows (no replica's work is skipped).  The master sums a message's
  shards with the decode coefficient, and the collector counts the message as arrived when its
  last shard is ready (csrc/runtime/collector.h).  The price: every replica of a partition now
  lives on ONE rank, so a physically slow GPU delays every message that has a shard there (at
  N = 8, most of them) and the code's redundancy protects nothing physical.  The injected
  straggler model is unaffected when it is virtual (--delay-on collector), not when a rank is
  really late (--delay-on worker, --slow-ranks).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass(frozen=True)
class Shard:
    """A placed unit of work: all (shard = 0, n_shards = 1) or one partition of message (worker, part)."""
    worker: int
    part: int
    segments: Tuple[Tuple[int, float], ...]
    shard: int = 0
    n_shards: int = 1


def make_shards(messages, mode: str = "message") -> List[Shard]:
    """One Shard per message ("message") or per (message, partition) ("partition")."""
    out: List[Shard] = []
    for m in messages:
        segs = tuple((int(p), float(c)) for p, c in m.segments)
        if mode == "partition" and len(segs) > 1:
            out += [Shard(m.worker, m.part, (sg,), k, len(segs)) for k, sg in enumerate(segs)]
        elif mode in ("message", "partition"):
            out.append(Shard(m.worker, m.part, segs))
        else:
            raise ValueError(f"unknown shard mode {mode!r}")
    return out


def place_spread(workers: Sequence[int], world: int) -> List[int]:
    """owner[u] = worker(u) mod world: the reference topology compressed onto `world` ranks.

    The reference runs every logical worker in its own process (worker w on MPI rank w+1, ref
    src/approximate_coding.py:47-53, run_approx_coding.sh:47-49), so a slow or dead machine
    erases exactly one worker's message and the gradient code's redundancy covers it.  Dealing
    workers round-robin keeps that property on fewer GPUs: the members of an FRC group and cyclic
    neighbours (consecutive worker ids) land on different ranks whenever world >= s + 1, so one
    slow GPU delays at most ceil(W / world) workers, never all replicas of a partition.  This is
    the default placement of multi-rank training runs; partition shards (place_units) trade that
    tolerance for bandwidth and are a benchmark opt-in.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    return [int(w) % world for w in workers]


def place_units(parts: Sequence[Sequence[Tuple[int, int]]], world: int, replica_weight: float) -> List[int]:
    """owner[u] for placement units (messages or shards), sharing-aware.

    Starts from an LPT placement of *partition bundles* (the units whose first partition is the
    same, costed with the sharing model) so replicas start out together, then refines with
    :func:`place_workers_shared`'s moves and swaps.
    """
    U = len(parts)
    if world <= 1:
        return [0] * U
    bundles: Dict[int, List[int]] = {}
    for u in range(U):
        key = parts[u][0][0] if parts[u] else -1 - u
        bundles.setdefault(key, []).append(u)
    keys = list(bundles)
    bcost = [rank_cost(bundles[k], parts, replica_weight) for k in keys]
    border = place_workers(bcost, world)
    init = [0] * U
    for b, k in enumerate(keys):
        for u in bundles[k]:
            init[u] = border[b]
    return place_workers_shared(parts, world, replica_weight, init=init)


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
                         replica_weight: float, init: Optional[Sequence[int]] = None) -> List[int]:
    """owner[w] minimising (max rank cost, idle ranks, total cost) with the sharing-aware cost model.

    Starts from the LPT placement on message rows and improves it by single-worker moves and
    pairwise swaps (first improvement, fixed scan order): deterministic on every rank.  With
    replica_weight = 1 nothing is shared and the result balances message rows like LPT.
    """
    W = len(parts)
    if world <= 1:
        return [0] * W
    owner = list(init) if init is not None else place_workers([float(sum(n for _, n in parts[w])) for w in range(W)],
                                                             world)

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
