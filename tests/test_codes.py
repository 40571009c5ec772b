"""Coding theory: cyclic MDS decodability, FRC placement invariants, stop rules, naming."""
import itertools

import numpy as np
import pytest

from erasurehead_amd.codes import (Arrival, DecodeCache, SchemeError, decode_error, make_cyclic_B, make_scheme,
                                   pattern_index, scheme_key)
from erasurehead_amd.codes.schemes import RULE_ALL, RULE_COUNT, RULE_FRC, RULE_PARTIAL_COUNT, RULE_PARTIAL_FRC


@pytest.mark.parametrize("W,s", [(2, 1), (4, 1), (6, 2), (8, 2), (8, 3), (5, 4)])
def test_cyclic_every_pattern_decodes(W, s):
    B = make_cyclic_B(W, s, np.random.RandomState(W * 10 + s))
    S = (np.arange(W)[:, None] + np.arange(s + 1)[None, :]) % W
    for i in range(W):  # support + unit diagonal (ref src/util.py:74-81)
        assert B[i, i] == 1.0
        assert set(np.flatnonzero(B[i])) <= set(S[i])
    for stragglers in itertools.combinations(range(W), s):
        done = [w for w in range(W) if w not in stragglers]
        assert decode_error(B, done) < 1e-8


def test_decode_cache_matches_getA_order():
    W, s = 6, 2
    B = make_cyclic_B(W, s, np.random.RandomState(0))
    dc = DecodeCache(B)
    A = dc.precompute_all(s)
    assert A.shape == (15, W)
    for row, pos in zip(A, itertools.combinations(range(W), s)):
        assert np.all(row[list(pos)] == 0)
        assert np.max(np.abs(row @ B - 1)) < 1e-9
    assert dc([0, 1, 2, 3]) is dc([3, 2, 1, 0])  # cached by bitmask


def test_pattern_index_is_a_bijection():
    W, k = 6, 4
    seen = set()
    for comb in itertools.combinations(range(W), k):
        mask = [w in comb for w in range(W)]
        seen.add(pattern_index(mask))
    assert len(seen) == 15


def test_frc_placement_reference_layout():
    sch = make_scheme("replication", 6, 2, 600)
    # W=6, s=2: workers 0,1,2 hold {0,1,2} rotated; 3,4,5 hold {3,4,5}
    parts = [[p for p, _ in m.segments] for m in sch.messages]
    assert parts == [[0, 1, 2], [1, 2, 0], [2, 0, 1], [3, 4, 5], [4, 5, 3], [5, 3, 4]]
    assert sch.group_of == [0, 0, 0, 1, 1, 1] and sch.n_groups == 2
    assert sch.rule() == (RULE_FRC, 6)


def test_frc_requires_divisibility_unless_uneven():
    with pytest.raises(SchemeError, match="multiple of n_stragglers"):
        make_scheme("approx", 8, 2, 800, num_collect=6)
    sch = make_scheme("approx", 8, 2, 800, num_collect=6, allow_uneven=True)
    assert sch.n_groups == 3 and sch.group_of == [0, 0, 0, 1, 1, 1, 2, 2]
    parts = [sorted(p for p, _ in m.segments) for m in sch.messages]
    assert parts[6] == parts[7] == [6, 7]
    covered = set()
    for g in range(3):  # one member per group covers every partition exactly once
        w = sch.group_of.index(g)
        covered |= set(parts[w])
    assert covered == set(range(8))


def test_agc_decode_first_per_group_and_stop():
    sch = make_scheme("approx", 6, 1, 600, num_collect=2)
    arr = [Arrival(1, 0, 0.1), Arrival(0, 0, 0.2), Arrival(4, 0, 0.3)]
    used = sch.decode(arr)
    assert used == {(1, 0): 1.0, (4, 0): 1.0}  # group 0 first = worker 1; group 2 = worker 4; group 1 uncovered
    assert sch.rule() == (RULE_FRC, 2)
    row = sch.worker_times(arr)
    assert list(row) == [0.2, 0.1, -1, -1, 0.3, -1]


def test_cyclic_decode_recovers_full_gradient():
    W, s = 5, 2
    sch = make_scheme("coded", W, s, 500, rng=np.random.RandomState(3))
    rng = np.random.RandomState(0)
    gp = rng.randn(W, 7)  # per-partition gradients
    msgs = {m.worker: sum(c * gp[p] for p, c in m.segments) for m in sch.messages}
    arr = [Arrival(w, 0, 0.0) for w in (4, 0, 2)]
    used = sch.decode(arr)
    g = sum(c * msgs[w] for (w, _), c in used.items())
    np.testing.assert_allclose(g, gp.sum(0), rtol=1e-9, atol=1e-9)
    assert sch.rule() == (RULE_COUNT, 3)


def test_partial_placements():
    W, s, P = 4, 1, 4
    pr = make_scheme("partial_replication", W, s, 1200, n_partitions=P)
    assert pr.n_partition_files == (P - s) * W == 12 and pr.data_subdir() == "partial/12/"
    assert pr.rule() == (RULE_PARTIAL_FRC, W)
    m = {(x.worker, x.part): [p for p, _ in x.segments] for x in pr.messages}
    assert m[(0, 1)] == [0, 1] and m[(3, 1)] == [6, 7]  # n_separate = 2 private partitions each
    assert m[(0, 0)] == m[(1, 0)] == [8, 9] and m[(2, 0)] == [10, 11]
    pc = make_scheme("partial_coded", W, s, 1200, n_partitions=P, rng=np.random.RandomState(1))
    assert pc.rule() == (RULE_PARTIAL_COUNT, W - s)
    m = {(x.worker, x.part): x.segments for x in pc.messages}
    assert [p for p, _ in m[(3, 0)]] == [11, 8]
    assert m[(3, 0)][1][1] == pytest.approx(pc.B[3, 0])
    names = pc.output_names()
    assert names["training_loss"] == "partialreplication_1_4_training_loss.dat"  # ref partial_coded.py:286
    assert names["auc"] == "partialcoded_1_4_auc.dat"


def test_dispatch_table_and_names():
    assert scheme_key(0, 0, 3) == "naive"
    assert scheme_key(1, 0, 0) == "coded"
    assert scheme_key(1, 0, 1) == "replication"
    assert scheme_key(1, 0, 2) == "avoidstragg"
    assert scheme_key(1, 0, 3) == "approx"
    assert scheme_key(1, 3, 1) == "partial_replication"
    assert scheme_key(1, 3, 0) == "partial_coded"
    assert make_scheme("approx", 4, 1, 40, 3).output_names()["timeset"] == "replication_acc_1_timeset.dat"
    assert make_scheme("naive", 4, 1, 40).output_names()["worker_timeset"] == "naive_acc_worker_timeset.dat"
    assert make_scheme("avoidstragg", 4, 1, 40).grad_scale() == pytest.approx(4 / 3)
    assert make_scheme("naive", 3, 0, 30).rule() == (RULE_ALL, 3)


def test_banners_verbatim():
    assert make_scheme("approx", 4, 1, 40, 3).banner(1) == \
        "---- Starting Approx Coding Iterations for 1 stragglerssimulated delay 1-------"
    assert make_scheme("replication", 4, 1, 40).banner(0) == \
        "---- Starting Replication Iterations for 1 stragglerssimulated delay 0-------"
    assert make_scheme("coded", 4, 1, 40).banner(0) == "---- Starting Coded Iterations for 1 stragglers ----"
    assert make_scheme("avoidstragg", 4, 1, 40).banner(0) == "---- Starting AvoidStragg Iterations with 1 stragglers ----"
    assert make_scheme("partial_replication", 4, 1, 40, n_partitions=3).setup_lines() == \
        ["Stragglers are allowed to be atmost 3.00 times slower"]


def test_replica_dispatch_order_coschedules_replicas_on_one_xcd():
    """Tasks that read identical rows are placed 8 dispatch slots apart (same XCD), none is lost."""
    from erasurehead_amd.ops.grad import XCDS, replica_dispatch_order

    # headline-like layout: 3 replicas of partitions 0..5, 2 replicas of 6..7, 10 row chunks each
    keys = []
    groups = [[0, 1, 2]] * 3 + [[3, 4, 5]] * 3 + [[6, 7]] * 2
    for parts in groups:
        for p in parts:
            keys += [(p, r) for r in range(10)]
    order = replica_dispatch_order(keys)
    assert sorted(order) == list(range(len(keys)))
    pos = {t: i for i, t in enumerate(order)}
    by_key = {}
    for i, k in enumerate(keys):
        by_key.setdefault(k, []).append(pos[i])
    aligned = sum(1 for v in by_key.values() if len({x % XCDS for x in v}) == 1)
    assert aligned >= 0.9 * len(by_key)  # only the partial last chunk of each size class can break the stride
    for v in by_key.values():
        assert max(v) - min(v) <= XCDS * (len(v) - 1)  # replicas start within a few slots of each other
    # no replicas at all: identity
    assert replica_dispatch_order([(p, 0) for p in range(5)]) == list(range(5))


def test_sharing_aware_placement_keeps_replicas_together():
    """GPU placement: co-located replicas share HBM reads, so groups stay together when that lowers
    the slowest rank; with weight 1 (nothing shared) it balances message rows like LPT."""
    from erasurehead_amd.parallel.placement import place_workers, place_workers_shared, rank_cost, workers_by_rank

    parts = [[(p, 1) for p in ([0, 1, 2] if w < 3 else [3, 4, 5] if w < 6 else [6, 7])] for w in range(8)]

    def slowest(owner, N, wt):
        by = workers_by_rank(owner, N)
        return max(rank_cost(by[r], parts, wt) for r in range(N))

    for N in (2, 4, 8):
        lpt = place_workers([float(len(p)) for p in parts], N)
        shared = place_workers_shared(parts, N, 0.25)
        assert slowest(shared, N, 0.25) <= slowest(lpt, N, 0.25)
        assert all(workers_by_rank(shared, N)[r] for r in range(N))  # no idle GPU
        assert place_workers_shared(parts, N, 0.25) == shared  # deterministic
    assert slowest(place_workers_shared(parts, 4, 0.25), 4, 0.25) == 4.5  # vs 6.0 for LPT pairs
    flat = place_workers_shared(parts, 2, 1.0)
    assert slowest(flat, 2, 1.0) == 11.0  # 22 message rows over 2 ranks
    assert place_workers_shared(parts, 1, 0.25) == [0] * 8


def test_partition_shards_keep_each_partitions_replicas_on_one_rank():
    """Partition shards (multi-rank default): the headline's 22 (worker, partition) shards over N
    ranks; every partition's replicas share a rank, the slowest rank streams ceil(8/N) partitions,
    and at N = 8 each GPU holds one partition (1 + 2 x 0.12 replica units)."""
    from erasurehead_amd.codes import make_scheme
    from erasurehead_amd.parallel.placement import make_shards, place_units, rank_cost, workers_by_rank

    sch = make_scheme("approx", 8, 2, 8000, 6, 0, allow_uneven=True)
    shards = make_shards(sch.messages, "partition")
    assert len(shards) == 22 and all(len(u.segments) == 1 for u in shards)
    assert {(u.worker, u.part): u.n_shards for u in shards}[(6, 0)] == 2
    parts = [[(u.segments[0][0], 1)] for u in shards]
    for N in (1, 2, 4, 8):
        own = place_units(parts, N, 0.12)
        home = {}
        for u, o in zip(shards, own):
            assert home.setdefault(u.segments[0][0], o) == o  # one rank per partition
        by = workers_by_rank(own, N)
        cost = [rank_cost(by[r], parts, 0.12) for r in range(N)]
        assert max(len({parts[i][0][0] for i in by[r]}) for r in range(N)) == -(-8 // N)
        assert place_units(parts, N, 0.12) == own  # deterministic on every rank
    assert abs(max(cost) - 1.24) < 1e-9
    assert make_shards(sch.messages, "message")[0].segments == tuple(sch.messages[0].segments)
