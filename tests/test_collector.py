"""Native arrival collector: stop rules, virtual straggler delays, lag carry-over, drain."""
import math
import os
import time

import pytest

from erasurehead_amd.codes.schemes import RULE_ALL, RULE_COUNT, RULE_FRC, RULE_PARTIAL_COUNT, RULE_PARTIAL_FRC


@pytest.fixture
def C(native):
    return native


def test_frc_stop_on_groups(C):
    c = C.Collector(6, [0, 0, 0, 1, 1, 1], 2)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_FRC, 5)
    ids = [c.add_host_probe(w, 0, 0, 0.0) for w in range(6)]
    for w in (1, 2):
        c.mark_seen(ids[w], t0)
    assert not c.step()
    c.mark_seen(ids[4], t0)
    assert c.step()  # both groups covered after 3 arrivals (k=5 not needed)
    assert [a.worker for a in c.arrivals()] == [1, 2, 4]


def test_count_rule_and_virtual_delay_order(C):
    c = C.Collector(4, [0, 1, 2, 3], 4)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_COUNT, 2)
    delays = [0.03, 0.0, 0.01, 1.0]
    ids = [c.add_host_probe(w, 0, 0, delays[w]) for w in range(4)]
    for i in ids:
        c.mark_seen(i, t0)
    assert c.wait(5.0)
    arr = c.arrivals()
    assert [a.worker for a in arr] == [1, 2]
    assert arr[1].t_rel == pytest.approx(0.01, abs=1e-6)
    assert C.Collector.now() - t0 >= 0.0099


def test_all_rule_timeout_dead_worker(C):
    c = C.Collector(3, [0, 1, 2], 3)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_ALL, 3)
    ids = [c.add_host_probe(w, 0, 0, math.inf if w == 2 else 0.0) for w in range(3)]
    for i in ids:
        c.mark_seen(i, t0)
    assert not c.wait(0.05)  # worker 2 never arrives -> timeout, erasure
    assert sorted(a.worker for a in c.arrivals()) == [0, 1]
    assert c.drain(0, 1.0)  # dead worker was seen: drain does not hang


def test_partial_rules(C):
    c = C.Collector(3, [0, 1, 2], 3)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_PARTIAL_COUNT, 2)
    p1 = [c.add_host_probe(w, 1, 0, 0.0) for w in range(3)]
    p0 = [c.add_host_probe(w, 0, 0, 0.0) for w in range(3)]
    for w in range(3):
        c.mark_seen(p0[w], t0)
    assert not c.step()  # coded parts done but first parts missing
    for w in range(3):
        c.mark_seen(p1[w], t0)
    assert c.step()
    c2 = C.Collector(4, [0, 0, 1, 1], 2)
    c2.begin_round(0, t0, RULE_PARTIAL_FRC, 4)
    q1 = [c2.add_host_probe(w, 1, 0, 0.0) for w in range(4)]
    q0 = [c2.add_host_probe(w, 0, 0, 0.0) for w in range(4)]
    for w in range(4):
        c2.mark_seen(q1[w], t0)
    c2.mark_seen(q0[1], t0)
    assert not c2.step()
    c2.mark_seen(q0[3], t0)
    assert c2.step()


def test_lag_carries_into_next_round(C):
    """Without a drain, a straggler's virtual finish delays its next-round arrival (reference lag)."""
    c = C.Collector(2, [0, 1], 2)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_COUNT, 1)
    a = c.add_host_probe(0, 0, 0, 0.0)
    b = c.add_host_probe(1, 0, 0, 0.2)
    c.mark_seen(a, t0)
    c.mark_seen(b, t0)
    assert c.wait(1.0)
    assert [x.worker for x in c.arrivals()] == [0]
    t1 = C.Collector.now()
    c.begin_round(1, t1, RULE_COUNT, 1)
    a1 = c.add_host_probe(0, 0, 1, 0.3)
    b1 = c.add_host_probe(1, 0, 1, 0.0)
    c.mark_seen(a1, t1)
    c.mark_seen(b1, t1)
    assert c.wait(2.0)
    arr = c.arrivals()
    # worker 1 finished round 0 at t0+0.2 (virtual), so it arrives ~0.2 - (t1-t0) after round 1 starts
    assert arr[0].worker == 1
    assert arr[0].t_rel == pytest.approx(0.2 - (t1 - t0), abs=2e-3)
    assert c.drain(1, 2.0)
    assert c.pending() == 0


def test_rounds_must_increase(C):
    c = C.Collector(1, [0], 1)
    c.begin_round(3, C.Collector.now(), RULE_ALL, 1)
    with pytest.raises(ValueError):
        c.begin_round(2, C.Collector.now(), RULE_ALL, 1)


def test_collector_host_asan_ubsan():
    """The collector state machine under AddressSanitizer + UBSan (host build, tools/sanitize_host.sh)."""
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["bash", os.path.join(root, "tools", "sanitize_host.sh")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "collector selftest ok" in r.stdout


def test_wait_seen_ignores_virtual_delay(C):
    """Slot reuse needs the data, not the virtual arrival: a straggler seen long before its
    virtual arrival does not block wait_seen."""
    col = C.Collector(2, [0, 1], 2)
    t0 = C.Collector.now()
    col.begin_round(0, t0, RULE_COUNT, 1)
    a = col.add_host_probe(0, 0, 0, 0.0)
    b = col.add_host_probe(1, 0, 0, 30.0)  # arrives (virtually) 30 s later
    col.mark_seen(a, t0)
    assert not col.wait_seen(0, 0.0)
    col.mark_seen(b, t0)
    t = time.perf_counter()
    assert col.wait_seen(0, 5.0)
    assert time.perf_counter() - t < 1.0
    assert not col.drain(0, 0.01)  # the reference Waitall still waits for the virtual arrival


def _tied_round_order(C, seed, rnd, W=8):
    c = C.Collector(W, list(range(W)), W)
    c.set_tie_seed(seed)
    t0 = C.Collector.now()
    c.begin_round(rnd, t0, RULE_ALL, 0)
    for w in range(W):
        c.mark_seen(c.add_host_probe(w, 0, rnd, 0.0), t0)  # all at the same instant
    assert c.step()
    return [a.worker for a in c.arrivals()]


def test_simultaneous_arrivals_use_seeded_round_permutation(C):
    orders = [_tied_round_order(C, 0, r) for r in range(12)]
    for r, o in enumerate(orders):
        assert sorted(o) == list(range(8))
        keys = [C.Collector.tie_key(0, r, w) for w in o]
        assert keys == sorted(keys)  # the documented, replayable permutation
    assert len({tuple(o) for o in orders}) > 6  # changes from round to round
    assert _tied_round_order(C, 0, 3) == orders[3]  # deterministic
    assert _tied_round_order(C, -1, 3) == list(range(8))  # tie_seed < 0: worker order


def test_agc_zero_delay_covers_every_group_across_rounds():
    """W=8, s=2, k=6 (uneven groups {0,1,2},{3,4,5},{6,7}) with add_delay=0: the stop rule fires
    after 6 simultaneous arrivals; with the seeded tie permutation every group, and so every
    partition, reaches the decoded gradient in some round (worker order would drop {6,7} forever)."""
    import numpy as np
    import torch

    from erasurehead_amd.codes import make_scheme
    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.data.source import ArraySource
    from erasurehead_amd.engine import Trainer
    from erasurehead_amd.parallel.dist import DistEnv

    rows, d, W = 12, 5, 8
    rng = np.random.RandomState(0)
    parts = [(rng.randn(rows, d), rng.choice([-1.0, 1.0], rows)) for _ in range(W)]
    src = ArraySource(parts, (rng.randn(4, d), np.ones(4)))
    covered = {}
    for tie in ("permute", "worker"):
        cfg = RunConfig(9, rows * W, d, "/tmp/eh_tie/", 0, "x", 1, 2, 0, 3, 6, 0, "AGD", num_itrs=16, seed=0,
                        verbose=False, allow_uneven_groups=True, tie_break=tie)
        sch = make_scheme("approx", W, 2, rows * W, 6, 0, allow_uneven=True)
        res = Trainer(cfg, DistEnv(), src, scheme=sch).run()
        used = set()
        for arr in res.arrivals:
            from erasurehead_amd.codes.schemes import Arrival
            for (w, p) in sch.decode([Arrival(*a) for a in arr]):
                used.add(sch.group_of[w])
        covered[tie] = used
    assert covered["permute"] == {0, 1, 2}
    assert covered["worker"] == {0, 1}  # the degenerate order the default avoids


def test_sharded_message_arrives_with_its_last_shard(C):
    c = C.Collector(3, [0, 1, 2], 3)
    c.set_shards(0, 0, 3)  # worker 0's message is computed as 3 partition shards
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_COUNT, 2)
    sh = [c.add_host_probe(0, 0, 0, d) for d in (0.0, 0.02, 0.0)]
    w1 = c.add_host_probe(1, 0, 0, 0.01)
    for i in sh + [w1]:
        c.mark_seen(i, t0)
    assert c.wait(5.0)
    arr = c.arrivals()
    assert [a.worker for a in arr] == [1, 0]  # worker 0 counts once, at its slowest shard
    assert arr[1].t_rel == pytest.approx(0.02, abs=1e-6)


def _lazy_two_rounds(C, skip):
    """Worker 1 is still busy with round 0 (virtual delay 0.2 s) when rounds 1 and 2 begin."""
    c = C.Collector(2, [0, 1], 2)
    c.set_skip_stale(skip)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_COUNT, 1)
    c.mark_seen(c.add_host_probe(0, 0, 0, 0.0), t0)
    c.mark_seen(c.add_host_probe(1, 0, 0, 0.2), t0)
    assert c.wait(1.0) and [x.worker for x in c.arrivals()] == [0]
    t1 = C.Collector.now()
    c.begin_round(1, t1, RULE_COUNT, 1)
    c.mark_seen(c.add_host_probe(0, 0, 1, 0.0), t1)
    c.mark_seen(c.add_host_probe(1, 0, 1, 0.1), t1)  # would finish at t0 + 0.3 if it ran
    assert c.wait(1.0) and [x.worker for x in c.arrivals()] == [0]
    t2 = C.Collector.now()
    c.begin_round(2, t2, RULE_COUNT, 1)
    c.mark_seen(c.add_host_probe(0, 0, 2, 0.5), t2)
    c.mark_seen(c.add_host_probe(1, 0, 2, 0.0), t2)
    assert c.wait(2.0)
    arr = c.arrivals()
    assert arr[0].worker == 1
    return c, arr[0].t_rel + (t2 - t0)  # worker 1's round-2 arrival, from t0


def test_lazy_drain_skips_the_stale_round(C):
    """Drain "lazy": worker 1, busy until t0 + 0.2 when round 2 began, skips round 1 (beta(2) was
    out before it could start it) and delivers round 2 at t0 + 0.2; with the lag carried (the
    reference's no-Waitall schemes) it runs round 1 first and round 2 lands at t0 + 0.3."""
    c, t_lazy = _lazy_two_rounds(C, True)
    assert t_lazy == pytest.approx(0.2, abs=3e-3)
    assert c.skipped == 1
    assert c.drain(2, 2.0)
    assert c.stale_arrivals >= 1  # its round-0 message landed during round 2: drained, never decoded
    c2, t_carry = _lazy_two_rounds(C, False)
    assert t_carry == pytest.approx(0.3, abs=3e-3)
    assert c2.skipped == 0


def test_end_run_skips_what_a_late_worker_has_not_started(C):
    c = C.Collector(2, [0, 1], 2)
    c.set_skip_stale(True)
    t0 = C.Collector.now()
    for r in range(3):
        t = C.Collector.now()
        c.begin_round(r, t, RULE_COUNT, 1)
        c.mark_seen(c.add_host_probe(0, 0, r, 0.0), t)
        c.mark_seen(c.add_host_probe(1, 0, r, 5.0), t)  # worker 1: 5 s late every round
        assert c.wait(1.0)
    c.end_run(C.Collector.now())
    # rounds 1 and 2 of worker 1 never start (it is busy with round 0 until t0 + 5 s): skipped, so the
    # final drain only waits for its round-0 message
    assert c.skipped == 2
    assert c.pending_upto(2) == 1
    assert C.Collector.now() - t0 < 1.0


def test_physical_probes_arrive_when_seen(C):
    """--delay-on worker: a remote message's completion time is its arrival; a rank that was late in
    round 0 carries no virtual lag into round 1 (it really was late, and really is on time now)."""
    c = C.Collector(2, [0, 1], 2)
    t0 = C.Collector.now()
    c.begin_round(0, t0, RULE_ALL, 2)
    a = c.add_host_probe(0, 0, 0, 0.0, True)
    b = c.add_host_probe(1, 0, 0, 0.0, True)
    c.mark_seen(a, t0)
    c.mark_seen(b, t0 + 0.05)  # really late by 50 ms
    assert c.wait(1.0)
    assert [round(x.t_rel, 3) for x in c.arrivals()] == [0.0, 0.05]
    t1 = t0 + 0.06
    c.begin_round(1, t1, RULE_ALL, 2)
    p = [c.add_host_probe(w, 0, 1, 0.0, True) for w in range(2)]
    for q in p:
        c.mark_seen(q, t1 + 0.001)
    assert c.wait(1.0)
    assert max(x.t_rel for x in c.arrivals()) == pytest.approx(0.001, abs=1e-9)


def test_schedule_model_matches_the_collector_rules():
    """utils/delay.schedule: drain all / carry / lazy on a hand-checked 3-round, 2-worker case."""
    import numpy as np

    from erasurehead_amd.utils.delay import schedule

    d = np.array([[0.0, 0.2], [0.0, 0.1], [0.5, 0.0]])
    lazy, _ = schedule(d, "count", 1, [0, 1], "lazy")
    carry, _ = schedule(d, "count", 1, [0, 1], "carry")
    drained, _ = schedule(d, "count", 1, [0, 1], "all")
    assert lazy == [[0], [0], [1]]  # round 2: worker 1 (free at 0.2, skipped round 1) beats 0.5
    assert carry == [[0], [0], [1]]  # worker 1 at 0.3 still beats worker 0 at 0.5
    assert drained == [[0], [0], [1]]
    d2 = d.copy()
    d2[2, 0] = 0.25  # worker 0 lands at 0.25: before carry's 0.3, after lazy's 0.2
    assert schedule(d2, "count", 1, [0, 1], "lazy")[0][2] == [1]
    assert schedule(d2, "count", 1, [0, 1], "carry")[0][2] == [0]


def test_shards_seen_at_different_times_count_from_the_round_start(C):
    """A message computed as two partition shards on different ranks, seen at t1 < t2 in the same round:
    each shard's compute counts from the round start (t2 - ts for the second, not t2 - t1), so the
    message's virtual arrival is at its slowest shard, t2."""
    c = C.Collector(2, [0, 1], 2)
    c.set_shards(0, 0, 2)
    t0 = C.Collector.now() - 1.0  # the round began a second ago: every time below is in the past
    c.begin_round(0, t0, RULE_ALL, 2)
    a = c.add_host_probe(0, 0, 0, 0.0)
    b = c.add_host_probe(0, 0, 0, 0.0)
    w1 = c.add_host_probe(1, 0, 0, 0.0)
    c.mark_seen(a, t0 + 0.01)
    c.mark_seen(b, t0 + 0.03)
    c.mark_seen(w1, t0 + 0.02)
    assert c.wait(1.0)
    got = {x.worker: x.t_rel for x in c.arrivals()}
    assert got[0] == pytest.approx(0.03, abs=1e-9)
    assert got[1] == pytest.approx(0.02, abs=1e-9)
    # round 1: each shard's busy time starts at the round start or at round 0's last shard (t0 + 0.03)
    t1 = t0 + 0.025
    c.begin_round(1, t1, RULE_ALL, 2)
    a = c.add_host_probe(0, 0, 1, 0.0)
    b = c.add_host_probe(0, 0, 1, 0.0)
    w1 = c.add_host_probe(1, 0, 1, 0.0)
    c.mark_seen(a, t1 + 0.015)
    c.mark_seen(b, t1 + 0.02)
    c.mark_seen(w1, t1 + 0.001)
    assert c.wait(1.0)
    got = {x.worker: x.t_rel for x in c.arrivals()}
    # worker 0 starts round 1 at its round-0 finish t0 + 0.03 and is busy t1 + 0.02 - (t0 + 0.03) = 0.015
    assert got[0] == pytest.approx(0.03 + 0.015 - 0.025, abs=1e-9)


def test_schedule_floors_sum_the_event_model():
    import numpy as np

    from erasurehead_amd.utils.delay import schedule_floors

    d = np.array([[0.0, 0.2], [0.0, 0.1], [0.5, 0.0]])
    assert schedule_floors(d, "count", 1, [0, 1], "lazy") == pytest.approx((0.2, 0.2))
    # drain all: every round lasts until its last arrival (0.2, 0.1, 0.5); decodes at the first one
    assert schedule_floors(d, "count", 1, [0, 1], "all") == pytest.approx((0.0, 0.8))


def test_lazy_flag_probe_past_its_round_leaves_as_skipped(C):
    """Drain lazy over the IPC mailbox: a worker rank whose device gate skipped round 0 never signals it;
    its counter goes straight to round 1's value.  The round-0 probe, first seen with the counter already
    past it, leaves as skipped (no compute time charged to a round that never ran) instead of arriving."""
    import numpy as np

    flag = np.zeros(1, dtype=np.uint64)
    addr = flag.ctypes.data
    c = C.Collector(2, [0, 1], 2)
    c.set_skip_stale(True)
    t0 = C.Collector.now() - 1.0
    c.begin_round(0, t0, RULE_COUNT, 1)
    c.mark_seen(c.add_host_probe(0, 0, 0, 0.0), t0)
    c.add_flag_probe(1, 0, 0, addr, 1, 0.0)
    assert c.step() and [a.worker for a in c.arrivals()] == [0]
    c.begin_round(1, t0 + 0.5, RULE_COUNT, 2)
    c.add_flag_probe(1, 0, 1, addr, 2, 0.0)
    c.mark_seen(c.add_host_probe(0, 0, 1, 0.0), t0 + 0.5)
    flag[0] = 2  # round 1's put landed; round 0 was skipped on the device
    assert c.wait(1.0)
    assert sorted(a.worker for a in c.arrivals()) == [0, 1]
    assert c.skipped == 1 and c.stale_arrivals == 0
    assert c.drain(1, 1.0)
