"""Physically late worker ranks (--delay-on worker) and slow GPUs (--slow-ranks) on gloo.

The reference sleeps Exp(0.5) seconds on every worker after its gradient and before its Isend
(ref src/naive.py:141-148, src/approximate_coding.py:198-205), so the master really sees late
messages.  With ``delay_on="worker"`` a worker rank sleeps (host) / spins (device) at that point
and the master's collector applies no virtual delay to remote messages; its own co-located
worker keeps the virtual delay.  With one logical worker per rank (``shard="message"``, the
reference topology) the physical arrival sets must match the virtual model's stop rule on every
round whose delays are well separated, and the trajectory must replay exactly through the fp64
oracle from the arrivals it logged.
"""
import numpy as np
import pytest

from test_distributed_cpu import _run
from test_engine_cpu import make

pytestmark = pytest.mark.slow

MEAN, MARGIN = 0.08, 0.012


def _predict(d, rule, k, groups):
    """Arrival list (worker ids) of the virtual model: order by delay, stop by the scheme's rule."""
    order = list(np.argsort(d, kind="stable"))
    out, covered = [], set()
    for w in order:
        out.append(int(w))
        covered.add(groups[w])
        if rule == "count" and len(out) >= k:
            break
        if rule == "frc" and (len(out) >= k or len(covered) == len(set(groups))):
            break
    return out


def _separated(d):
    s = np.sort(d)
    return np.all(np.diff(s) > MARGIN)


@pytest.mark.parametrize("case,world,rule,k,groups", [
    ((1, 0, 0, 4, 1, 0), 3, "count", 2, [0, 1, 2]),           # cyclic W=3 s=1: the 2 fastest, drained
    ((1, 0, 3, 5, 1, 3), 4, "frc", 3, [0, 0, 1, 1]),          # AGC W=4 s=1 k=3: groups {0,1}, {2,3}
])
def test_physical_delays_match_virtual_model(case, world, rule, k, groups, tmp_path):
    from oracle import replay

    R = 12
    kw = dict(delay_mode="exp", delay_mean=MEAN, delay_on="worker", shard="message", drain="all", rounds=R)
    cfg, src, sch, parts = make(case, "GD", **{x: v for x, v in kw.items() if x != "rounds"})
    cfg.num_itrs = R
    r = _run(world, case, "GD", tmp_path, **kw)
    checked = 0
    for i, a in enumerate(r["arrivals"]):
        d = np.random.RandomState(i).exponential(MEAN, cfg.n_workers)
        if not _separated(d):
            continue
        assert [w for (w, p) in a] == _predict(d, rule, k, groups), (i, d, a)
        checked += 1
    assert checked >= 2
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "GD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-10, atol=1e-12)


def test_slow_rank_is_skipped_with_message_placement(tmp_path):
    """AGC W=4 s=1 k=3 on 4 ranks, rank 3 physically late by 80 ms every round (fixed straggler,
    slept on the worker): with whole messages per rank the decode never waits for it."""
    case = (1, 0, 3, 5, 1, 3)
    r = _run(4, case, "GD", tmp_path, delay_mode="fixed", fixed_stragglers=[4], fixed_sleep=0.08,
             delay_on="worker", shard="message", rounds=6)
    for a in r["arrivals"]:
        assert 3 not in {w for (w, p) in a}
        assert len(a) in (2, 3)  # k = 3 arrivals or both groups covered
