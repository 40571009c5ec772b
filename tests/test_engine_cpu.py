"""Engine on CPU (torch fp64): every scheme vs the NumPy replay of the reference math."""
import os

import numpy as np
import pytest
import torch

from erasurehead_amd.codes import make_scheme, scheme_key
from erasurehead_amd.config import RunConfig
from erasurehead_amd.data.source import ArraySource
from erasurehead_amd.engine import Trainer, evaluate
from erasurehead_amd.models.losses import LEAST_SQUARES, LOGISTIC, logistic_loss, roc_auc
from erasurehead_amd.parallel.dist import DistEnv
from oracle import replay, stops_exactly_at_last

CASES = [  # key args: (is_coded, partitions, coded_ver, n_procs, s, num_collect)
    (0, 0, 0, 5, 0, 0),
    (1, 0, 0, 7, 2, 0),
    (1, 0, 1, 7, 2, 0),
    (1, 0, 2, 7, 2, 0),
    (1, 0, 3, 7, 2, 4),
    (1, 0, 3, 9, 2, 6),  # W=8, s=2: uneven FRC groups (extension)
    (1, 4, 1, 7, 1, 0),
    (1, 4, 0, 7, 1, 0),
]


def make(case, rule="AGD", rows=30, d=17, loss="auto", seed=0, precision="fp64", **kw):
    is_coded, P, ver, n_procs, s, k = case
    W = n_procs - 1
    key = scheme_key(is_coded, P, ver)
    uneven = key in ("approx", "replication") and W % (s + 1) != 0
    probe = make_scheme(key, W, s, rows * W, k, P, allow_uneven=uneven)
    n_parts = probe.n_partition_files
    n = rows * n_parts
    rng = np.random.RandomState(seed)
    parts = [(rng.randn(rows, d) * 0.3, rng.choice([-1.0, 1.0], rows)) for _ in range(n_parts)]
    test = (rng.randn(rows * 2, d) * 0.3, rng.choice([-1.0, 1.0], rows * 2))
    src = ArraySource(parts, test)
    cfg = RunConfig(n_procs, n, d, "/tmp/eh_cpu_eng/", 0, "x", is_coded, s, P, ver, k, 0, rule, num_itrs=6, seed=0,
                    verbose=False, allow_uneven_groups=uneven, loss=loss, precision=precision, **kw)
    sch = make_scheme(key, W, s, n, k, P, allow_uneven=uneven, rng=np.random.RandomState(7))
    return cfg, src, sch, parts


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("rule", ["GD", "AGD"])
def test_engine_matches_numpy_replay(case, rule):
    cfg, src, sch, parts = make(case, rule)
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    ref = replay(sch, parts, tr.beta0, res.arrivals, rule, cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(res.betaset, ref, rtol=1e-10, atol=1e-12)
    assert stops_exactly_at_last(sch, res.arrivals)  # the collector's stop rule, independently re-derived
    assert res.timeset.shape == (6,) and np.all(res.timeset > 0)
    assert res.worker_timeset.shape == (6, cfg.n_workers)


def test_least_squares_engine():
    cfg, src, sch, parts = make((1, 0, 3, 7, 2, 4), "GD", loss="least_squares")
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    ref = replay(sch, parts, tr.beta0, res.arrivals, "GD", cfg.alpha_value, cfg.n_rows, cfg.eta(), LEAST_SQUARES)
    np.testing.assert_allclose(res.betaset, ref, rtol=1e-10, atol=1e-12)


def test_fp32_close_to_fp64():
    a = make((1, 0, 3, 7, 2, 4), "GD")
    b = make((1, 0, 3, 7, 2, 4), "GD", precision="fp32")
    ra = Trainer(a[0], DistEnv(), a[1], scheme=a[2]).run()
    rb = Trainer(b[0], DistEnv(), b[1], scheme=b[2]).run()
    np.testing.assert_allclose(rb.betaset, ra.betaset, rtol=1e-4, atol=1e-5)


def test_evaluate_matches_reference_epilogue(tmp_path):
    cfg, src, sch, parts = make((0, 0, 0, 5, 0, 0), "GD")
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    lines = []
    cfg.input_dir = str(tmp_path) + "/"
    ev = evaluate(tr, res, log=lines.append, write=False)
    # training set = partitions 1..W-1 (skips partition W, ref src/naive.py:161)
    Xtr = np.vstack([parts[p][0] for p in range(cfg.n_workers - 1)])
    ytr = np.concatenate([parts[p][1] for p in range(cfg.n_workers)])[: Xtr.shape[0]]
    Xte, yte = src._test
    for i in range(len(res.betaset)):
        b = res.betaset[i]
        assert ev.training_loss[i] == pytest.approx(logistic_loss(ytr, Xtr @ b), rel=1e-10)
        assert ev.testing_loss[i] == pytest.approx(logistic_loss(yte, Xte @ b), rel=1e-10)
        assert ev.auc[i] == pytest.approx(roc_auc(yte, Xte @ b), rel=1e-12)


def test_delay_virtual_floor():
    """add_delay=1 (scaled mean): AGC time-to-decode sums to the deterministic floor + overhead."""
    from erasurehead_amd.utils.delay import delay_floor

    cfg, src, sch, parts = make((1, 0, 3, 7, 2, 4), "GD", delay_mean=0.01)
    cfg.add_delay = 1
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    floor = delay_floor(6, 6, groups=sch.group_of, k=4, mean=0.01)
    assert floor <= res.timeset.sum() < floor + 6 * 0.02
    # the wall-clock per round includes the drained straggler tail (replication/AGC Waitall)
    assert np.all(res.loop_time >= res.timeset)


def test_killed_worker_becomes_erasure():
    cfg, src, sch, parts = make((1, 0, 0, 7, 2, 0), "GD", kill_workers=[2], round_timeout=5.0)
    cfg.add_delay = 1
    cfg.delay_mode = "none"
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    assert res.timeouts == 0  # cyclic tolerates s=2 dead/slow workers
    assert np.all(res.worker_timeset[:, 1] == -1)
    ref = replay(sch, parts, tr.beta0, res.arrivals, "GD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(res.betaset, ref, rtol=1e-10, atol=1e-12)


def test_checkpoint_written(tmp_path):
    cfg, src, sch, parts = make((1, 0, 3, 7, 2, 4), "GD", checkpoint_every=2,
                                checkpoint_path=str(tmp_path / "ck.pt"))
    res = Trainer(cfg, DistEnv(), src, scheme=sch).run()
    st = torch.load(str(tmp_path / "ck.pt"), weights_only=True)
    assert st["next_round"] == 6
    np.testing.assert_allclose(st["hist"].numpy()[:, :17], res.betaset)


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[4]])
def test_resume_continues_trajectory(case, tmp_path):
    """Checkpoint at round 3, resume in a fresh trainer: the trajectory equals the replay."""
    ck = str(tmp_path / "ck.pt")
    cfg, src, sch, parts = make(case, "AGD", checkpoint_every=3, checkpoint_path=ck)
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    full = tr.run()
    st = torch.load(ck, weights_only=True)
    assert st["next_round"] == 6
    # rewrite a round-3 checkpoint from the full run and resume from it
    torch.save({**st, "next_round": 3, "hist": st["hist"][:3],
                "beta": torch.from_numpy(np.pad(full.betaset[2], (0, tr.ld - tr.d))),
                "timeset": st["timeset"][:3], "worker_timeset": st["worker_timeset"][:3],
                "u": _u_after(sch, parts, tr.beta0, full.arrivals[:3], cfg, tr.ld)}, ck)
    cfg2, src2, sch2, _ = make(case, "AGD", resume=ck)
    tr2 = Trainer(cfg2, DistEnv(), src2, scheme=sch2)
    res2 = tr2.run()
    np.testing.assert_allclose(res2.betaset[:3], full.betaset[:3])
    arr = full.arrivals[:3] + res2.arrivals[3:]
    ref = replay(sch, parts, tr.beta0, arr, "AGD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(res2.betaset, ref, rtol=1e-10, atol=1e-12)


def _u_after(sch, parts, beta0, arrivals, cfg, ld):
    """AGD auxiliary vector u after len(arrivals) rounds (NumPy oracle)."""
    from erasurehead_amd.codes.schemes import Arrival
    from erasurehead_amd.models.losses import UpdateRule, worker_grad

    up = UpdateRule("AGD", cfg.alpha_value, cfg.n_rows, sch.grad_scale())
    beta = np.array(beta0, dtype=np.float64)
    u = np.zeros_like(beta)
    for i, arr in enumerate(arrivals):
        used = sch.decode([Arrival(w, p, t) for (w, p, t) in arr])
        g = np.zeros_like(beta)
        for (w, part), c in used.items():
            m = [x for x in sch.messages if x.worker == w and x.part == part][0]
            g += c * sum(worker_grad(LOGISTIC, parts[p][0], parts[p][1], beta, coef) for p, coef in m.segments)
        up.apply(i, 10.0, beta, u, g)
    return torch.from_numpy(np.pad(u, (0, ld - len(u))))


@pytest.mark.parametrize("case,k", [((1, 0, 3, 7, 1, 2), 2), ((1, 0, 0, 7, 2, 0), 4), ((0, 0, 0, 5, 0, 0), 4)])
def test_arrival_sets_replay_reference_delays(case, k):
    """Scheduler replay (SURVEY §4 layer 3): with the reference's seeded Exp delays, the workers
    used each round and the -1 marks of worker_timeset follow the stop rule applied to
    RandomState(i).exponential(mean, W) (rounds whose delays are too close to call are skipped)."""
    mean = 0.02
    cfg, src, sch, parts = make(case, "GD", delay_mean=mean)
    cfg.add_delay = 1
    cfg.num_itrs = 8
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    W = cfg.n_workers
    T, fin = 0.0, np.zeros(W)  # virtual round start and per-worker finish (non-draining schemes carry lag)
    for i in range(cfg.num_itrs):
        d = np.random.RandomState(i).exponential(mean, W)
        ready = np.maximum(T, fin) + d
        order = list(np.argsort(ready, kind="stable"))
        # the oracle stop rule on the arrival order
        got_groups, used = set(), []
        for w in order:
            used.append(w)
            got_groups.add(sch.group_of[w])
            if sch.key == "naive" and len(used) == W:
                break
            if sch.key == "coded" and len(used) == W - cfg.n_stragglers:
                break
            if sch.key == "approx" and (len(used) >= k or len(got_groups) == sch.n_groups):
                break
        fin = ready
        T = float(np.max(ready)) if tr.drain else float(ready[used[-1]])
        # the used SET is decided at the stop boundary: skip rounds where the last used and the
        # first unused worker are too close for wall-clock scheduling noise (a loaded CPU)
        noise = 10e-3  # host wake-up jitter of a loaded CPU (pytest -n, a build running alongside)
        nxt = ready[order[len(used)]] if len(used) < W else np.inf
        if nxt - ready[used[-1]] < noise:
            continue
        arrived = [w for (w, p, _) in res.arrivals[i]]
        assert sorted(arrived) == sorted(used), (i, arrived, used)
        assert arrived[-1] in {w for w in used if ready[used[-1]] - ready[w] < noise}, (i, arrived, used)
        if sch.marks_unused:
            assert set(np.where(res.worker_timeset[i] == -1)[0]) == set(range(W)) - set(used)


@pytest.mark.parametrize("case", CASES)
def test_share_partitions_matches_numpy_replay(case):
    """--share-partitions: distinct partitions once + encode, same trajectory as the reference math."""
    cfg, src, sch, parts = make(case, "AGD", share_partitions=True)
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    from erasurehead_amd.ops.grad import SharedGradPlan

    shared = SharedGradPlan.worthwhile([m.segments for m in sch.messages], lambda p: 1)
    assert isinstance(tr.plan, SharedGradPlan) == shared
    assert shared == (case[4] > 0 and case[2] != 2)  # every scheme but naive / avoidstragg replicates
    res = tr.run()
    ref = replay(sch, parts, tr.beta0, res.arrivals, "AGD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(res.betaset, ref, rtol=1e-10, atol=1e-12)


def test_shared_plan_encoding_matrix():
    from erasurehead_amd.ops.grad import SharedGradPlan

    msgs = [[(0, 1.0), (1, -2.0)], [(1, 0.5), (2, 1.0)], [(2, 3.0)]]
    seen = []

    class Inner:
        prec, loss, d, ld, device = None, 0, 4, 4, torch.device("cpu")

        def __init__(self, ms):
            seen.append(ms)

        def out_buffer(self, n=1):
            return torch.zeros((n, 3, 4), dtype=torch.float64)

    class P:
        acc = torch.float64

    Inner.prec = P
    sp = SharedGradPlan(msgs, Inner)
    assert seen == [[[(0, 1.0)], [(1, 1.0)], [(2, 1.0)]]]
    np.testing.assert_array_equal(sp.E.numpy(), [[1, -2, 0], [0, 0.5, 1], [0, 0, 3]])
    assert SharedGradPlan.worthwhile(msgs, lambda p: 10)
    assert not SharedGradPlan.worthwhile([[(0, 1.0)], [(1, 1.0)]], lambda p: 10)


def test_delay_floor_with_carried_lag():
    """avoidstragg does not drain: Σtimeset follows the carried-lag replay, which exceeds the
    independent per-round order statistic."""
    from erasurehead_amd.utils.delay import delay_floor

    cfg, src, sch, parts = make((1, 0, 2, 7, 2, 0), "AGD", delay_mean=0.01)
    cfg.add_delay = 1
    cfg.force_delay = True
    tr = Trainer(cfg, DistEnv(), src, scheme=sch)
    res = tr.run()
    plain = delay_floor(6, 6, stop_count=4, mean=0.01)
    carried = delay_floor(6, 6, stop_count=4, mean=0.01, carry=True)
    assert carried >= plain
    assert carried <= res.timeset.sum() < carried + 6 * 0.02


def test_checkpoint_restores_cyclic_code(tmp_path):
    """A resumed cyclic-MDS run decodes with the checkpoint's B, not a freshly drawn one."""
    ck = str(tmp_path / "ck.pt")
    cfg, src, sch, parts = make(CASES[1], "AGD", checkpoint_every=3, checkpoint_path=ck)
    tr = Trainer(cfg, DistEnv(), src)  # B drawn from cfg.seed
    tr.run()
    st = torch.load(ck, weights_only=True)
    np.testing.assert_array_equal(st["B"].numpy(), tr.scheme.B)
    cfg2, src2, _, _ = make(CASES[1], "AGD", resume=ck)
    cfg2.seed = None  # unseeded: without the checkpoint's B a new random code would be drawn
    tr2 = Trainer(cfg2, DistEnv(), src2)
    np.testing.assert_array_equal(tr2.scheme.B, tr.scheme.B)
