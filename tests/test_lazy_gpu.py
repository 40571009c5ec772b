"""Drain "lazy" on the GPU: stale-round gates in the kernels and physically late worker ranks.

Reference: cyclic / naive / avoidstragg never Waitall, and a worker cancels its previous send once
the next beta arrives (ref src/coded.py:137-196, :178-180); AGC's stop rule ends a round at k
arrivals (ref src/approximate_coding.py:144-158).  Here a worker rank still busy when beta(i+1)
is published skips round i on the device (csrc/kernels/common.h gate_closed, decided by its
previous round's put kernel from the beta counter), and the master never waits for the tail.
"""
import json
import os

import numpy as np
import pytest
import torch

from erasurehead_amd.models.losses import LOGISTIC
from erasurehead_amd.ops import DenseGradPlan, SparseGradPlan, get_precision
from erasurehead_amd.ops.grad import KernelChoice

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _dense_parts(rng, sizes, d, prec):
    parts = {}
    for p, n in enumerate(sizes):
        X = torch.zeros((n, prec.ld(d)), dtype=torch.float64)
        X[:, :d] = torch.from_numpy(rng.randn(n, d) * 0.3)
        y = torch.from_numpy(rng.choice([-1.0, 1.0], n))
        parts[p] = (X.to(prec.storage).to(DEV).contiguous(), y.to(prec.acc).to(DEV))
    return parts


@pytest.mark.parametrize("prec_name,d,msgs,choice", [
    ("fp64", 1000, [[(0, 1.0)], [(1, 1.0)]], None),                                   # one-wave bundles of one
    ("fp64", 1000, [[(0, 1.0), (1, 1.0)], [(0, 0.5), (1, 1.0)]], None),               # replica bundles
    ("fp32", 1000, [[(0, 1.0), (1, 1.0)], [(0, 0.5), (1, 1.0)], [(1, 2.0)]], None),   # staged / pair
    ("bf16", 1000, [[(0, 1.0), (1, 1.0)], [(0, 0.5), (1, 1.0)]], None),               # MFMA bundles
    ("fp64", 3000, [[(0, 1.0)], [(1, -1.0)]], None),                                  # wide rows
    ("fp64", 17000, [[(0, 1.0)]], None),                                              # two-pass
    ("fp64", 256, [[(0, 1.0)], [(1, 1.0)]], KernelChoice(kind="fused", rows=4)),       # fused, 4 rows in flight
])
def test_closed_gate_skips_every_gradient_kernel(prec_name, d, msgs, choice, native):
    """gate = 1: the whole launch chain (gradient, slab reduction, encode) returns at once and the
    message rows keep their previous contents; gate = 0: bitwise the ungated result."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(d)
    parts = _dense_parts(rng, [300, 257], d, prec)
    kw = {"choice": choice} if choice is not None else {}
    plan = DenseGradPlan(msgs, parts, prec, LOGISTIC, d, **kw)
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    beta[:d] = torch.from_numpy(rng.randn(d) * 0.2).to(prec.acc)
    launcher = plan.native_launcher()
    ref = plan.out_buffer()[0]
    launcher.launch(beta, ref)
    gate = torch.ones(1, dtype=torch.int32, device=DEV)
    G = torch.full_like(ref, 7.0)
    launcher.launch(beta, G, gate)
    torch.cuda.synchronize()
    assert torch.all(G == 7.0)
    gate.zero_()
    launcher.launch(beta, G, gate)
    torch.cuda.synchronize()
    assert torch.equal(G, ref)


def test_closed_gate_skips_the_sparse_ell_kernels(native):
    import scipy.sparse as sps

    prec = get_precision("fp64")
    rng = np.random.RandomState(1)
    d, parts = 500, {}
    for p in range(2):
        n = 300
        cols = np.stack([rng.choice(d, 4, replace=False) for _ in range(n)])
        parts[p] = (sps.csr_matrix((np.ones(cols.size), cols.ravel(), np.arange(0, cols.size + 1, 4)), shape=(n, d)),
                    rng.choice([-1.0, 1.0], n))
    plan = SparseGradPlan([[(0, 1.0), (1, 1.0)], [(1, 1.0)]], parts, prec, LOGISTIC, d, device=DEV, use_ell=True)
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    beta[:d] = torch.from_numpy(rng.randn(d) * 0.2)
    launcher = plan.native_launcher()
    ref = plan.out_buffer()[0]
    launcher.launch(beta, ref)
    G = torch.full_like(ref, 7.0)
    launcher.launch(beta, G, torch.ones(1, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    assert torch.all(G == 7.0)
    launcher.launch(beta, G, torch.zeros(1, dtype=torch.int32, device=DEV))
    torch.cuda.synchronize()
    assert torch.equal(G, ref)


def test_gated_put_and_next_gate(native):
    """The put kernel of round i: open gate -> payload + signal, then next gate = (beta counter >=
    stale_next); closed gate -> nothing put or signalled, next gate still decided."""
    import uuid

    C = native
    flags = C.ShmFlags("/eh_gate_" + uuid.uuid4().hex[:12], 4, True)
    try:
        src = torch.arange(64, dtype=torch.float64, device=DEV) + 1.0
        dst = torch.zeros_like(src)
        counters = torch.zeros(4, dtype=torch.int32, device=DEV)
        gate = torch.zeros(2, dtype=torch.int32, device=DEV)
        flags.store(0, 5)  # beta counter: beta(4) is out
        C.put_signal_gated(src, dst, flags.dev_addr(1), 5, counters, gate, flags.dev_addr(0), 6)
        torch.cuda.synchronize()
        assert torch.equal(dst, src) and flags.load(1) == 5 and gate.tolist() == [0, 0]
        flags.store(0, 6)  # beta(5) out: the next round (5) is stale before it starts
        C.put_signal_gated(src * 2, dst, flags.dev_addr(1), 6, counters, gate, flags.dev_addr(0), 6)
        torch.cuda.synchronize()
        assert torch.equal(dst, src * 2) and flags.load(1) == 6 and gate.tolist() == [0, 1]
        gate[0] = 1  # a closed gate: the round was skipped
        C.put_signal_gated(src * 3, dst, flags.dev_addr(1), 7, counters, gate, flags.dev_addr(0), 9)
        torch.cuda.synchronize()
        assert torch.equal(dst, src * 2) and flags.load(1) == 6 and gate.tolist() == [1, 0]
        assert counters.tolist() == [0, 0, 0, 0]  # the block counter protocol is untouched by a skip
    finally:
        flags.close()


# ---- multi-rank runs, ranks sharing the test box's GPU ---------------------------------------------
from test_multiproc_gpu import _launch  # noqa: E402


def _lazy_run(world, case, over, tmp_path, **env):
    r = _launch(world, 0, "GD", str(tmp_path / "z.npz"), EH_TEST_CASE=json.dumps(case), EH_TEST_CFG=json.dumps(over),
                EH_TEST_ROUND_TIMEOUT="30", **env)
    owner = {int(w): int(o) for w, o in json.loads(str(r["owner"])).items()}
    skipped = json.loads(str(r["skipped"]))
    return r, owner, skipped


@pytest.mark.parametrize("world,case,rule,k,groups,mean,R,transport", [
    (4, (1, 0, 0, 4, 1, 0), "count", 2, [0, 1, 2], 0.05, 16, "ipc"),                  # cyclic W=3 s=1
    (5, (1, 0, 3, 5, 1, 3), "frc", 3, [0, 0, 1, 1], 0.05, 16, "ipc"),                 # AGC W=4 s=1 k=3
    (9, (1, 0, 3, 9, 2, 6), "frc", 6, [0, 0, 0, 1, 1, 1, 2, 2], 0.05, 18, "ipc"),     # AGC W=8 s=2 k=6
    # the same over stream-ordered p2p (loopback: RCCL's code path).  9 processes parking device-side waits
    # on ONE GPU oversubscribe its hardware queues, whose rotation paces the rounds by tens of ms: longer
    # delays there, so ranks still fall behind (the checks themselves need no margin)
    (4, (1, 0, 0, 4, 1, 0), "count", 2, [0, 1, 2], 0.05, 16, "loopback"),
    (9, (1, 0, 3, 9, 2, 6), "frc", 6, [0, 0, 0, 1, 1, 1, 2, 2], 0.3, 14, "loopback"),
])
def test_lazy_drain_physically_late_ranks(world, case, rule, k, groups, mean, R, transport, tmp_path):
    """--delay-on worker --drain lazy, the reference topology (rank 0 the master only, one logical worker
    per worker rank): every worker rank spins Exp(mean) after its gradient; the master never waits for
    the tail and a rank still busy when the next beta is out skips that round on the device.  Checked
    against the ranks' own device records (tests/lazy_check.py), no model and no margin: the decoded set
    of every round is the stop rule over that round's messages in landing order, the collector's order
    is the workers' landing stamps, every skip / run decision is implied by the beta-put stamps, every
    run round spun its full delay.  Late rows never reach a decode (every decoded mailbox row's integrity
    tag names its round), and the trajectory replays exactly through the fp64 oracle."""
    from lazy_check import check_lazy_device
    from oracle import replay, stops_exactly_at_last
    from test_engine_cpu import make

    over = dict(add_delay=1, delay_mode="exp", delay_mean=mean, delay_on="worker", shard="message", drain="lazy",
                num_itrs=R, dedicated_master=True, device_records=True)
    env = {"ERASUREHEAD_TRANSPORT": transport} if transport != "ipc" else {}
    r, owner, skipped = _lazy_run(world, case, over, tmp_path, **env)
    assert str(r["transport"]) == transport
    cfg, src, sch, parts = make(case, "GD")
    W = cfg.n_workers
    assert sorted(owner.values()) == list(range(1, W + 1))  # rank 0 hosts nothing
    d = np.asarray(json.loads(str(r["delays"])))
    assert d.shape == (R, W)
    arrivals = [[int(w) for (w, p) in a] for a in r["arrivals"]]
    got = check_lazy_device(arrivals, json.loads(str(r["records"])), owner, skipped, d, rule, k, groups, transport)
    assert got["rounds"] == R and got["spins"] >= R and got["skips"] >= W
    assert got["inversions"] <= 1  # flag-visibility races: microseconds out of ~50 ms delays
    if transport == "ipc":
        assert got["order"] == R and got["tail_after_next_beta"] >= 1
    assert sum(len(v) for v in skipped) >= 1  # some rank fell behind and skipped a stale round
    full = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    assert stops_exactly_at_last(sch, full)
    ref = replay(sch, parts, r["beta0"], full, "GD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(R))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)
    rep = json.loads(str(r["rank_report"]))
    assert rep["drain"] == "lazy" and rep["round_loop"] == "native pump"
    assert rep["stale_arrivals"] >= 1  # late messages landed during later rounds and were not decoded
    reports = json.loads(str(r["reports"]))
    assert sum(x.get("stale_rounds_skipped", 0) for x in reports) == sum(len(v) for v in skipped)


@pytest.mark.parametrize("loop", ["pump", "arbiter", "loopback"])
def test_lazy_fixed_straggler_is_skipped_and_costs_nothing(loop, tmp_path):
    """AGC W=4 s=1 k=3 on 4 ranks, worker 3's rank 40 ms late every round (fixed straggler, physically
    spun): with drain lazy the master's rounds never wait for it, the rank computes one round, then
    finds every later round stale and skips it; on the host pump and on the device arbiter over the IPC
    mailbox, and on the host pump over stream-ordered p2p (loopback, RCCL's code path: the skipped
    rounds still send their stale rows, which land after their round and are never decoded)."""
    from oracle import replay
    from test_engine_cpu import make

    case, R = (1, 0, 3, 5, 1, 3), 16
    over = dict(add_delay=1, delay_mode="fixed", fixed_stragglers=[4], fixed_sleep=0.04, delay_on="worker",
                shard="message", drain="lazy", num_itrs=R)
    # loopback also runs its rounds in two segments with a fence between them (bench.py's timed_start): the
    # beta receives a p2p worker posts ahead must not cross the fence
    env = {"arbiter": {"ERASUREHEAD_DEVICE_MASTER": "on"},
           "loopback": {"ERASUREHEAD_TRANSPORT": "loopback", "EH_TEST_TIMED_START": "3"}}.get(loop, {})
    r, owner, skipped = _lazy_run(4, case, over, tmp_path, **env)
    assert json.loads(str(r["rank_report"]))["round_loop"] == ("arbiter" if loop == "arbiter" else "native pump")
    assert str(r["transport"]) == ("loopback" if loop == "loopback" else "ipc")
    for a in r["arrivals"]:
        assert 3 not in {int(w) for (w, p) in a}
    assert float(np.sum(r["loop_time"])) < 0.04 * R / 4  # the straggler's 40 ms never enter the rounds
    late_rank = owner[3]
    assert len(skipped[late_rank]) >= R - 4  # it ran a handful of rounds (one per 40 ms), skipped the rest
    cfg, src, sch, parts = make(case, "GD")
    full = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], full, "GD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(R))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("arbiter", [False, True])
def test_carry_keeps_every_round_of_a_late_rank(arbiter, tmp_path):
    """The reference's no-Waitall semantics (drain carry): the late rank computes and sends every
    round in order (no skipping), so it is still busy after the master's last round; its late messages
    of earlier rounds land during later ones and are never decoded.  On the host pump and on the device
    arbiter, the trajectory replays exactly through the fp64 oracle."""
    from oracle import replay
    from test_engine_cpu import make

    case, R = (1, 0, 3, 5, 1, 3), 8
    over = dict(add_delay=1, delay_mode="fixed", fixed_stragglers=[4], fixed_sleep=0.03, delay_on="worker",
                shard="message", drain="carry", num_itrs=R)
    env = {"ERASUREHEAD_DEVICE_MASTER": "on"} if arbiter else {}
    r, owner, skipped = _lazy_run(4, case, over, tmp_path, **env)
    assert json.loads(str(r["rank_report"]))["round_loop"] == ("arbiter" if arbiter else "native pump")
    assert all(len(v) == 0 for v in skipped)
    for a in r["arrivals"]:
        assert 3 not in {int(w) for (w, p) in a}
    cfg, src, sch, parts = make(case, "GD")
    full = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], full, "GD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(R))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)
