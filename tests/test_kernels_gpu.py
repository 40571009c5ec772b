"""Numerics of the gfx950 HIP kernels against fp64 NumPy/PyTorch references (GPU only)."""
import collections

import numpy as np
import pytest
import scipy.sparse as sps
import torch

from erasurehead_amd.models.losses import LEAST_SQUARES, LOGISTIC, least_squares_grad, logistic_grad, logistic_loss, mse
from erasurehead_amd.ops import DenseGradPlan, SparseGradPlan, auc_columns, combine_update, get_precision, loss_sums, predictions
from erasurehead_amd.models.losses import roc_auc, UpdateRule
from erasurehead_amd.ops.grad import KernelChoice

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _parts(rng, sizes, d, prec):
    parts = {}
    host = {}
    for p, n in enumerate(sizes):
        X = rng.randn(n, d) * 0.3
        y = rng.choice([-1.0, 1.0], n)
        Xp = torch.zeros((n, prec.ld(d)), dtype=torch.float64)
        Xp[:, :d] = torch.from_numpy(X)
        Xs = Xp.to(prec.storage)
        host[p] = (Xs[:, :d].double().numpy(), y)  # oracle sees the stored (rounded) values
        parts[p] = (Xs.to(DEV).contiguous(), torch.from_numpy(y).to(prec.acc).to(DEV))
    return parts, host


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 2e-4), ("bf16", 2e-4)])
@pytest.mark.parametrize("d", [1, 37, 1000, 2048, 2500, 5000, 9000, 17000])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
def test_dense_grad(prec_name, tol, d, loss, native):
    """Narrow fused (d <= 2048), wide single-pass (d <= 8192 fp64 / 16384 fp32) and two-pass kernels."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(d + loss)
    parts, host = _parts(rng, [257, 64, 1], d, prec)
    msgs = [[(0, 1.0), (1, -0.7)], [(2, 2.5)], [(1, 1.0), (0, 0.3), (2, 1.0)]]
    plan = DenseGradPlan(msgs, parts, prec, loss, d, target_tasks=7)
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    b = rng.randn(d) * 0.5
    beta[:d] = torch.from_numpy(b).to(prec.acc)
    bh = beta[:d].double().cpu().numpy()
    G = plan.out_buffer()[0]
    plan.run(beta, G)
    torch.cuda.synchronize()
    f = logistic_grad if loss == LOGISTIC else least_squares_grad
    for s, m in enumerate(msgs):
        ref = sum(f(host[p][0], host[p][1], bh, c) for p, c in m)
        got = G[s, :d].double().cpu().numpy()
        err = np.max(np.abs(got - ref)) / max(1e-12, np.max(np.abs(ref)))
        assert err < tol, (s, err)
        assert torch.all(G[s, d:] == 0)
    G2 = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G2)  # the native executors' launch path
    torch.cuda.synchronize()
    assert torch.equal(G, G2)


def test_dense_grad_many_tasks_deterministic(native):
    prec = get_precision("fp64")
    rng = np.random.RandomState(5)
    parts, host = _parts(rng, [5000, 3001], 300, prec)
    plan = DenseGradPlan([[(0, 1.0), (1, 1.0)]], parts, prec, LOGISTIC, 300, target_tasks=100)
    beta = torch.randn(plan.ld, dtype=torch.float64, device=DEV) * 0.1
    G1 = plan.out_buffer()[0]
    G2 = plan.out_buffer()[0]
    plan.run(beta, G1)
    plan.run(beta, G2)
    torch.cuda.synchronize()
    assert torch.equal(G1, G2)  # slab reduction is order-fixed: bitwise reproducible


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 1e-4)])
@pytest.mark.parametrize("pattern_only", [True, False])
@pytest.mark.parametrize("use_ell", [True, False])
def test_sparse_grad_row_blocks(prec_name, tol, pattern_only, use_ell, native):
    """Partitions longer than one column-pass sub-block (4096 rows): the row-blocked CSC tiles with the
    residuals staged in LDS, the sub-block sums added per partition inside the encoding, against the
    scipy oracle, and bitwise equal from run to run."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(17)
    d = 3000
    parts = {}
    for p, n in enumerate((9000, 4097, 300)):
        heavy = rng.choice(3, (n, 1))  # a few heavy columns: spans crossing tiles inside sub-blocks
        rest = np.stack([3 + rng.choice(d - 3, 7, replace=False) for _ in range(n)])
        cols = np.sort(np.concatenate([heavy, rest], axis=1), axis=1)
        vals = np.ones(cols.size) if pattern_only else rng.randn(cols.size)
        X = sps.csr_matrix((vals, cols.ravel(), np.arange(0, cols.size + 1, 8)), shape=(n, d))
        parts[p] = (X, rng.choice([-1.0, 1.0], n))
    msgs = [[(0, 1.0), (1, 0.5)], [(2, -1.5), (0, 2.0)], [(1, 1.0)]]
    plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, d, device=DEV, use_ell=use_ell)
    assert plan.nsub == 3 + 2 + 1 and plan.sub_begin is not None
    assert plan.ell == use_ell and plan.pattern_only == pattern_only
    b = rng.randn(d) * 0.2
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    beta[:d] = torch.from_numpy(b).to(prec.acc)
    bh = beta[:d].double().cpu().numpy()
    G = plan.out_buffer()[0]
    plan.run(beta, G)
    G2 = plan.out_buffer()[0]
    plan.run(beta, G2)
    torch.cuda.synchronize()
    assert torch.equal(G, G2)
    for s, m in enumerate(msgs):
        ref = sum(logistic_grad(parts[p][0], parts[p][1], bh, c) for p, c in m)
        got = G[s, :d].double().cpu().numpy()
        err = np.max(np.abs(got - ref)) / max(1e-12, np.max(np.abs(ref)))
        assert err < tol, (s, err)


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 1e-4)])
@pytest.mark.parametrize("pattern_only", [True, False])
@pytest.mark.parametrize("use_ell", [True, False])
def test_sparse_grad(prec_name, tol, pattern_only, use_ell, native):
    prec = get_precision(prec_name)
    rng = np.random.RandomState(3)
    d = 700
    parts = {}
    for p in range(3):
        n = 400 + 37 * p
        cols = np.stack([rng.choice(d, 5, replace=False) for _ in range(n)])
        vals = np.ones(cols.size) if pattern_only else rng.randn(cols.size)
        X = sps.csr_matrix((vals, cols.ravel(), np.arange(0, cols.size + 1, 5)), shape=(n, d))
        parts[p] = (X, rng.choice([-1.0, 1.0], n))
    msgs = [[(0, 1.0), (1, 0.5)], [(2, -1.5)], [(0, 1.0)]]
    for loss in (LOGISTIC, LEAST_SQUARES):
        plan = SparseGradPlan(msgs, parts, prec, loss, d, device=DEV, use_ell=use_ell)
        assert plan.pattern_only == pattern_only and plan.ell == use_ell
        b = rng.randn(d) * 0.2
        beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
        beta[:d] = torch.from_numpy(b).to(prec.acc)
        bh = beta[:d].double().cpu().numpy()
        G = plan.out_buffer()[0]
        plan.run(beta, G)
        torch.cuda.synchronize()
        f = logistic_grad if loss == LOGISTIC else least_squares_grad
        for s, m in enumerate(msgs):
            ref = sum(f(parts[p][0], parts[p][1], bh, c) for p, c in m)
            got = G[s, :d].double().cpu().numpy()
            err = np.max(np.abs(got - ref)) / max(1e-12, np.max(np.abs(ref)))
            assert err < tol, (loss, s, err)


@pytest.mark.parametrize("d", [700, 30000])
def test_sparse_naive_identity_plan_writes_the_messages(d, native):
    """Naive (message i = distinct partition i, coefficient 1, no sub-blocks): no device encoding, the column
    pass writes the message rows themselves; a second launch into the same buffer gives the same bits; the
    row format follows the beta footprint (ELL with beta in LDS at d = 700, CSR rows at d = 30000: 240 KB of
    fp64 beta does not fit)."""
    prec = get_precision("fp64")
    rng = np.random.RandomState(11)
    parts = {}
    for p in range(3):
        n = 300 + 41 * p
        cols = np.stack([rng.choice(d, 6, replace=False) for _ in range(n)])
        X = sps.csr_matrix((np.ones(cols.size), cols.ravel(), np.arange(0, cols.size + 1, 6)), shape=(n, d))
        parts[p] = (X, rng.choice([-1.0, 1.0], n))
    msgs = [[(p, 1.0)] for p in range(3)]
    plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, d, device=DEV)
    assert plan.identity and plan.ell == (d == 700)
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    beta[:d] = torch.from_numpy(rng.randn(d) * 0.2)
    bh = beta[:d].double().cpu().numpy()
    G = plan.out_buffer()[0]
    plan.run(beta, G)
    torch.cuda.synchronize()
    first = G.clone()
    plan.run(beta, G)
    torch.cuda.synchronize()
    assert torch.equal(G, first)
    for s, m in enumerate(msgs):
        ref = sum(logistic_grad(parts[p][0], parts[p][1], bh, c) for p, c in m)
        got = G[s, :d].double().cpu().numpy()
        assert np.max(np.abs(got - ref)) / max(1e-12, np.max(np.abs(ref))) < 1e-11
    assert torch.all(G[:, d:] == 0)


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 1e-4)])
@pytest.mark.parametrize("wide,idx16", [(20000, True), (70000, False)])
def test_ell_onehot_blocks_and_wide_windows(prec_name, tol, wide, idx16, native):
    """One-hot feature blocks plus one feature with a 20000- or 70000-category window: 16-bit window
    offsets in the row pass while every window fits 2^16, int32 columns beyond; both through plan.run
    and the native GradLauncher, and bitwise reproducible (no float atomics in the column pass)."""
    from erasurehead_amd.data.synthetic import onehot_partitions

    prec = get_precision(prec_name)
    rng = np.random.RandomState(9)
    parts_l, _, d = onehot_partitions(3000, 900, 6, 3, seed=4)
    parts = {}
    for p, (X, y) in enumerate(parts_l):
        extra = sps.csr_matrix((np.ones(X.shape[0]), d + rng.randint(0, wide, X.shape[0]),
                                np.arange(X.shape[0] + 1)), shape=(X.shape[0], d + wide))
        Xw = sps.csr_matrix(sps.hstack([X, sps.csr_matrix((X.shape[0], wide))]) + extra)
        Xw.sort_indices()
        parts[p] = (Xw, y)
    D = d + wide
    msgs = [[(0, 1.0), (1, 0.5)], [(2, -1.5)]]
    b = rng.randn(D) * 0.1
    for loss in (LOGISTIC, LEAST_SQUARES):
        plan = SparseGradPlan(msgs, parts, prec, loss, D, device=DEV, use_ell=True)  # (auto: CSR past LDS)
        assert plan.ell and plan.idx16 == idx16 and plan.row16
        beta = torch.zeros(prec.ld(D), dtype=prec.acc, device=DEV)
        beta[:D] = torch.from_numpy(b).to(prec.acc)
        bh = beta[:D].double().cpu().numpy()
        f = logistic_grad if loss == LOGISTIC else least_squares_grad
        for via_launcher in (False, True):
            G = plan.out_buffer()[0]
            if via_launcher:
                plan.native_launcher().launch(beta, G)
            else:
                plan.run(beta, G)
            torch.cuda.synchronize()
            for s_, m in enumerate(msgs):
                ref = sum(f(parts[p][0], parts[p][1], bh, c) for p, c in m)
                got = G[s_, :D].double().cpu().numpy()
                err = np.max(np.abs(got - ref)) / max(1e-12, np.max(np.abs(ref)))
                assert err < tol, (loss, via_launcher, s_, err)
            if via_launcher:
                G2 = plan.out_buffer()[0]
                plan.run(beta, G2)
                torch.cuda.synchronize()
                assert torch.equal(G, G2)  # bitwise, run to run


def test_sparse_replicas_share_reads_and_match_per_message(native):
    """FRC / AGC replicas on one GPU: every distinct partition is streamed once and each message is
    encoded from it with its own coefficient; the result matches the per-message oracle and is
    bitwise identical over repeated runs (covtype-like one-hot blocks, 4 partitions x 2 replicas)."""
    from erasurehead_amd.data.synthetic import onehot_partitions

    prec = get_precision("fp64")
    parts_l, _, d = onehot_partitions(40000, 2000, 12, 4, seed=2)
    parts = {p: xy for p, xy in enumerate(parts_l)}
    msgs = [[(w, 1.0), ((w + 1) % 4, 1.0)] for w in range(4)] + [[(w, -0.5)] for w in range(4)]
    plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, d, device=DEV)
    assert plan.basis == [0, 1, 2, 3] and plan.msg_rows == 3 * plan.nrows
    rng = np.random.RandomState(1)
    b = rng.randn(d) * 0.1
    beta = torch.zeros(prec.ld(d), dtype=torch.float64, device=DEV)
    beta[:d] = torch.from_numpy(b)
    G1, G2 = plan.out_buffer()[0], plan.out_buffer()[0]
    plan.run(beta, G1)
    plan.run(beta, G2)
    torch.cuda.synchronize()
    assert torch.equal(G1, G2)
    for s_, m in enumerate(msgs):
        ref = sum(logistic_grad(parts[p][0], parts[p][1], b, c) for p, c in m)
        got = G1[s_, :d].double().cpu().numpy()
        assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-11


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 1e-4)])
@pytest.mark.parametrize("rows,use_ell", [(1500, True), (3100, True), (3100, False)])
def test_sparse_frc_units_write_every_replica(prec_name, tol, rows, use_ell, native):
    """FRC / AGC messages (each group's members send the sum of the group's partitions, coefficient 1,
    ref src/replication.py:56-68): the device stacks a group's partitions into one unit, the column pass
    stages the whole unit (up to 8192 rows, 8 residuals per thread: the UNITS variant) and writes its sums into
    every member's message row -- no partition rows, no encoding launch.  Every row against the scipy
    oracle, bitwise run to run, through plan.run and the native launcher, padding columns untouched."""
    from erasurehead_amd.data.synthetic import onehot_partitions

    prec = get_precision(prec_name)
    parts_l, _, d = onehot_partitions(4 * rows, 1800, 9, 4, seed=6)
    parts = {p: xy for p, xy in enumerate(parts_l)}
    msgs = [[(0, 1.0), (1, 1.0)], [(0, 1.0), (1, 1.0)], [(2, 1.0), (3, 1.0)], [(2, 1.0), (3, 1.0)], [(2, 1.0), (3, 1.0)]]
    plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, d, device=DEV, use_ell=use_ell)
    assert plan.units == [(0, 1), (2, 3)] and plan.identity and plan.sub_begin is None
    assert plan.dst.cpu().tolist() == [[0, 1, -1, -1], [2, 3, 4, -1]]
    rng = np.random.RandomState(2)
    b = rng.randn(d) * 0.1
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    beta[:d] = torch.from_numpy(b).to(prec.acc)
    bh = beta[:d].double().cpu().numpy()
    G1, G2 = plan.out_buffer()[0], plan.out_buffer()[0]
    plan.run(beta, G1)
    plan.native_launcher().launch(beta, G2)
    torch.cuda.synchronize()
    assert torch.equal(G1, G2)
    for s_, m in enumerate(msgs):
        ref = sum(logistic_grad(parts[p][0], parts[p][1], bh, c) for p, c in m)
        got = G1[s_, :d].double().cpu().numpy()
        assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < tol, s_
    assert torch.equal(G1[0], G1[1]) and torch.equal(G1[2], G1[4])
    assert torch.all(G1[:, d:] == 0)


@pytest.mark.parametrize("rule", ["GD", "AGD"])
@pytest.mark.parametrize("msg_dtype", [torch.float64, torch.float32])
def test_combine_update(rule, msg_dtype, native):
    rng = np.random.RandomState(1)
    d, ld = 1001, 1002
    msgs_h = [rng.randn(ld) for _ in range(5)]
    msgs = [torch.from_numpy(m).to(msg_dtype).to(DEV) for m in msgs_h]
    coefs = [1.0, -0.5, 0.0, 2.0, 0.25]
    b0 = rng.randn(ld)
    b0[d:] = 0
    u0 = rng.randn(ld)
    u0[d:] = 0
    beta = torch.from_numpy(b0.copy()).to(DEV)
    u = torch.from_numpy(u0.copy()).to(DEV)
    hist = torch.zeros(ld, dtype=torch.float64, device=DEV)
    bw = torch.full((ld,), 7.0, dtype=torch.float32, device=DEV)
    g_out = torch.zeros(ld, dtype=torch.float64, device=DEV)
    up = UpdateRule(rule, 1e-3, 5000)
    i = 3
    decay, gm, l2, theta, code = up.coeffs(i, 10.0)
    combine_update(msgs, coefs, beta, u, d, decay, gm, l2, theta, code, hist=hist, beta_w=bw, g_out=g_out)
    torch.cuda.synchronize()
    g = sum(c * torch.from_numpy(m).to(msg_dtype).double().numpy() for c, m in zip(coefs, msgs_h))[:d]
    bref, uref = b0[:d].copy(), u0[:d].copy()
    up.apply(i, 10.0, bref, uref, g)
    np.testing.assert_allclose(g_out[:d].cpu().numpy(), g, rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(beta[:d].cpu().numpy(), bref, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(hist[:d].cpu().numpy(), bref, rtol=1e-13, atol=1e-13)
    if rule == "AGD":
        np.testing.assert_allclose(u[:d].cpu().numpy(), uref, rtol=1e-12, atol=1e-12)
    assert torch.all(bw[d:] == 0)
    np.testing.assert_allclose(bw[:d].cpu().double().numpy(), bref.astype(np.float32), rtol=1e-6)


@pytest.mark.parametrize("prec_name,tol", [("fp64", 1e-11), ("fp32", 2e-5), ("bf16", 2e-5)])
@pytest.mark.parametrize("R", [1, 16, 100, 130])
def test_eval_gemm_loss(prec_name, tol, R, native):
    prec = get_precision(prec_name)
    rng = np.random.RandomState(R)
    n, d = 333, 257
    X = rng.randn(n, d) * 0.2
    y = rng.choice([-1.0, 1.0], n)
    Xp = torch.zeros((n, prec.ld(d)), dtype=torch.float64)
    Xp[:, :d] = torch.from_numpy(X)
    Xs = Xp.to(prec.storage)
    Xh = Xs[:, :d].double().numpy()
    B = torch.zeros((R, prec.ld(d)), dtype=torch.float64)
    B[:, :d] = torch.from_numpy(rng.randn(R, d) * 0.3)
    Bh = B[:, :d].to(prec.acc).double().numpy()
    Xd = Xs.to(DEV)
    Bd = B.to(DEV)
    for kind in (LOGISTIC, LEAST_SQUARES):
        sums, nn = loss_sums([(Xd, torch.from_numpy(y).to(DEV))], Bd, d, kind)
        P = Xh @ Bh.T
        ref = np.array([logistic_loss(y, P[:, j], 1) if kind == LOGISTIC else mse(y, P[:, j]) * n for j in range(R)])
        assert nn == n
        np.testing.assert_allclose(sums, ref, rtol=tol * 10, atol=tol)
    Pd = predictions(Xd, Bd, d).double().cpu().numpy()
    np.testing.assert_allclose(Pd, Xh @ Bh.T, rtol=tol * 10, atol=tol)
    auc = auc_columns(torch.from_numpy(y).to(DEV), torch.from_numpy(Xh @ Bh.T).to(DEV))
    np.testing.assert_allclose(auc, [roc_auc(y, (Xh @ Bh.T)[:, j]) for j in range(R)], rtol=1e-12)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_encode_messages(dtype, native):
    """encode.hip: G = E . Gb over a sparse E, against the fp64 torch product."""
    rng = np.random.RandomState(3)
    nb, ns, ld = 5, 7, 1003
    Gb = torch.from_numpy(rng.randn(nb, ld)).to(dtype).cuda()
    ptr, idx, coef = [0], [], []
    E = np.zeros((ns, nb))
    for s in range(ns):
        for b in rng.choice(nb, size=1 + s % 3, replace=False):
            c = rng.randn()
            idx.append(int(b))
            coef.append(c)
            E[s, b] = c
        ptr.append(len(idx))
    G = torch.full((ns, ld), float("nan"), dtype=dtype, device="cuda")
    native.encode_messages(Gb, torch.tensor(ptr, dtype=torch.int32, device="cuda"),
                           torch.tensor(idx, dtype=torch.int32, device="cuda"),
                           torch.tensor(coef, dtype=torch.float64, device="cuda"), G)
    ref = E @ Gb.double().cpu().numpy()
    tol = 1e-13 if dtype == torch.float64 else 1e-5
    np.testing.assert_allclose(G.double().cpu().numpy(), ref, rtol=tol, atol=tol)


MESSAGE_MAJOR = KernelChoice("fused", rows=1)  # one row per wave, message-major tasks: the plain reference


@pytest.mark.parametrize("prec_name", ["fp64", "fp32", "bf16"])
def test_dense_grad_interleaved_dispatch_is_bitwise_identical(prec_name, native):
    """Replica-interleaved task order: same bits as message-major order."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(11)
    parts, _ = _parts(rng, [3000, 2000, 1000], 1000, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(1, 0.5), (2, -1.0)]] * 2 + [[(2, 1.0)]]
    a = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000, target_tasks=256,
                      choice=KernelChoice("fused", rows=1, interleave=True))
    b = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000, target_tasks=256, choice=MESSAGE_MAJOR)
    assert a.max_rep > 1 and not torch.equal(a.tasks, b.tasks)
    beta = torch.randn(a.ld, dtype=prec.acc, device=DEV) * 0.05
    Ga, Gb = a.out_buffer()[0], b.out_buffer()[0]
    a.native_launcher().launch(beta, Ga)
    b.run(beta, Gb)
    torch.cuda.synchronize()
    assert torch.equal(Ga, Gb)


@pytest.mark.parametrize("prec_name", ["fp64", "fp32"])
@pytest.mark.parametrize("d,rows", [(1000, [3000, 2000, 1000]), (3000, [700, 300, 90]), (17000, [300, 200, 50])])
def test_fused_slab_reduction_is_bitwise_the_two_stages(prec_name, d, rows, native):
    """slab_reduce_fused (one launch, the default) sums the slab rows in exactly the two-stage order:
    the messages are bitwise equal to set_slab_reduce_mode(0) (one-wave bundles, wide rows, two-pass)."""
    C = native
    prec = get_precision(prec_name)
    rng = np.random.RandomState(13)
    parts, _ = _parts(rng, rows, d, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(1, 0.5), (2, -1.0)]] * 2 + [[(2, 1.0)]]
    plan = DenseGradPlan(msgs, parts, prec, LOGISTIC, d)
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    out = {}
    try:
        for mode in (0, 1):
            C.set_slab_reduce_mode(mode)
            G = plan.out_buffer()[0]
            plan.run(beta, G)
            torch.cuda.synchronize()
            out[mode] = G.clone()
    finally:
        C.set_slab_reduce_mode(1)
    assert torch.equal(out[0], out[1])
    assert torch.count_nonzero(out[1]) > 0


@pytest.mark.parametrize("d,sizes", [(1000, [3000, 2000, 1000]), (1000, [37, 5, 70]), (504, [900, 33, 64]),
                                     (256, [129, 64, 7])])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
def test_bf16_mfma_vgpr_ring_is_bitwise_the_lds_ring(d, sizes, loss, native):
    """Both feeds of the packed bf16 bundles -- the LDS-DMA stage ring (0) and grad_vring_mfma (the ring
    fed through two / three register sets; 3, 4) -- run the same MFMAs on the same operands in the same
    order, so bitwise the same messages: bundles of 1-3 replicas, partial last stages, d below a full wave
    slice; and against message-major order."""
    prec = get_precision("bf16")
    rng = np.random.RandomState(d + sum(sizes))
    parts, _ = _parts(rng, sizes, d, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(1, 0.5), (2, -1.0)]] * 2 + [[(2, 1.0)]]
    a = DenseGradPlan(msgs, parts, prec, loss, d)
    b = DenseGradPlan(msgs, parts, prec, loss, d, choice=MESSAGE_MAJOR)
    assert a.choice.kind == "mfma"
    beta = torch.randn(a.ld, dtype=prec.acc, device=DEV) * 0.05
    out = []
    try:
        for on in (0, 3, 4):
            native.set_mfma_stream(on)
            G = a.out_buffer()[0]
            a.native_launcher().launch(beta, G)
            torch.cuda.synchronize()
            out.append(G)
    finally:
        native.set_mfma_stream(0)  # the default
    assert all(torch.equal(out[0], o) for o in out[1:])
    Gb = b.out_buffer()[0]
    b.run(beta, Gb)
    torch.cuda.synchronize()
    torch.testing.assert_close(out[1], Gb, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("prec_name", ["fp64", "fp32", "bf16"])
def test_dense_grad_staged_is_the_replica_default(prec_name, native):
    """Co-located replicas in bundles of more than 3 default to the LDS-staged bundles for fp64/fp32
    (MFMA for bf16), and the staged messages match message-major order to rounding."""
    from erasurehead_amd.ops.grad import staged_bundle_rows

    prec = get_precision(prec_name)
    rng = np.random.RandomState(12)
    parts, _ = _parts(rng, [3000, 2000, 1000], 1000, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(1, 0.5), (2, -1.0)]] * 2 + [[(2, 1.0)]]
    a = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000)
    b = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000, choice=MESSAGE_MAJOR)
    assert a.choice.kind == ("mfma" if prec_name == "bf16" else "staged")
    if a.choice.kind == "staged":  # 6000 distinct rows: a short-stream rank, pair form, 128-row bundles
        assert a.choice.pair and a.bundle_rows == staged_bundle_rows(6000) == 128
    beta = torch.randn(a.ld, dtype=prec.acc, device=DEV) * 0.05
    Ga, Gb = a.out_buffer()[0], b.out_buffer()[0]
    a.native_launcher().launch(beta, Ga)
    b.run(beta, Gb)
    torch.cuda.synchronize()
    tol = 1e-12 if prec_name == "fp64" else 1e-4
    torch.testing.assert_close(Ga, Gb, rtol=tol, atol=tol)


@pytest.mark.parametrize("prec_name", ["fp64", "fp32", "bf16"])
def test_dense_grad_one_wave_bundles_are_the_fp64_default(prec_name, native):
    """Bundles of 3 replicas default to grad_dense_multi for fp64 and fp32 (bundle length from
    multi_bundle_rows) and to MFMA for bf16; the messages match message-major order to rounding."""
    from erasurehead_amd.ops.grad import multi_bundle_rows

    prec = get_precision(prec_name)
    rng = np.random.RandomState(13)
    parts, _ = _parts(rng, [3000, 2000, 1000], 1000, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(2, -1.0)]] * 2
    a = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000)
    b = DenseGradPlan(msgs, parts, prec, LOGISTIC, 1000, choice=MESSAGE_MAJOR)
    assert a.choice.kind == {"fp64": "multi", "fp32": "multi", "bf16": "mfma"}[prec_name]
    if a.choice.kind == "multi":
        # (fp32 rows of 16 columns per lane: sized like fp64, ops/grad.py choose_kernel)
        assert a.choice.fold and a.choice.lane_epi and a.bundle_rows == multi_bundle_rows(6000, False)
    beta = torch.randn(a.ld, dtype=prec.acc, device=DEV) * 0.05
    Ga, Gb = a.out_buffer()[0], b.out_buffer()[0]
    a.native_launcher().launch(beta, Ga)
    b.run(beta, Gb)
    torch.cuda.synchronize()
    tol = 1e-12 if prec_name == "fp64" else 1e-4
    torch.testing.assert_close(Ga, Gb, rtol=tol, atol=tol)


def test_eval_gemm_unaligned_rows_use_scalar_staging(native):
    """Rows whose stride is not a 16-byte multiple take the scalar-staging eval kernel (v1)."""
    rng = np.random.RandomState(9)
    n, d, R = 301, 257, 37
    X = torch.from_numpy(rng.randn(n, d) * 0.2).to(DEV)  # ld = 257 doubles: rows not 16-B aligned
    y = torch.from_numpy(rng.choice([-1.0, 1.0], n)).to(DEV)
    B = torch.from_numpy(rng.randn(R, d) * 0.3).to(DEV)
    s = torch.zeros(R, dtype=torch.float64, device=DEV)
    P = torch.empty((n, R), dtype=torch.float64, device=DEV)
    native.eval_gemm_loss(LOGISTIC, X, n, d, y, B, s, P)
    Ph = X.cpu().numpy() @ B.cpu().numpy().T
    np.testing.assert_allclose(P.cpu().numpy(), Ph, rtol=1e-11, atol=1e-11)
    ref = [logistic_loss(y.cpu().numpy(), Ph[:, j], 1) for j in range(R)]
    np.testing.assert_allclose(s.cpu().numpy(), ref, rtol=1e-10)


@pytest.mark.parametrize("layout", ["mixed", "pairs"])
@pytest.mark.parametrize("pair", [False, True])
@pytest.mark.parametrize("rows,d,prec_name", [(64, 1000, "fp64"), (37, 1000, "fp64"), (100, 250, "fp64"),
                                              (64, 1000, "fp32"), (64, 1000, "bf16")])
def test_dense_grad_staged_bundles(native, rows, d, prec_name, pair, layout):
    """LDS-staged replica bundles (rows streamed once through an LDS ring by LDS-DMA, a wave per
    replica) against the fp64 oracle.  Row counts that leave partial stages and partial bundles are
    included.  "mixed": bundles of 5 and 3 replicas (one wave per replica); "pairs": bundles of 2
    (two waves per replica, folded); pair: two rows per step sharing one reduction."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(21)
    parts, host = _parts(rng, [700, 500, 301], d, prec)
    if layout == "mixed":
        msgs = [[(0, 1.0), (1, 1.0)]] * 3 + [[(1, 0.5), (2, -1.0)]] * 2 + [[(2, 1.0)]]
    else:
        msgs = [[(0, 1.0)]] * 2 + [[(1, 1.0), (2, 0.5)], [(1, -1.0), (2, 2.0)]]
    R = max(collections.Counter(p for m in msgs for p, _ in m).values())
    plan = DenseGradPlan(msgs, parts, prec, LOGISTIC, d,
                         choice=KernelChoice("staged", replicas=R, bundle_rows=rows, pair=pair))
    assert plan.bundle_rows == rows
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    G = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G)
    torch.cuda.synchronize()
    bh = beta[:d].double().cpu().numpy()
    tol = 1e-10 if prec_name == "fp64" else 2e-4
    for s, m in enumerate(msgs):
        ref = sum(logistic_grad(host[p][0], host[p][1], bh, c) for p, c in m)
        np.testing.assert_allclose(G[s, :d].double().cpu().numpy(), ref, rtol=tol, atol=tol * 1e-2)


@pytest.mark.parametrize("form", ["fold-lane", "fold-wave", "unfolded"])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
@pytest.mark.parametrize("rows,d,prec_name", [(64, 1000, "fp64"), (37, 1000, "fp64"), (64, 1000, "fp32"),
                                              (33, 500, "fp32")])
def test_dense_grad_one_wave_bundles_of_two(native, rows, d, prec_name, loss, form):
    """grad_dense_multi with bundles of 2 replicas (FRC s = 1: groups of two workers sharing two
    partitions, the default for 2 co-located replicas): each replica's dot product, residual and
    gradient from the shared row registers, distinct coefficients per replica, against the fp64 oracle."""
    fold = form != "unfolded"
    prec = get_precision(prec_name)
    rng = np.random.RandomState(8)
    parts, host = _parts(rng, [700, 501, 300, 64], d, prec)
    msgs = [[(0, 1.0), (1, 1.0)], [(0, 0.5), (1, -2.0)], [(2, 1.0), (3, 1.0)], [(2, -1.0), (3, 3.0)]]
    plan = DenseGradPlan(msgs, parts, prec, loss, d,
                         choice=KernelChoice("multi", replicas=2, bundle_rows=rows, fold=fold,
                                             lane_epi=form == "fold-lane"))
    assert plan.bundle_rows == rows and plan.max_rep == 2
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    G = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G)
    torch.cuda.synchronize()
    bh = beta[:d].double().cpu().numpy()
    f = logistic_grad if loss == LOGISTIC else least_squares_grad
    tol = 1e-10 if prec_name == "fp64" else 2e-4
    atol = tol * 1e-2 if prec_name == "fp64" else 2e-5  # fp32: coefficients up to 3 over 1.2k rows
    for s, m in enumerate(msgs):
        ref = sum(f(host[p][0], host[p][1], bh, c) for p, c in m)
        np.testing.assert_allclose(G[s, :d].double().cpu().numpy(), ref, rtol=tol, atol=atol)


@pytest.mark.parametrize("prec_name", ["fp64", "fp32", "bf16"])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
def test_distinct_rows_default_to_one_wave_bundles_of_one(native, prec_name, loss):
    """Distinct rows (naive, message-placed ranks) at 16 columns per lane pick grad_dense_multi with
    one replica per bundle; messages with two partitions and label coefficients against the oracle."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(17)
    parts, host = _parts(rng, [900, 700, 333, 64], 1000, prec)
    msgs = [[(0, 1.0), (1, 0.5)], [(2, -1.0)], [(3, 2.0)]]
    plan = DenseGradPlan(msgs, parts, prec, loss, 1000)
    assert plan.choice.kind == "multi" and plan.choice.replicas == 1 and plan.max_rep == 1
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    G = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G)
    torch.cuda.synchronize()
    bh = beta[:1000].double().cpu().numpy()
    f = logistic_grad if loss == LOGISTIC else least_squares_grad
    tol = 1e-10 if prec_name == "fp64" else 2e-4
    atol = tol * 1e-2 if prec_name == "fp64" else 2e-5
    for s_, m in enumerate(msgs):
        ref = sum(f(host[p][0], host[p][1], bh, c) for p, c in m)
        np.testing.assert_allclose(G[s_, :1000].double().cpu().numpy(), ref, rtol=tol, atol=atol)


def test_frc_pairs_default_to_one_wave_bundles(native):
    """Two co-located replicas per partition (FRC s = 1) pick grad_dense_multi with R = 2."""
    prec = get_precision("fp64")
    rng = np.random.RandomState(3)
    parts, _ = _parts(rng, [900, 800], 1000, prec)
    plan = DenseGradPlan([[(0, 1.0), (1, 1.0)]] * 2, parts, prec, LOGISTIC, 1000)
    assert plan.choice.kind == "multi" and plan.choice.replicas == 2 and plan.choice.lane_epi


@pytest.mark.parametrize("form", ["fold-lane", "fold-wave", "fold-pair", "unfolded"])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
@pytest.mark.parametrize("rows,d,prec_name", [(64, 1000, "fp64"), (37, 1000, "fp64"), (256, 250, "fp64"),
                                              (33, 500, "fp64"), (64, 1000, "fp32"), (33, 130, "fp32"),
                                              (35, 512, "fp32"), (8, 250, "fp32"), (8, 1000, "fp64"),
                                              # bf16 rows: six in flight per wave (kMultiDepth), bundles ending
                                              # anywhere in the ring
                                              (64, 1000, "bf16"), (37, 1000, "bf16"), (13, 504, "bf16"),
                                              (5, 1000, "bf16")])
def test_dense_grad_one_wave_bundles(native, rows, d, prec_name, loss, form):
    """grad_dense_multi: one wave computes every replica of its bundle from rows double-buffered in
    registers, each replica with its own dot product, residual and gradient.  Bundles of 3 replicas,
    of 2 padded to 3, and partial / odd-length bundles (the two-rows-per-trip loop ends on either
    buffer) against the fp64 oracle; with the workgroup fold (4 bundles of one partition per
    workgroup, pad bundles at partition ends, one slab row per workgroup and replica) and all three
    epilogues (replicas reduce-scattered with one lane per replica's residual, wave-uniform, or two
    rows per 8-value reduce-scatter on narrow rows: odd bundles end on a half pair), and without
    the fold."""
    fold = form != "unfolded"
    prec = get_precision(prec_name)
    if form == "fold-pair" and -(-prec.ld(d) // (64 * prec.vec)) * prec.vec > 8:
        pytest.skip("pair rows: narrow rows only (<= 8 columns per lane)")
    rng = np.random.RandomState(5)
    parts, host = _parts(rng, [700, 501, 300], d, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 2 + [[(0, -0.5), (1, 2.0)]] + [[(2, 1.0)], [(2, -3.0)]]
    plan = DenseGradPlan(msgs, parts, prec, loss, d,
                         choice=KernelChoice("multi", replicas=3, bundle_rows=rows, fold=fold,
                                             lane_epi=form == "fold-lane", pair=form == "fold-pair"))
    assert plan.bundle_rows == rows
    if fold:  # slab rows: one per (workgroup, replica), a contiguous range per message
        stb = plan.slot_task_begin.cpu().numpy()
        assert stb[0] == 0 and np.all(np.diff(stb) > 0) and stb[-1] <= plan.ntasks // 4
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    G = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G)
    torch.cuda.synchronize()
    bh = beta[:d].double().cpu().numpy()
    f = logistic_grad if loss == LOGISTIC else least_squares_grad
    tol = 1e-10 if prec_name == "fp64" else 2e-4
    for s, m in enumerate(msgs):
        ref = sum(f(host[p][0], host[p][1], bh, c) for p, c in m)
        np.testing.assert_allclose(G[s, :d].double().cpu().numpy(), ref, rtol=tol, atol=tol * 1e-2 * max(1.0, np.abs(ref).max()))


@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
@pytest.mark.parametrize("rows,d,prec_name", [(16, 4096, "fp64"), (33, 3000, "fp64"), (64, 8000, "fp32"),
                                              (17, 5000, "bf16"), (20, 4000, "fp32"), (16, 2100, "fp32"),
                                              (9, 3000, "bf16")])
def test_dense_grad_wide_row_bundles(native, rows, d, prec_name, loss):
    """grad_dense_wide with replica bundles: a workgroup loads each wide row once and computes every
    replica's dot product, residual (own coefficient) and gradient from registers (fp32 / bf16 rows
    of <= 4096 columns: the half-width 256-thread instance; wider rows: 512 threads).
    Bundles of 3, of 2 padded to 3 and odd-length bundles against the fp64 oracle, and equal to the
    one-replica wide kernel message by message (to rounding: the row split into tasks differs)."""
    prec = get_precision(prec_name)
    rng = np.random.RandomState(9)
    parts, host = _parts(rng, [301, 200, 77], d, prec)
    msgs = [[(0, 1.0), (1, 1.0)]] * 2 + [[(0, -0.5), (1, 2.0)]] + [[(2, 1.0)], [(2, -3.0)]]
    plan = DenseGradPlan(msgs, parts, prec, loss, d, choice=KernelChoice("wide", replicas=3, bundle_rows=rows))
    assert plan.cpl == 256 and plan.bundle_rows == rows and plan.choice.bundled
    beta = torch.randn(plan.ld, dtype=prec.acc, device=DEV) * 0.05
    G = plan.out_buffer()[0]
    plan.native_launcher().launch(beta, G)
    torch.cuda.synchronize()
    bh = beta[:d].double().cpu().numpy()
    f = logistic_grad if loss == LOGISTIC else least_squares_grad
    tol = 1e-10 if prec_name == "fp64" else 2e-4
    for s, m in enumerate(msgs):
        ref = sum(f(host[p][0], host[p][1], bh, c) for p, c in m)
        np.testing.assert_allclose(G[s, :d].double().cpu().numpy(), ref, rtol=tol,
                                   atol=tol * 1e-2 * max(1.0, np.abs(ref).max()))
    single = DenseGradPlan(msgs, parts, prec, loss, d, choice=KernelChoice("wide"))
    G1 = single.out_buffer()[0]
    single.run(beta, G1)
    torch.cuda.synchronize()
    g1 = G1.double().cpu().numpy()
    np.testing.assert_allclose(G.double().cpu().numpy(), g1, rtol=tol, atol=tol * 1e-2 * max(1.0, np.abs(g1).max()))


@pytest.mark.parametrize("shape", [(20000, 15509, 55), (17290, 27654, 19), (6000, 241915, 45)])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
@pytest.mark.parametrize("R,valued", [(100, False), (300, True), (7, True)])
def test_sparse_eval_kernel(shape, loss, R, valued, native):
    """Hand CSR evaluation kernel (eval_sparse.hip) vs the fp64 scipy oracle on one-hot data shaped
    like covtype / kc_house / amazon (ref src/naive.py:166-169,190-193): predictions and the fused
    loss sums, pattern-only and valued rows, R > 256 column passes."""
    from erasurehead_amd.data.synthetic import onehot_partitions
    from erasurehead_amd.ops.eval import sparse_eval_device

    n, d, m = shape
    parts, test, dd = onehot_partitions(n, d, m, 1, seed=R + loss, least_squares=loss == LEAST_SQUARES)
    X, y = parts[0]
    X = X.tocsr()
    if valued:
        X.data = np.random.RandomState(1).uniform(0.5, 1.5, X.nnz)
    rng = np.random.RandomState(3)
    B = rng.randn(R, dd) * 0.2
    Bt = torch.from_numpy(np.ascontiguousarray(B.T)).to(DEV)
    P, s = sparse_eval_device(X, torch.from_numpy(y), Bt, loss, True)
    Pref = np.asarray(X @ B.T)
    np.testing.assert_allclose(P.cpu().numpy(), Pref, rtol=1e-12, atol=1e-12)
    if loss == LOGISTIC:
        mref = -y[:, None] * Pref
        sref = (np.maximum(mref, 0) + np.log1p(np.exp(-np.abs(mref)))).sum(0)
    else:
        sref = ((y[:, None] - Pref) ** 2).sum(0)
    np.testing.assert_allclose(s.cpu().numpy(), sref, rtol=1e-11)
    _, s2 = sparse_eval_device(X, torch.from_numpy(y), Bt, loss, False)  # loss only, no P
    np.testing.assert_allclose(s2.cpu().numpy(), sref, rtol=1e-11)


def test_mfma_bf16_fragment_maps(native):
    """The lane maps grad_mfma.hip assumes for v_mfma_f32_16x16x32_bf16, checked with exact integers:
    A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], C[row 4(l>>4)+reg][col l&15]."""
    rng = np.random.RandomState(0)
    A = rng.randint(-4, 5, (16, 32)).astype(np.float32)
    B = rng.randint(-4, 5, (32, 16)).astype(np.float32)
    C = torch.zeros(256, dtype=torch.float32, device=DEV)
    native._mfma_probe(torch.from_numpy(A).to(DEV), torch.from_numpy(B).to(DEV), C)
    np.testing.assert_array_equal(C.cpu().numpy().reshape(16, 16), A @ B)


@pytest.mark.parametrize("rowlen", [32, 40, 64])
def test_lds_transpose_read_map(rowlen, native):
    """ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses block row q, columns 4p..4p+3;
    lane i receives column i of the 4 rows (row q in element q).  Two tiles of bf16-exact integers:
    one holding each element's row index, one its column index."""
    rows = np.repeat(np.arange(8, dtype=np.float32)[:, None], rowlen, 1)
    cols = np.repeat(np.arange(rowlen, dtype=np.float32)[None, :], 8, 0)
    got = {}
    for name, tile in (("row", rows), ("col", cols)):
        out = torch.zeros(256, dtype=torch.float32, device=DEV)
        native._tr_probe(torch.from_numpy(np.ascontiguousarray(tile)).reshape(-1).to(DEV), rowlen, out)
        got[name] = out.cpu().numpy().reshape(64, 4)
    for l in range(64):
        g, i = l >> 4, l & 15
        np.testing.assert_array_equal(got["row"][l], [4 * (g & 1) + q for q in range(4)])
        np.testing.assert_array_equal(got["col"][l], [16 * (g >> 1) + i] * 4)


@pytest.mark.parametrize("d", [1000, 1024, 333, 8])
@pytest.mark.parametrize("loss", [LOGISTIC, LEAST_SQUARES])
@pytest.mark.parametrize("pack", [True, False])
def test_mfma_bf16_replica_bundles(d, loss, pack, native):
    """bf16 replica bundles on MFMA (grad_mfma.hip) at the staged geometry: the headline's uneven FRC
    layout (bundles of 3 and 2 replicas) plus cyclic-style distinct coefficients, every message
    against the fp64 oracle on the stored bf16 values; and close to the VALU kernels.  pack: the
    bf16 terms as M rows (R <= 4, the default) or one MFMA per term."""
    native.set_mfma_pack(pack)
    try:
        _mfma_bundles_case(d, loss)
    finally:
        native.set_mfma_pack(True)


def _mfma_bundles_case(d, loss):
    prec = get_precision("bf16")
    rng = np.random.RandomState(d + 7 * loss)
    parts, host = _parts(rng, [1500, 1501, 777], d, prec)
    msgs = [[(0, 1.0), (1, 1.0)], [(1, 1.0), (0, 1.0)], [(0, 1.0), (1, 1.0)],  # group of 3, rotated
            [(2, 1.0)], [(2, 1.0)],  # group of 2
            [(0, 0.5), (2, -1.25)], [(1, 2.0)]]  # distinct coefficients
    plan = DenseGradPlan(msgs, parts, prec, loss, d)
    assert plan.choice.kind == "mfma" and plan.choice.replicas == 4  # partition 0 is read by messages 0, 1, 2 and 5
    beta = torch.zeros(prec.ld(d), dtype=prec.acc, device=DEV)
    b = rng.randn(d) * 0.3
    beta[:d] = torch.from_numpy(b).to(prec.acc)
    G = plan.out_buffer()[0]
    plan.run(beta, G)
    grad = logistic_grad if loss == LOGISTIC else least_squares_grad
    bref = beta[:d].double().cpu().numpy()
    for slot, m in enumerate(msgs):
        ref = sum(grad(host[p][0], host[p][1], bref, c) for p, c in m)
        got = G[slot, :d].double().cpu().numpy()
        err = np.max(np.abs(got - ref)) / max(1e-30, np.max(np.abs(ref)))
        assert err < 2e-4, (slot, err)
    valu = DenseGradPlan(msgs, parts, prec, loss, d, choice=KernelChoice("fused", rows=1, interleave=True))
    G2 = valu.out_buffer()[0]
    valu.run(beta, G2)
    np.testing.assert_allclose(G[:, :d].cpu().numpy(), G2[:, :d].cpu().numpy(), rtol=2e-4,
                               atol=2e-4 * float(G2.abs().max()))
