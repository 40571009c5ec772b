"""End-to-end engine on the GPU: every scheme matches the CPU (fp64 torch) engine round by round."""
import numpy as np
import pytest
import torch

from erasurehead_amd.config import RunConfig
from erasurehead_amd.data.source import ArraySource
from erasurehead_amd.engine import Trainer, evaluate
from erasurehead_amd.parallel.dist import DistEnv

pytestmark = pytest.mark.gpu

CASES = [  # (is_coded, partitions, coded_ver, n_procs, s, num_collect)
    (0, 0, 0, 5, 0, 0),
    (1, 0, 0, 7, 2, 0),
    (1, 0, 1, 7, 2, 0),
    (1, 0, 2, 7, 2, 0),
    (1, 0, 3, 7, 2, 4),
    (1, 4, 1, 7, 1, 0),
    (1, 4, 0, 7, 1, 0),
]


def _source(n_parts, rows, d, seed=0):
    rng = np.random.RandomState(seed)
    parts = [(rng.randn(rows, d) * 0.2, rng.choice([-1.0, 1.0], rows)) for _ in range(n_parts)]
    test = (rng.randn(rows, d) * 0.2, rng.choice([-1.0, 1.0], rows))
    return ArraySource(parts, test)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("rule", ["GD", "AGD"])
@pytest.mark.parametrize("native_loop,device_loop", [(True, "graph"), (True, "stream"), (True, "off"), (False, "off")])
def test_gpu_matches_cpu(case, rule, native_loop, device_loop, native):
    is_coded, P, ver, n_procs, s, k = case
    W = n_procs - 1
    d, rows = 33, 40
    from erasurehead_amd.codes import make_scheme, scheme_key

    key = scheme_key(is_coded, P, ver)
    probe = make_scheme(key, W, s, rows * W, k, P, rng=np.random.RandomState(0))
    n_parts = probe.n_partition_files
    n = rows * n_parts
    src = _source(n_parts, rows, d)
    out = {}
    for dev in ("cpu", "cuda"):
        cfg = RunConfig(n_procs, n, d, "/tmp/eh_gpu_eng/", 0, "x", is_coded, s, P, ver, k, 0, rule, num_itrs=8,
                        seed=0, verbose=False, native_loop=native_loop, device_loop=device_loop)
        env = DistEnv(device=torch.device(dev))
        sch = make_scheme(key, W, s, n, k, P, rng=np.random.RandomState(0))
        tr = Trainer(cfg, env, src, scheme=sch)
        assert tr.native_loop == (dev == "cuda" and native_loop)
        res = tr.run()
        if dev == "cuda":
            assert tr.device_loop == (None if device_loop == "off" else device_loop)
            assert np.all(res.timeset > 0) and np.all(np.isfinite(res.timeset))
            out["arr_" + dev] = res.arrivals
        else:
            out["arr_" + dev] = res.arrivals
        out[dev] = res.betaset
        if dev == "cuda":
            ev = evaluate(tr, res, write=False)
            assert np.all(np.isfinite(ev.training_loss))
    np.testing.assert_allclose(out["cuda"], out["cpu"], rtol=1e-9, atol=1e-11)
    # same arrival sets and order, round by round
    assert [[(w, p) for (w, p, _t) in r] for r in out["arr_cuda"]] == \
        [[(w, p) for (w, p, _t) in r] for r in out["arr_cpu"]]


def test_gpu_device_loop_timed_segments(native):
    """bench-style timed fence inside a device-driven run: two graph segments, same betas as host-driven."""
    src = _source(6, 40, 33)
    out = {}
    for mode in ("graph", "off"):
        cfg = RunConfig(7, 240, 33, "/tmp/eh_gpu_eng/", 0, "x", 1, 2, 0, 3, 4, 0, "AGD", num_itrs=12, seed=0,
                        verbose=False, device_loop=mode)
        from erasurehead_amd.codes import make_scheme

        sch = make_scheme("approx", 6, 2, 240, 4, 0, rng=np.random.RandomState(0))
        tr = Trainer(cfg, DistEnv(device=torch.device("cuda")), src, scheme=sch)
        res = tr.run(timed_start=5)
        assert res.timed_rounds == 7 and res.timed_seconds > 0
        out[mode] = res.betaset
    np.testing.assert_allclose(out["graph"], out["off"], rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("mode", ["graph", "stream"])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("case", [(1, 0, 3, 7, 2, 4), (1, 0, 0, 7, 2, 0), (0, 0, 0, 5, 0, 0)])
def test_gpu_fused_update_is_bitwise_identical(case, precision, mode, native):
    """Device-driven local rounds with the combine + update inside the slab reduction
    (grad_dense.hip slab_reduce_update) give bitwise the betas of the separate slab_reduce_final +
    combine_update launches, AGD and GD, fp64 and fp32 messages, d not a multiple of the 64-column
    chunk."""
    is_coded, P, ver, n_procs, s, k = case
    from erasurehead_amd.codes import make_scheme, scheme_key

    W = n_procs - 1
    key = scheme_key(is_coded, P, ver)
    d, rows = 150, 64
    n_parts = make_scheme(key, W, s, rows * W, k, P, rng=np.random.RandomState(0)).n_partition_files
    src = _source(n_parts, rows, d, seed=3)
    out = {}
    for fused in (True, False):
        for rule in ("AGD", "GD"):
            cfg = RunConfig(n_procs, rows * n_parts, d, "/tmp/eh_gpu_eng/", 0, "x", is_coded, s, P, ver, k, 0, rule,
                            num_itrs=9, seed=0, verbose=False, device_loop=mode, precision=precision)
            sch = make_scheme(key, W, s, rows * n_parts, k, P, rng=np.random.RandomState(0))
            tr = Trainer(cfg, DistEnv(device=torch.device("cuda")), src, scheme=sch)
            tr.fused_update = fused
            res = tr.run()
            assert tr.device_loop == mode
            out[(fused, rule)] = res.betaset
    for rule in ("AGD", "GD"):
        assert np.array_equal(out[(True, rule)], out[(False, rule)]), rule


def test_gpu_delay_semantics(native):
    """AGC with the reference Exp(0.5)*0.02 delays: time-to-decode tracks the deterministic floor."""
    from erasurehead_amd.utils.delay import delay_floor

    W, s, k = 6, 2, 4
    rows, d = 50, 20
    src = _source(W, rows, d)
    cfg = RunConfig(W + 1, rows * W, d, "/tmp/eh_gpu_eng/", 0, "x", 1, s, 0, 3, k, 1, "GD", num_itrs=10, seed=0,
                    verbose=False, delay_mean=0.02)
    tr = Trainer(cfg, DistEnv(device=torch.device("cuda")), src)
    res = tr.run()
    floor = delay_floor(W, 10, groups=[w // 3 for w in range(W)], k=k, mean=0.02)
    assert res.timeset.sum() >= floor
    assert res.timeset.sum() < floor + 10 * 0.01  # < 10 ms overhead per round


def test_native_loop_timeout_falls_back_to_host_decode(native):
    """Cyclic code with s+1 dead workers: rounds time out, the native executor hands the
    off-table completion pattern back to the host decode and training continues."""
    W, s = 6, 1
    rows, d = 30, 12
    src = _source(W, rows, d)
    cfg = RunConfig(W + 1, rows * W, d, "/tmp/eh_gpu_eng/", 0, "x", 1, s, 0, 0, 0, 1, "GD", num_itrs=3, seed=0,
                    verbose=False, kill_workers=[2, 4], delay_mode="none", round_timeout=0.2)
    tr = Trainer(cfg, DistEnv(device=torch.device("cuda")), src)
    assert tr.native_loop
    res = tr.run()
    assert res.timeouts == 3
    assert np.all(res.worker_timeset[:, [1, 3]] == -1)
    assert np.all(np.isfinite(res.betaset))


def test_native_loop_large_cyclic_table_on_demand(native):
    """C(20, 8) = 125970 completion patterns: the native executor fills its decode table on demand."""
    from erasurehead_amd.codes import make_scheme

    W, s, rows, d = 20, 8, 12, 9
    src = _source(W, rows, d)
    out = {}
    for dev in ("cpu", "cuda"):
        cfg = RunConfig(W + 1, rows * W, d, "/tmp/eh_gpu_eng/", 0, "x", 1, s, 0, 0, 0, 0, "GD", num_itrs=4, seed=0,
                        verbose=False)
        sch = make_scheme("coded", W, s, rows * W, rng=np.random.RandomState(0))
        tr = Trainer(cfg, DistEnv(device=torch.device(dev)), src, scheme=sch)
        assert tr.native_loop == (dev == "cuda")
        res = tr.run()
        assert res.timeouts == 0
        out[dev] = res.betaset
    np.testing.assert_allclose(out["cuda"], out["cpu"], rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("ver,k", [(3, 4), (0, 0), (2, 0)])
@pytest.mark.parametrize("native_loop", [True, False])
def test_gpu_sparse_onehot_matches_cpu(ver, k, native_loop, native):
    """One-hot CSR data (the real datasets' layout) through the ELL path vs the CPU engine."""
    from erasurehead_amd.codes import make_scheme, scheme_key
    from erasurehead_amd.data.synthetic import onehot_partitions

    W, s = 6, 2
    parts, test, d = onehot_partitions(6 * 150, 400, 8, W, seed=11)
    src = ArraySource(parts, test, sparse=True)
    n = sum(p[0].shape[0] for p in parts)
    key = scheme_key(1, 0, ver)
    out = {}
    for dev in ("cpu", "cuda"):
        cfg = RunConfig(W + 1, n, d, "/tmp/eh_gpu_eng/", 1, "covtype", 1, s, 0, ver, k, 0, "AGD", num_itrs=6,
                        seed=0, verbose=False, native_loop=native_loop)
        sch = make_scheme(key, W, s, n, k, 0, rng=np.random.RandomState(0))
        tr = Trainer(cfg, DistEnv(device=torch.device(dev)), src, scheme=sch)
        if dev == "cuda":
            assert tr.plan.ell
        res = tr.run()
        out[dev] = res.betaset
    np.testing.assert_allclose(out["cuda"], out["cpu"], rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("precision,tol", [("fp32", 2e-4), ("bf16", 2e-2)])
def test_gpu_reduced_precision_tracks_fp64(precision, tol, native):
    """fp32 / bf16 worker storage: the trajectory stays close to the fp64 engine."""
    case = (1, 0, 3, 7, 2, 4)
    is_coded, P, ver, n_procs, s, k = case
    W, d, rows = n_procs - 1, 64, 200
    src = _source(W, rows, d)
    out = {}
    for prec in ("fp64", precision):
        cfg = RunConfig(n_procs, rows * W, d, "/tmp/eh_gpu_eng/", 0, "x", is_coded, s, P, ver, k, 0, "AGD",
                        num_itrs=10, seed=0, verbose=False, precision=prec, lr=1.0)
        from erasurehead_amd.codes import make_scheme

        sch = make_scheme("approx", W, s, rows * W, k, P, rng=np.random.RandomState(0))
        res = Trainer(cfg, DistEnv(device=torch.device("cuda")), src, scheme=sch).run()
        out[prec] = res.betaset
    err = np.max(np.abs(out[precision] - out["fp64"])) / np.max(np.abs(out["fp64"]))
    assert err < tol, err


@pytest.mark.parametrize("case", [c for c in CASES if c[4] > 0 and c[2] != 2])
@pytest.mark.parametrize("native_loop", [True, False])
def test_gpu_share_partitions_matches_cpu(case, native_loop, native):
    """--share-partitions on the GPU (distinct partitions once + encode.hip) vs the faithful CPU engine."""
    from erasurehead_amd.codes import make_scheme, scheme_key
    from erasurehead_amd.ops.grad import SharedGradPlan

    is_coded, P, ver, n_procs, s, k = case
    W, d, rows = n_procs - 1, 33, 40
    key = scheme_key(is_coded, P, ver)
    n_parts = make_scheme(key, W, s, rows * W, k, P, rng=np.random.RandomState(0)).n_partition_files
    src = _source(n_parts, rows, d)
    out = {}
    for dev, share in (("cpu", False), ("cuda", True)):
        cfg = RunConfig(n_procs, rows * n_parts, d, "/tmp/eh_gpu_eng/", 0, "x", is_coded, s, P, ver, k, 0, "AGD",
                        num_itrs=8, seed=0, verbose=False, native_loop=native_loop, share_partitions=share)
        sch = make_scheme(key, W, s, rows * n_parts, k, P, rng=np.random.RandomState(0))
        tr = Trainer(cfg, DistEnv(device=torch.device(dev)), src, scheme=sch)
        assert isinstance(tr.plan, SharedGradPlan) == share
        out[dev] = tr.run().betaset
    np.testing.assert_allclose(out["cuda"], out["cpu"], rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("ver,k", [(3, 4), (0, 0)])
def test_gpu_share_partitions_sparse(ver, k, native):
    """Shared partitions over the one-hot ELL path."""
    from erasurehead_amd.codes import make_scheme, scheme_key
    from erasurehead_amd.data.synthetic import onehot_partitions
    from erasurehead_amd.ops.grad import SharedGradPlan

    W, s = 6, 2
    parts, test, d = onehot_partitions(6 * 150, 400, 8, W, seed=11)
    src = ArraySource(parts, test, sparse=True)
    n = sum(p[0].shape[0] for p in parts)
    out = {}
    for dev, share in (("cpu", False), ("cuda", True)):
        cfg = RunConfig(W + 1, n, d, "/tmp/eh_gpu_eng/", 1, "covtype", 1, s, 0, ver, k, 0, "AGD", num_itrs=6,
                        seed=0, verbose=False, share_partitions=share)
        sch = make_scheme(scheme_key(1, 0, ver), W, s, n, k, 0, rng=np.random.RandomState(0))
        tr = Trainer(cfg, DistEnv(device=torch.device(dev)), src, scheme=sch)
        if share:
            assert isinstance(tr.plan, SharedGradPlan) and tr.plan.inner.ell
        out[dev] = tr.run().betaset
    np.testing.assert_allclose(out["cuda"], out["cpu"], rtol=1e-9, atol=1e-11)


def test_gpu_amazon_scale_onehot(native):
    """Amazon-shaped stand-in (26215 x 241915 one-hot, 45 nnz per row; ref run_approx_coding.sh:30-32,
    src/arrange_real_data.py:34-91; synthetic, parity unpinned): AGC W=8, s=1, k=6 through the
    native launcher (CSR row pass -- a 1.94 MB beta does not fit the LDS of the ELL one --, 1.94 MB
    messages, 242k-column combine+update) and the native
    sparse evaluation, against the fp64 CPU engine + scipy/torch evaluation."""
    from erasurehead_amd.codes import make_scheme
    from erasurehead_amd.data.synthetic import REAL_SHAPES, onehot_partitions

    n_am, d_am, f_am = REAL_SHAPES["amazon-dataset"]
    W, s, k = 8, 1, 6
    parts, test, d = onehot_partitions(n_am, d_am, f_am, W, seed=21)
    assert d == d_am
    src = ArraySource(parts, test, sparse=True)
    n = sum(p[0].shape[0] for p in parts)
    out = {}
    for dev in ("cpu", "cuda"):
        cfg = RunConfig(W + 1, n, d, "/tmp/eh_gpu_amazon/", 1, "amazon-dataset", 1, s, 0, 3, k, 0, "AGD", num_itrs=5,
                        seed=0, verbose=False, fix_quirks=True)
        sch = make_scheme("approx", W, s, n, k, 0)
        tr = Trainer(cfg, DistEnv(device=torch.device(dev)), src, scheme=sch)
        if dev == "cuda":
            assert not tr.plan.ell and tr.native_loop  # (ops/grad.py SparseGradPlan use_ell="auto")
        res = tr.run()
        ev = evaluate(tr, res, write=False)
        out[dev] = (res.betaset, ev.training_loss, ev.testing_loss, ev.auc)
    np.testing.assert_allclose(out["cuda"][0], out["cpu"][0], rtol=1e-9, atol=1e-11)
    for a, b in zip(out["cuda"][1:], out["cpu"][1:]):
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12)
