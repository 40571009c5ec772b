"""Multi-process engine on the GPU: ranks share one MI355X and talk over the IPC mailbox.

Each case is launched with torchrun as child processes (2 and 3 ranks on the one GPU of the
test box; on an 8-GPU node the same code path runs one rank per GPU over xGMI), and the
master's trajectory is replayed with the fp64 NumPy oracle on the arrival sets it reports.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch_raw(world, case_i, rule, extra_env, delay=0.0, timeout=600):
    """torchrun `world` ranks of mp_engine_run.py; returns the CompletedProcess (out path: EH_TEST_OUT)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "mp_engine_run.py"),
           env.get("EH_TEST_OUT", os.devnull), str(case_i), rule, str(delay)]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)


def _launch(world, case_i, rule, out, delay=0.0, **extra_env):
    r = _launch_raw(world, case_i, rule, dict(extra_env, EH_TEST_OUT=out), delay)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return np.load(out, allow_pickle=True)  # our own file (contains the arrival lists)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case_i", [0, 1, 4, 6])
def test_ipc_multiprocess_matches_replay(world, case_i, tmp_path):
    from oracle import replay
    from test_engine_cpu import CASES, make

    r = _launch(world, case_i, "AGD", str(tmp_path / "r.npz"))
    assert str(r["transport"]) == "ipc"
    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    eta = 10.0 * np.ones(len(arrivals))
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, eta)
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("world,case_i", [(8, 5), (5, 5), (4, 7)])
def test_ipc_many_ranks(world, case_i, tmp_path):
    """The 8-GPU layout (one logical worker per rank, 8 ranks) rehearsed on one GPU."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    r = _launch(world, case_i, "AGD", str(tmp_path / "m.npz"))
    assert str(r["transport"]) == "ipc"
    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("wait", ["device", "host"])
def test_ipc_worker_wait_modes(wait, tmp_path):
    """Worker rounds with the beta wait on the device stream (hipStreamWaitValue64; the default
    when a rank has its GPU to itself) or on the host, the message put fused into the final
    reduction (the put as its own kernel runs in the physically-late-rank tests): both match the
    oracle replay."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    r = _launch(3, 1, "AGD", str(tmp_path / "w.npz"), ERASUREHEAD_WORKER_WAIT=wait)
    assert str(r["transport"]) == "ipc"
    cfg, src, sch, parts = make(CASES[1], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("world,case_i,wait,drain", [(2, 2, "device", ""), (3, 4, "host", ""), (3, 5, "device", ""),
                                                     (3, 0, "device", ""), (8, 5, "device", ""),
                                                     (3, 1, "device", "all"), (3, 6, "device", "all"),
                                                     (3, 7, "host", "all")])
def test_device_arbiter_rounds(world, case_i, wait, drain, tmp_path):
    """Multi-rank rounds driven by the arbiter kernel (csrc/kernels/arbiter.hip: the master GPU polls the
    workers' counters, applies the stop rule, decodes, updates and releases the next beta): the
    trajectory replays exactly from the arrivals it logged (FRC, AGC, uneven AGC groups, naive; and
    with a drain, the cyclic-MDS decode table, partial replication and partial coded)."""
    from oracle import replay, stops_exactly_at_last
    from test_engine_cpu import CASES, make

    extra = {"EH_TEST_DRAIN": drain} if drain else {}
    r = _launch(world, case_i, "AGD", str(tmp_path / "a.npz"), ERASUREHEAD_DEVICE_MASTER="on",
                ERASUREHEAD_WORKER_WAIT=wait, EH_TEST_ROUND_TIMEOUT="20", **extra)
    assert str(r["transport"]) == "ipc" and str(r["round_loop"]) == "arbiter"
    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    assert all(len(a) for a in arrivals)
    assert stops_exactly_at_last(sch, arrivals)  # the wave-parallel books: no late arrival logged, no early stop
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)
    assert np.all(r["timeset"] > 0)


@pytest.mark.parametrize("master", ["on", "off"])
def test_strict_release_forms(master, tmp_path):
    """ERASUREHEAD_RELEASE=strict (launchers.h strict_release): every put, signal and arbiter release
    in the job uses the release-ordered stores and acquire polls of before round 4, the switch for a
    first cross-GPU node; 3 integrity-tagged ranks on the arbiter and on the host pump replay exactly."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    r = _launch(3, 4, "AGD", str(tmp_path / "s.npz"), ERASUREHEAD_RELEASE="strict", ERASUREHEAD_DEVICE_MASTER=master,
                ERASUREHEAD_WORKER_WAIT="device", EH_TEST_ROUND_TIMEOUT="20")
    assert str(r["transport"]) == "ipc"
    assert (str(r["round_loop"]) == "arbiter") == (master == "on")
    cfg, src, sch, parts = make(CASES[4], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


def test_ipc_multiprocess_delayed_agc(tmp_path):
    """AGC (W=6, s=2, k=4) with the reference delay model: the decode only uses fast workers."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    r = _launch(3, 4, "GD", str(tmp_path / "d.npz"), delay=0.01)
    cfg, src, sch, parts = make(CASES[4], "GD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    for i, a in enumerate(r["arrivals"]):
        d = np.random.RandomState(i).exponential(0.01, 6)
        used = {w for (w, p) in a}
        slowest = int(np.argmax(d))
        if d[slowest] - np.sort(d)[-2] > 0.004:  # a clear straggler never makes the cut
            assert slowest not in used or len(used) == 6
    ref = replay(sch, parts, r["beta0"], arrivals, "GD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


def test_cli_two_ranks_synthetic(tmp_path):
    """main.py under torchrun (2 ranks sharing the GPU): reference console lines and result files."""
    import re

    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    root = str(tmp_path) + "/"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(os.path.dirname(HERE), "main.py"),
           "7", "60000", "200", root, "0", "synthetic", "1", "2", "0", "3", "4", "0", "AGD", "--data", "synthetic",
           "--num-itrs", "20", "--seed", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert any(l.startswith("---- Starting Approx Coding Iterations for 2 stragglers") for l in lines)
    its = [l for l in lines if re.match(r"^Iteration \d+: Train Loss = ", l)]
    assert len(its) == 20
    losses = [float(l.split("Train Loss = ")[1].split(",")[0]) for l in its]
    assert losses[-1] < losses[0]
    assert os.path.exists(os.path.join(root, "results", "replication_acc_2_training_loss.dat"))


def _gpu_count():
    import torch

    return torch.cuda.device_count()


@pytest.mark.parametrize("transport", ["ipc", "rccl"])
@pytest.mark.parametrize("case_i", [4, 1])
def test_one_rank_per_gpu_matches_replay(transport, case_i, tmp_path, monkeypatch):
    """SURVEY §4 layer 5: one rank per MI355X (2-4 GPUs), IPC over xGMI and RCCL p2p, against the
    fp64 oracle.  Skipped on one-GPU boxes (there RCCL cannot run two ranks on one device)."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    n = _gpu_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs")
    monkeypatch.setenv("ERASUREHEAD_TRANSPORT", transport)
    r = _launch(min(4, n), case_i, "AGD", str(tmp_path / "g.npz"))
    assert str(r["transport"]) == transport
    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


def test_ipc_handshake_failure_names_pair_and_step(tmp_path, monkeypatch):
    """A worker rank that never answers the setup handshake: --transport ipc fails with an error
    naming the pair and the step instead of training on garbage or hanging."""
    monkeypatch.setenv("ERASUREHEAD_TRANSPORT", "ipc")
    monkeypatch.setenv("ERASUREHEAD_SABOTAGE", "handshake:1")
    monkeypatch.setenv("EH_TEST_ROUND_TIMEOUT", "3")  # the handshake waits at most the run's round timeout
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(HERE, "mp_engine_run.py"),
           str(tmp_path / "x.npz"), "4", "AGD"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    err = r.stdout + r.stderr
    assert "IPC mailbox handshake failed" in err and "rank 1 -> rank 0: message flag never signalled" in err, err[-3000:]


@pytest.mark.parametrize("transport", ["ipc", "loopback"])
def test_physically_late_worker_ranks_decode_in_landing_order(transport, tmp_path):
    """--delay-on worker on the native pumps, the reference topology (rank 0 the master only, one logical
    worker per worker rank): each worker rank spins Exp delays on the device between its gradient and its
    put, the master's collector sees the real flags / receive events.  Cyclic W=3 s=1 with a drain:
    checked against the ranks' own device records (tests/lazy_check.py, no host-timing model): every
    round decodes the first 2 messages in landing order, every round spun its full delay, and the
    trajectory replays through the oracle.  Over the IPC mailbox and over the RCCL code path (loopback)."""
    import json

    from lazy_check import check_lazy_device
    from oracle import replay
    from test_engine_cpu import make

    case, mean, R = (1, 0, 0, 4, 1, 0), 0.03, 12
    over = dict(add_delay=1, delay_mode="exp", delay_mean=mean, delay_on="worker", shard="message", drain="all",
                dedicated_master=True, device_records=True)
    env = {"ERASUREHEAD_TRANSPORT": transport} if transport != "ipc" else {}
    r = _launch(4, 0, "GD", str(tmp_path / "p.npz"), EH_TEST_CASE=json.dumps(case), EH_TEST_CFG=json.dumps(over),
                EH_TEST_ROUND_TIMEOUT="30", **env)
    assert str(r["transport"]) == transport
    cfg, src, sch, parts = make(case, "GD")
    owner = {int(w): int(o) for w, o in json.loads(str(r["owner"])).items()}
    skipped = json.loads(str(r["skipped"]))
    d = np.asarray(json.loads(str(r["delays"])))
    arrivals = [[int(w) for (w, p) in a] for a in r["arrivals"]]
    got = check_lazy_device(arrivals, json.loads(str(r["records"])), owner, skipped, d, "count", 2, [0, 1, 2],
                            transport)
    assert got["rounds"] == R and got["spins"] >= 2 * R and got["inversions"] <= 1
    assert all(len(a) == 2 for a in arrivals)
    full = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], full, "GD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(full)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)
    rep = json.loads(str(r["rank_report"]))
    assert rep["round_loop"] == "native pump"


def test_dead_worker_with_drain_never_feeds_stale_messages(tmp_path):
    """a dead logical worker in a draining scheme makes every master round last a stop-rule
    wait plus a drain timeout.  Healthy worker ranks with device-side beta waits must keep waiting
    (their timeout exceeds the master's worst round) instead of releasing their queued rounds on a
    beta that never arrived; the run completes and replays exactly through the oracle."""
    import json

    from oracle import replay
    from test_engine_cpu import CASES, make

    over = dict(kill_workers=[2], round_timeout=1.5, num_itrs=4)
    r = _launch(3, 2, "AGD", str(tmp_path / "k.npz"), EH_TEST_CFG=json.dumps(over), ERASUREHEAD_WORKER_WAIT="device")
    cfg, src, sch, parts = make(CASES[2], "AGD")
    assert all(1 not in {w for (w, p) in a} for a in r["arrivals"])
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("world,case_i,native", [(2, 4, True), (3, 1, True), (4, 7, True), (8, 5, True), (3, 4, False)])
def test_loopback_comm_matches_replay(world, case_i, native, tmp_path):
    """The RCCL transport's code path (csrc/runtime/comm.h: per-peer stream-ordered send/recv, a HIP
    event behind every receive feeding the collector, the native pumps' comm mode) on one GPU,
    where RCCL itself refuses two ranks: the loopback communicator has the same semantics over IPC
    staging rings.  2-8 ranks, every trajectory replayed through the fp64 oracle; also the Python
    round loop over the same communicator."""
    import json

    from oracle import replay
    from test_engine_cpu import CASES, make

    extra = {} if native else {"EH_TEST_CFG": json.dumps({"native_loop": False})}
    r = _launch(world, case_i, "AGD", str(tmp_path / "l.npz"), ERASUREHEAD_TRANSPORT="loopback", **extra)
    assert str(r["transport"]) == "loopback"
    assert json.loads(str(r["rank_report"]))["round_loop"] == ("native pump" if native else "python")
    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)


def test_loopback_dead_worker_teardown_finishes(tmp_path):
    """a worker rank that stops mid-run on the stream-ordered p2p path (the loopback twin of
    RCCL) and never sends again.  Its receives stay queued on the master's per-peer streams; the
    master's final drain times out, aborts the communicator (which releases them) before anything
    synchronises the device, and the run ends with that reason instead of hanging in a device sync.
    (The rank hangs rather than exits: an exited rank resets the gloo control sockets, the surviving
    worker's post-run collectives fail first and the launcher tears the job down before the
    master's drain deadline.)"""
    import json
    import time

    over = dict(round_timeout=5.0, num_itrs=12, drain="lazy")
    t0 = time.time()
    r = _launch_raw(3, 4, "AGD", dict(EH_TEST_OUT=str(tmp_path / "x.npz"), ERASUREHEAD_TRANSPORT="loopback",
                                      ERASUREHEAD_SABOTAGE="hang:2:4", EH_TEST_CFG=json.dumps(over)), timeout=400)
    assert time.time() - t0 < 300
    err = r.stdout + r.stderr
    assert "messages never arrived; aborting the transport" in err, err[-3000:]


def test_loopback_lazy_with_ranks_hosting_no_message(tmp_path):
    """over stream-ordered p2p with the lazy drain, the master's end-of-run beta(R) goes only
    to the ranks that send messages (their WorkerPumps wait for it); ranks hosting no logical worker
    run the Python worker loop, which receives beta(0..R-1) only, so an end-of-run send to them would
    stay unmatched.  AGC W=6 on 8 ranks (workers on ranks 0-5, ranks 6 and 7 idle) completes and
    replays through the oracle."""
    import json

    from oracle import replay
    from test_engine_cpu import CASES, make

    over = dict(shard="message", drain="lazy", round_timeout=20.0)
    r = _launch(8, 4, "AGD", str(tmp_path / "i.npz"), ERASUREHEAD_TRANSPORT="loopback", EH_TEST_CFG=json.dumps(over))
    assert str(r["transport"]) == "loopback"
    owner = json.loads(str(r["owner"]))
    assert sorted(set(owner.values())) == [0, 1, 2, 3, 4, 5]
    reps = json.loads(str(r["reports"]))
    assert [x["messages"] for x in reps][6:] == [0, 0] and all(x["drain"] == "lazy" for x in reps)
    cfg, src, sch, parts = make(CASES[4], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in r["arrivals"]]
    ref = replay(sch, parts, r["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(r["betaset"], ref, rtol=1e-9, atol=1e-11)
