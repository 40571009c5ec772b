"""RCCL on the one-GPU test box (round-3 verdict: RcclComm had never executed an RCCL call).

* ``rccl-self``: master and worker ranks as threads of one process (parallel/dist.py ThreadEnv), the
  native pumps' comm mode over 1-rank RCCL communicators whose grouped ncclSend + ncclRecv to self
  move every beta and every message (csrc/runtime/comm.cpp RcclSelfLoop); the trajectory replays
  exactly through the fp64 oracle.
* RcclComm between two processes on one GPU ends with a named outcome within a deadline, never a hang.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _fresh_env(**kw):
    """A fresh process at the package's own hardware-queue setting (16: erasurehead_amd/__init__.py)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2", **kw)
    env.pop("GPU_MAX_HW_QUEUES", None)
    return env


@pytest.mark.parametrize("world,case_i", [(2, 4), (3, 1)])
def test_rccl_self_loop_pumps_match_replay(world, case_i):
    """In a fresh process at the package's 16 hardware queues (tests/rccl_self_run.py): thread ranks share
    one process, so all their streams share its queues; past the queue count a stream wait parked in a
    shared queue stalls the stream that would release it (seen at 3 ranks with 16 queues while the master
    kept a send and a receive stream per peer).  One link stream per peer (drain all / carry) keeps the
    3-rank loop within them."""
    env = _fresh_env()
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_self_run.py"), str(world), str(case_i)], env=env,
                       capture_output=True, text=True, timeout=115)
    res = [json.loads(l.split("RCCL_SELF_RESULT ", 1)[1]) for l in r.stdout.splitlines() if "RCCL_SELF_RESULT " in l]
    assert r.returncode == 0 and len(res) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    x = res[0]
    assert x["hw_queues"] == 16
    assert x["transport"] == "rccl-self" and x["round_loop"] == "native pump"
    assert all(l == "native pump" for l in x["worker_loops"])
    assert x["sends"] >= x["min_sends"]  # every beta and every message went through ncclSend/ncclRecv
    assert x["stops_exactly"]
    assert x["rel_err"] < 1e-9


@pytest.mark.parametrize("world,late", [(2, 2), (3, 3)])
def test_rccl_self_lazy_late_rank_skips_stale_rounds(world, late):
    """Drain lazy over RCCL (thread ranks, rccl-self): one worker rank is physically 40 ms late every round
    (a device spin before its send).  The master never waits for it; the rank receives beta a round ahead on
    its own stream, finds every later round stale before it starts (beta(i+1) already landed) and skips its
    gradient, still sending the round's stale rows so the FIFO pairing of ncclSend / ncclRecv holds.  Those
    rows land after their round ended and are never decoded; the trajectory replays exactly."""
    case = (1, 0, 3, 5, 1, 3)  # AGC W=4 s=1 k=3: groups {0,1}, {2,3}
    R = 16
    cfg = dict(add_delay=1, delay_mode="fixed", fixed_stragglers=[late], fixed_sleep=0.04, delay_on="worker",
               shard="message", drain="lazy", num_itrs=R, round_timeout=30.0)
    env = _fresh_env(EH_TEST_CASE=json.dumps(case), EH_TEST_RULE="GD", EH_TEST_CFG=json.dumps(cfg))
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_self_run.py"), str(world), "0"], env=env,
                       capture_output=True, text=True, timeout=115)
    res = [json.loads(l.split("RCCL_SELF_RESULT ", 1)[1]) for l in r.stdout.splitlines() if "RCCL_SELF_RESULT " in l]
    assert r.returncode == 0 and len(res) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    x = res[0]
    assert x["transport"] == "rccl-self" and x["drain"] == "lazy"
    late_rank = [int(k) for k, ws in x["owned"].items() if late - 1 in ws]
    assert late_rank and late_rank[0] != 0
    late_ws = set(x["owned"][str(late_rank[0])])
    assert not late_ws & set(x["arrived_workers"])  # the late rank's messages never reach a decode
    assert len(x["skipped"][str(late_rank[0])]) >= R - 4  # it ran a handful of rounds, skipped the rest
    assert x["loop_s"] < 0.04 * R / 4  # its 40 ms never enter the master's rounds
    assert x["stale_arrivals"] >= 1
    assert x["stops_exactly"] and x["rel_err"] < 1e-9


def test_rccl_comm_two_processes_one_gpu_named_outcome(tmp_path):
    """RCCL refuses two ranks on one device: RcclComm's ncclCommInitRank must fail with a named error
    on both ranks (or, should this RCCL accept it, carry a round trip), within a deadline."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(HERE, "rccl_dup_gpu.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    # the two ranks share the launcher's stdout: their lines can interleave, so decode each JSON
    # object where its marker starts
    dec, res, i = json.JSONDecoder(), [], r.stdout.find("RCCL_RESULT ")
    while i >= 0:
        res.append(dec.raw_decode(r.stdout, i + len("RCCL_RESULT "))[0])
        i = r.stdout.find("RCCL_RESULT ", i + 1)
    assert len(res) == 2, r.stdout[-3000:] + r.stderr[-3000:]
    for x in res:
        if "refused" in x:
            assert "ncclCommInitRank" in x["refused"]
        else:
            assert x["accepted"] and x["echo_ok"]
