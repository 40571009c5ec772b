"""RCCL on the one-GPU test box (round-3 verdict: RcclComm had never executed an RCCL call).

* ``rccl-self``: master and worker ranks as threads of one process (parallel/dist.py ThreadEnv), the
  native pumps' comm mode over 1-rank RCCL communicators whose grouped ncclSend + ncclRecv to self
  move every beta and every message (csrc/runtime/comm.cpp RcclSelfLoop); the trajectory replays
  exactly through the fp64 oracle.
* RcclComm between two processes on one GPU ends with a named outcome within a deadline, never a hang.
"""
import copy
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


# (At 4 thread ranks the one process holds ~16 streams plus RCCL's own: more than its hardware queues,
# and a stream wait parked in a shared queue stalls the stream that would release it -- the hang the
# per-rank processes of a real node never see, one process per GPU.  2 and 3 ranks stay within them.)
@pytest.mark.parametrize("world,case_i", [(2, 4), (3, 1)])
def test_rccl_self_loop_pumps_match_replay(world, case_i):
    from oracle import replay, stops_exactly_at_last
    from test_engine_cpu import CASES, make

    from erasurehead_amd.engine import Trainer
    from erasurehead_amd.parallel.dist import run_thread_ranks

    cfg, src, sch, parts = make(CASES[case_i], "AGD")
    cfg.num_itrs, cfg.transport = 10, "rccl-self"

    def fn(env):
        tr = Trainer(copy.deepcopy(cfg), env, src, scheme=sch)
        res = tr.run()
        rep = tr.rank_report()
        sends = tr.tx.selfloop.rccl_sends
        beta0 = getattr(tr, "beta0", None)
        tr.close()
        return res, beta0, rep, sends

    out = run_thread_ranks(world, fn, timeout=240)
    res, beta0, rep, sends = out[0]
    assert rep["transport"] == "rccl-self" and rep["round_loop"] == "native pump"
    assert all(o[2]["round_loop"] == "native pump" for o in out[1:] if o[2]["messages"])
    R = cfg.num_itrs
    senders = sum(1 for o in out[1:] if o[2]["messages"])
    assert sends >= (world - 1) * R + senders * R  # every beta and every message went through ncclSend/ncclRecv
    assert stops_exactly_at_last(sch, res.arrivals)
    ref = replay(sch, parts, beta0, res.arrivals, "AGD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    np.testing.assert_allclose(res.betaset, ref, rtol=1e-9, atol=1e-11)


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
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=180)
    res = [json.loads(l.split("RCCL_RESULT ", 1)[1]) for l in r.stdout.splitlines() if "RCCL_RESULT " in l]
    assert len(res) == 2, r.stdout[-3000:] + r.stderr[-3000:]
    for x in res:
        if "refused" in x:
            assert "ncclCommInitRank" in x["refused"]
        else:
            assert x["accepted"] and x["echo_ok"]
