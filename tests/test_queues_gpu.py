"""Hardware-queue headroom of the master's p2p stream set (round-4 verdict, Weak #8).

HIP maps streams onto at most GPU_MAX_HW_QUEUES in-order hardware queues; a stream beyond them shares a
queue, and a receive parked on a straggler there would hold back another worker's.  The package raises the
limit to 16 (erasurehead_amd/__init__.py).  An 8-rank master needs compute + one link stream per peer with
the reference's drains (8 of 16) and compute + a send and a receive stream per peer with the lazy drain
(15 of 16); a real MasterPump builds that set in a fresh process at 16 queues and every stream runs on at
once when the others are parked (tests/queue_probe_run.py).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("lazy,streams", [(0, 8), (1, 15)])
def test_eight_rank_master_streams_never_share_a_queue(lazy, streams):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "queue_probe_run.py"), "8", str(lazy)], env=env,
                       capture_output=True, text=True, timeout=100)
    res = [json.loads(l.split("QUEUE_PROBE ", 1)[1]) for l in r.stdout.splitlines() if "QUEUE_PROBE " in l]
    assert r.returncode == 0 and len(res) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    x = res[0]
    assert x["hw_queues"] == 16
    assert x["streams"] == streams and x["comm_streams"] == streams - 1
    assert all(x["independent"]), x  # no stream parked behind another's wait
