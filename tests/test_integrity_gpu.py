"""Message integrity tags on the IPC mailbox path (csrc/kernels/integrity.h), on the GPU.

Kernel level: a tagged put writes the payload, one (round + 1, rank, checksum) tag per row and the
counter; the tags match the host reference checksum (erasurehead_amd/parallel/integrity.py) and
the receiver-side check accepts clean rows and reports a flipped byte or a stale round.

Engine level (ranks sharing the GPU over the IPC mailbox, like tests/test_multiproc_gpu.py): the
sabotage hook flips one payload byte of one put AFTER its checksum (a torn put), and the run must
fail with an error naming the round, the rank and the mailbox slot: on the host-driven master
pump (a check kernel queued behind the next round's beta and local gradient), on the device
arbiter (the next round's idle waves check while wave 0 polls) and for beta on a worker (checked
behind the round that read it).  All checks sit off the round's critical path.  Also the
per-pair preflight.
"""
import json
import os
import uuid

import numpy as np
import pytest
import torch

from erasurehead_amd.parallel.integrity import parse_tags, row_checksum
from test_multiproc_gpu import _launch_raw

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,ld,rows", [(torch.float64, 1000, 3), (torch.float32, 1000, 1), (torch.float64, 24, 64)])
def test_tagged_put_tags_match_host_checksum(native, dtype, ld, rows):
    C = native
    flags = C.ShmFlags("/eh_t_" + uuid.uuid4().hex[:12], 2, True)
    try:
        g = torch.Generator(device="cuda").manual_seed(5)
        src = torch.randn((rows, ld), dtype=dtype, device="cuda", generator=g)
        dst = torch.zeros_like(src)
        tags = torch.zeros(rows * 16, dtype=torch.uint8, device="cuda")
        counters = torch.zeros(64, dtype=torch.int32, device="cuda")
        csum = torch.zeros(64, dtype=torch.int64, device="cuda")
        C.put_signal_tagged(src, dst, tags, flags.dev_addr(0), 7, 3, counters, csum)
        torch.cuda.synchronize()
        assert torch.equal(dst, src) and flags.load(0) == 7
        assert int(csum.abs().sum()) == 0 and int(counters.abs().sum()) == 0  # scratch left zero
        got = parse_tags(tags.cpu().numpy().tobytes())
        want = [(7, 3, row_checksum(src[r].cpu().numpy())) for r in range(rows)]
        assert got == want
        assert C.verify_rows(dst, tags, 7, 3) == {}
        # a stale round and a wrong sender are both caught
        assert C.verify_rows(dst, tags, 8, 3)["round1_got"] == 7
        assert C.verify_rows(dst, tags, 7, 2)["rank_got"] == 3
    finally:
        flags.close()


def test_torn_put_is_detected(native):
    C = native
    flags = C.ShmFlags("/eh_t_" + uuid.uuid4().hex[:12], 2, True)
    try:
        src = torch.linspace(-1, 1, 2 * 1000, dtype=torch.float64, device="cuda").reshape(2, 1000)
        dst = torch.zeros_like(src)
        tags = torch.zeros(32, dtype=torch.uint8, device="cuda")
        counters = torch.zeros(64, dtype=torch.int32, device="cuda")
        csum = torch.zeros(64, dtype=torch.int64, device="cuda")
        C.put_signal_tagged(src, dst, tags, flags.dev_addr(0), 5, 1, counters, csum, corrupt=True)
        torch.cuda.synchronize()
        diff = (dst != src).nonzero()
        assert diff.shape[0] == 1 and tuple(diff[0].tolist()) == (0, 0)  # one element, low mantissa byte
        assert abs(float(dst[0, 0] - src[0, 0])) < 1e-12  # numerically invisible...
        err = C.verify_rows(dst, tags, 5, 1)  # ...but the checksum sees it
        assert err and err["sum_got"] == row_checksum(src[0].cpu().numpy())
        assert err["sum_calc"] == row_checksum(dst[0].cpu().numpy())
    finally:
        flags.close()


def _fails(world, case_i, expect, **env):
    r = _launch_raw(world, case_i, "AGD", env)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-3000:]
    assert expect in out, out[-4000:]
    return out


def test_sabotaged_message_fails_host_pump(tmp_path):
    # naive (case 0): every message enters the decode, so the torn rows are always read
    out = _fails(3, 0, "message integrity check failed: round 3, rank 1's message in mailbox slot",
                 ERASUREHEAD_SABOTAGE="msg:1:3", ERASUREHEAD_DEVICE_MASTER="off", EH_TEST_ROUND_TIMEOUT="20",
                 EH_TEST_OUT=str(tmp_path / "x.npz"))
    assert "tag says round 3 rank 1" in out


def test_sabotaged_message_fails_arbiter(tmp_path):
    # round 5's idle waves check round 4's rows while wave 0 polls: round 5 fails, naming round 4
    _fails(3, 0, "device-driven round 5: message integrity check failed: round 4, rank 2's message",
           ERASUREHEAD_SABOTAGE="msg:2:4", ERASUREHEAD_DEVICE_MASTER="on", ERASUREHEAD_WORKER_WAIT="device",
           EH_TEST_ROUND_TIMEOUT="20", EH_TEST_OUT=str(tmp_path / "x.npz"))


def test_sabotaged_beta_fails_worker(tmp_path):
    _fails(3, 1, "rank 1: message integrity check failed: beta of round 2 from rank 0",
           ERASUREHEAD_SABOTAGE="beta:1:2", ERASUREHEAD_DEVICE_MASTER="off", EH_TEST_ROUND_TIMEOUT="20",
           EH_TEST_OUT=str(tmp_path / "x.npz"))


def test_untagged_transport_still_trains(tmp_path):
    """--no-integrity (A/B runs) keeps the plain put + signal path working."""
    from oracle import replay
    from test_engine_cpu import CASES, make

    out = str(tmp_path / "u.npz")
    r = _launch_raw(3, 1, "AGD", dict(EH_TEST_OUT=out, EH_TEST_NO_INTEGRITY="1"))
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    z = np.load(out, allow_pickle=True)
    cfg, src, sch, parts = make(CASES[1], "AGD")
    arrivals = [[(w, p, 0.0) for (w, p) in a] for a in z["arrivals"]]
    ref = replay(sch, parts, z["beta0"], arrivals, "AGD", cfg.alpha_value, cfg.n_rows, 10.0 * np.ones(len(arrivals)))
    np.testing.assert_allclose(z["betaset"], ref, rtol=1e-9, atol=1e-11)


def test_preflight_records_every_pair(tmp_path):
    out = str(tmp_path / "p.npz")
    r = _launch_raw(3, 1, "AGD", dict(EH_TEST_OUT=out, EH_TEST_PREFLIGHT="200"))
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    pf = json.loads(str(np.load(out, allow_pickle=True)["preflight"]))
    assert [p["rank"] for p in pf] == [1, 2]
    for p in pf:
        assert p["iters"] == 200 and p["payload_errors_master_to_rank"] == 0 and p["payload_errors_rank_to_master"] == 0
        assert 0 < p["rtt_us_p50"] <= p["rtt_us_p99"] <= p["rtt_us_max"]
