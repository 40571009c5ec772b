"""One rank of a multi-process engine run (launched by torchrun from tests/test_multiproc_gpu.py).

python -m torch.distributed.run --nproc-per-node N tests/mp_engine_run.py OUT.npz CASE_INDEX RULE [delay_mean]
Builds the same seeded ArraySource as tests/test_engine_cpu.py::make, trains on the GPU(s)
with the ranks' transport (ranks sharing one GPU -> IPC mailboxes) and writes, on rank 0,
the betaset, beta0 and per-round arrival lists so the test can replay them with the fp64
NumPy oracle.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def main():
    out, case_i, rule = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    delay = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    from erasurehead_amd.engine import Trainer
    from erasurehead_amd.parallel.dist import init_distributed
    from test_engine_cpu import CASES, make

    env = init_distributed(os.environ.get("EH_TEST_DEVICE", "cuda"))
    extra = {"delay_mean": delay} if delay else {}
    case = tuple(json.loads(os.environ["EH_TEST_CASE"])) if os.environ.get("EH_TEST_CASE") else CASES[case_i]
    cfg, src, sch, parts = make(case, rule, **extra)
    cfg.num_itrs = 12
    for k, v in json.loads(os.environ.get("EH_TEST_CFG", "{}")).items():  # RunConfig overrides
        setattr(cfg, k, v)
    if os.environ.get("EH_TEST_ROUND_TIMEOUT"):
        cfg.round_timeout = float(os.environ["EH_TEST_ROUND_TIMEOUT"])
    if delay:
        cfg.add_delay = 1
        cfg.force_delay = True
    if os.environ.get("EH_TEST_DRAIN"):
        cfg.drain = os.environ["EH_TEST_DRAIN"]
    if os.environ.get("EH_TEST_SHARD"):
        cfg.shard = os.environ["EH_TEST_SHARD"]
    if os.environ.get("EH_TEST_NO_INTEGRITY"):
        cfg.integrity = False
    tr = Trainer(cfg, env, src, scheme=sch)
    pf = tr.preflight(int(os.environ["EH_TEST_PREFLIGHT"])) if os.environ.get("EH_TEST_PREFLIGHT") else None
    ts = int(os.environ["EH_TEST_TIMED_START"]) if os.environ.get("EH_TEST_TIMED_START") else None
    res = tr.run(timed_start=ts)  # timed_start: the rounds run in two segments with a fence between them
    reports = env.gather_objects(tr.rank_report())  # every rank's (stale rounds skipped, ...)
    skipped = env.gather_objects([int(i) for i in getattr(tr, "skipped_rounds", [])])

    def plain(x):
        if isinstance(x, np.ndarray):
            return x.tolist()
        if isinstance(x, dict):
            return {k: plain(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return [plain(v) for v in x]
        return x
    records = env.gather_objects(plain(tr.device_records)) if cfg.device_records else None
    if env.is_master:
        arr = np.array([[(w, p) for (w, p, _) in a] for a in res.arrivals], dtype=object)
        t_rel = np.array([[t for (_, _, t) in a] for a in res.arrivals], dtype=object)
        np.savez(out, betaset=res.betaset, beta0=tr.beta0, arrivals=arr, t_rel=t_rel, transport=np.array(tr.transport),
                 timeset=res.timeset, loop_time=res.loop_time, round_loop=np.array(tr.device_loop or "host"),
                 preflight=np.array(json.dumps(pf)), rank_report=np.array(json.dumps(tr.rank_report())),
                 reports=np.array(json.dumps(reports)), skipped=np.array(json.dumps(skipped)),
                 owner=np.array(json.dumps({int(u.worker): int(o) for u, o in zip(tr.shards, tr.owner)})),
                 records=np.array(json.dumps(records).replace("NaN", "null")),
                 delays=np.array(json.dumps(tr.delay_table().tolist()).replace("Infinity", "1e308")))
    env.barrier()
    tr.close()
    env.shutdown()


if __name__ == "__main__":
    main()
