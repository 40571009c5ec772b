"""Child of tests/test_rccl_gpu.py: the rccl-self round loop in a FRESH process whose HIP runtime
starts with GPU_MAX_HW_QUEUES=32 (set by the parent before anything touches the GPU).

Thread ranks share one process, so all their streams (each rank's compute / send / receive streams,
RCCL's own) share its hardware queues; beyond the queue count a stream wait parked in a shared queue
stalls the stream that would release it.  32 queues hold the 2- and 3-rank loops without sharing.

    python tests/rccl_self_run.py <world> <case index>   -> prints "RCCL_SELF_RESULT <json>"
"""
import copy
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    world, case_i = int(sys.argv[1]), int(sys.argv[2])
    import numpy as np

    from oracle import replay, stops_exactly_at_last
    from test_engine_cpu import CASES, make

    import erasurehead_amd
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

    out = run_thread_ranks(world, fn, timeout=40)
    res, beta0, rep, sends = out[0]
    R = cfg.num_itrs
    senders = sum(1 for o in out[1:] if o[2]["messages"])
    ref = replay(sch, parts, beta0, res.arrivals, "AGD", cfg.alpha_value, cfg.n_rows, cfg.eta())
    err = float(np.max(np.abs(res.betaset - ref)) / max(1e-30, np.max(np.abs(ref))))
    print("RCCL_SELF_RESULT " + json.dumps({
        "hw_queues": erasurehead_amd.HW_QUEUES, "transport": rep["transport"], "round_loop": rep["round_loop"],
        "worker_loops": [o[2]["round_loop"] for o in out[1:] if o[2]["messages"]],
        "sends": int(sends), "min_sends": (world - 1) * R + senders * R,
        "stops_exactly": bool(stops_exactly_at_last(sch, res.arrivals)), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
