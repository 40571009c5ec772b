"""Child of tests/test_rccl_gpu.py: the rccl-self round loop in a FRESH process whose HIP runtime
starts with the package's GPU_MAX_HW_QUEUES (erasurehead_amd/__init__.py: 16).

Thread ranks share one process, so all their streams (each rank's compute / link / receive streams,
RCCL's own) share its hardware queues; beyond the queue count a stream wait parked in a shared queue
stalls the stream that would release it.

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

    case = tuple(json.loads(os.environ["EH_TEST_CASE"])) if os.environ.get("EH_TEST_CASE") else CASES[case_i]
    rule = os.environ.get("EH_TEST_RULE", "AGD")
    cfg, src, sch, parts = make(case, rule)
    cfg.num_itrs, cfg.transport = 10, "rccl-self"
    for k, v in json.loads(os.environ.get("EH_TEST_CFG", "{}")).items():  # RunConfig overrides
        setattr(cfg, k, v)

    def fn(env):
        tr = Trainer(copy.deepcopy(cfg), env, src, scheme=sch)
        res = tr.run()
        rep = tr.rank_report()
        sends = tr.tx.selfloop.rccl_sends
        beta0 = getattr(tr, "beta0", None)
        skipped = [int(i) for i in getattr(tr, "skipped_rounds", [])]
        owned = sorted({int(u.worker) for u, o in zip(tr.shards, tr.owner) if o == env.rank})
        tr.close()
        return res, beta0, rep, sends, skipped, owned

    out = run_thread_ranks(world, fn, timeout=40)
    res, beta0, rep, sends = out[0][:4]
    R = cfg.num_itrs
    senders = sum(1 for o in out[1:] if o[2]["messages"])
    ref = replay(sch, parts, beta0, res.arrivals, rule, cfg.alpha_value, cfg.n_rows, cfg.eta())
    err = float(np.max(np.abs(res.betaset - ref)) / max(1e-30, np.max(np.abs(ref))))
    print("RCCL_SELF_RESULT " + json.dumps({
        "hw_queues": erasurehead_amd.HW_QUEUES, "transport": rep["transport"], "round_loop": rep["round_loop"],
        "worker_loops": [o[2]["round_loop"] for o in out[1:] if o[2]["messages"]],
        "sends": int(sends), "min_sends": (world - 1) * R + senders * R,
        "stops_exactly": bool(stops_exactly_at_last(sch, res.arrivals)), "rel_err": err,
        "drain": rep["drain"], "stale_arrivals": rep.get("stale_arrivals"),
        "skipped": {str(r): o[4] for r, o in enumerate(out)}, "owned": {str(r): o[5] for r, o in enumerate(out)},
        "arrived_workers": sorted({int(w) for a in res.arrivals for (w, p, t) in a}),
        "loop_s": float(np.sum(res.loop_time))}), flush=True)


if __name__ == "__main__":
    main()
