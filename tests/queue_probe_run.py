"""Child of tests/test_queues_gpu.py: the master's comm stream set for an 8-rank run, built by a real
MasterPump in a FRESH process whose HIP runtime starts with GPU_MAX_HW_QUEUES as the parent set it.

    python tests/queue_probe_run.py <world> <lazy 0|1>   -> prints "QUEUE_PROBE <json>"

The pump's streams (compute + per-peer comm streams, MasterPump::set_comm) each park a wait on a host flag;
the flags are released in reverse order and every stream must run on at once (stream_wait_probe): none
waits behind another's parked wait, i.e. no two of them share an in-order hardware queue.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    world, lazy = int(sys.argv[1]), bool(int(sys.argv[2]))
    import torch

    import erasurehead_amd
    from erasurehead_amd._ext import native

    C = native()
    dev = torch.cuda.current_device()
    W, R, K, d = world - 1, 8, 2, 16
    col = C.Collector(W, list(range(W)), W)
    pump = C.MasterPump(col, W, R, K, d, d, dev, 10.0)
    pump.set_skip_stale(lazy)
    comm = C.LoopbackComm(dev, [])  # no channels: the probe only needs the pump's streams
    pump.set_comm(comm, [(r, r - 1, 1) for r in range(1, world)], list(range(1, world)))
    streams = pump.stream_handles()
    ok = C.stream_wait_probe(streams, 2.0)
    torch.cuda.synchronize()
    print("QUEUE_PROBE " + json.dumps({"hw_queues": erasurehead_amd.HW_QUEUES, "comm_streams": int(pump.comm_streams),
                                       "streams": len(streams), "independent": [bool(x) for x in ok]}), flush=True)


if __name__ == "__main__":
    main()
