"""Two processes, ONE GPU, one RcclComm between them (launched by tests/test_rccl_gpu.py under torchrun).

RCCL is expected to refuse two ranks on one device at ncclCommInitRank; every rank prints one line
RCCL_RESULT <json> saying what happened ({"refused": msg} or, if the library accepted it, whether a
send/recv round trip over it carried the data), so the test can assert a named outcome, never a hang.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import torch.distributed as dist

    from erasurehead_amd._ext import native

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = native()
    ids = [C.nccl_unique_id(), C.nccl_unique_id()] if rank == 0 else None
    box = [ids]
    dist.broadcast_object_list(box, src=0)
    ids = box[0]
    links = [(1, "out", ids[0], 0), (1, "in", ids[1], 1)] if rank == 0 else [(0, "in", ids[0], 1), (0, "out", ids[1], 0)]
    out = {}
    try:
        comm = C.RcclComm(0, links)
        x = torch.arange(256, dtype=torch.float64, device="cuda") + 1.0
        y = torch.zeros_like(x)
        if rank == 0:
            comm.send(1, x)
            comm.recv(1, y)
        else:
            comm.recv(0, y)
            comm.send(0, y)
        torch.cuda.synchronize()
        out = {"accepted": True, "echo_ok": bool(torch.equal(x, y)) if rank == 0 else True}
        comm.abort()
    except RuntimeError as e:
        out = {"refused": str(e)[:400]}
    print("RCCL_RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
