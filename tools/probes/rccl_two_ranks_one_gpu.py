"""Probe: can two ranks share one GPU for RCCL p2p (for testing the multi-GPU path on a 1-GPU box)?"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=2)
    x = torch.full((1000,), float(rank + 1), device="cuda", dtype=torch.float64)
    t0 = time.perf_counter()
    for i in range(20):
        if rank == 0:
            dist.isend(x, 1).wait()
            dist.irecv(x, 1).wait()
        else:
            dist.irecv(x, 0).wait()
            x += 1
            dist.isend(x, 0).wait()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 20
    print(f"rank {rank} ok value={x[0].item()} roundtrip_us={dt*1e6:.1f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
