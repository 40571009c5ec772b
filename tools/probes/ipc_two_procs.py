"""Probe: IPC mailbox primitives between two processes on one GPU (or two GPUs).

torchrun --nproc-per-node 2 tools/probes/ipc_two_procs.py
rank 1 puts a 1 MiB payload into rank 0's IpcRegion with put_signal (flag in shared host
memory); rank 0's host polls the flag, checks the payload on the GPU and acknowledges
(host store on even rounds, GPU signal kernel on odd rounds).  Prints the round-trip time.
"""
import os
import sys
import time
import uuid

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from erasurehead_amd._ext import native  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = native(build_if_missing=False)
    n = 131072
    if rank == 0:
        reg = C.IpcRegion(n * 8, dev)
        name = "/eh_probe_" + uuid.uuid4().hex[:12]
        flags = C.ShmFlags(name, 16, True)
        box = [(reg.handle(), name)]
    else:
        box = [None]
    dist.broadcast_object_list(box, 0)
    if rank != 0:
        h, name = box[0]
        reg = C.IpcRegion(h, n * 8, dev)
        flags = C.ShmFlags(name, 16, False)
    view = reg.view("float64", [n], 0)
    counters = torch.zeros(16, dtype=torch.int32, device="cuda")
    dist.barrier()
    R = 300
    bad = 0
    lat = []
    src = torch.zeros((n,), dtype=torch.float64, device="cuda")
    t0 = time.perf_counter()
    for r in range(R):
        if rank == 1:
            src.fill_(float(r))
            torch.cuda.synchronize()
            flags.store(2, time.monotonic_ns())
            C.put_signal([(src, view, flags.dev_addr(0), r + 1)], counters)
            if not flags.wait_ge(1, r + 1, 30.0):
                print("rank1 timeout waiting ack", r, flush=True)
                bad += 1
                break
        else:
            if not flags.wait_ge(0, r + 1, 30.0):
                print("rank0 timeout waiting data", r, flush=True)
                bad += 1
                break
            lat.append((time.monotonic_ns() - flags.load(2)) / 1e3)
            ok = bool(view.eq(float(r)).all().item())
            bad += 0 if ok else 1
            if r % 2 == 0:
                flags.store(1, r + 1)
            else:
                C.signal(flags.dev_addr(1), r + 1, dev)
                torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / R
    print(f"rank {rank} rounds {R} bad {bad} roundtrip_us {dt * 1e6:.1f}", flush=True)
    if lat:
        lat.sort()
        print(f"rank 0 one-way put->flag seen us: p10 {lat[len(lat)//10]:.1f} p50 {lat[len(lat)//2]:.1f} "
              f"p90 {lat[9*len(lat)//10]:.1f}", flush=True)
    dist.barrier()
    flags.close()
    reg.close()
    dist.destroy_process_group()
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
