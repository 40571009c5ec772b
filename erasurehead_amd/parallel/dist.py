"""Process topology: one process per GPU, torch.distributed over RCCL (xGMI) or gloo (CPU).

The reference launches W+1 MPI ranks on W+1 hosts (rank 0 = master / parameter server,
ref main.py:16-18, README.md:99-103).  Here the *logical* workers are decoupled from
processes: ``torchrun --nproc-per-node N`` starts N ranks (one per MI355X), logical
workers are placed on ranks (placement.py) and rank 0 also runs the master on its own
HIP stream.  Without torchrun everything runs in one process (N = 1).

Backends: device tensors move over the default group — "nccl" (= RCCL on ROCm) when the
ranks own GPUs, p2p only (per-peer communicators, never a collective on the hot path);
a separate gloo group carries host control traffic (barriers, the cyclic B matrix,
timing reductions).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    ctrl: Any = None  # gloo group for host control traffic
    owns_pg: bool = False

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    @property
    def gpu(self) -> bool:
        return self.device.type == "cuda"

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.ctrl)

    def broadcast_object(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.ctrl)
        return box[0]

    def allreduce_max(self, x: float) -> float:
        if self.world == 1:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        return float(t.item())

    def gather_objects(self, obj) -> Optional[List[Any]]:
        if self.world == 1:
            return [obj]
        out = [None] * self.world if self.rank == 0 else None
        dist.gather_object(obj, out, dst=0, group=self.ctrl)
        return out

    def shutdown(self) -> None:
        if self.owns_pg and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass


def init_distributed(device: str = "auto", timeout_min: float = 60.0) -> DistEnv:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    want_gpu = device in ("auto", "cuda") and torch.cuda.is_available()
    if device == "cuda" and not torch.cuda.is_available():
        raise RuntimeError("device=cuda requested but no GPU is visible")
    if want_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        dev = torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    if world == 1:
        return DistEnv(rank=0, world=1, local_rank=0, device=dev, backend="none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    to = datetime.timedelta(minutes=timeout_min)
    owns = False
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))  # ranks on this node (torchrun)
    shared_gpu = want_gpu and local_world > torch.cuda.device_count()  # several ranks per GPU: RCCL impossible
    if not dist.is_initialized():
        backend = "nccl" if want_gpu and not shared_gpu else "gloo"
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=to, **kw)
        owns = True
    backend = dist.get_backend()
    ctrl = dist.new_group(backend="gloo", timeout=to) if backend != "gloo" else dist.group.WORLD
    if want_gpu and backend == "gloo":
        os.environ.setdefault("ERASUREHEAD_TRANSPORT", "ipc")  # device data can only move over IPC
    return DistEnv(rank=rank, world=world, local_rank=local, device=dev, backend=backend, ctrl=ctrl, owns_pg=owns)
