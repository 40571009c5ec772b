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


class ThreadGroup:
    """In-process rendezvous of ThreadEnv ranks (barriers with a deadline: a rank that fails breaks
    the group, so the others raise instead of waiting forever)."""

    def __init__(self, world: int, timeout: float = 300.0):
        import threading

        self.world = world
        self.timeout = timeout
        self._bar = threading.Barrier(world)
        self.slots: List[Any] = [None] * world

    def wait(self) -> None:
        self._bar.wait(self.timeout)

    def abort(self) -> None:
        self._bar.abort()


@dataclass
class ThreadEnv(DistEnv):
    """Ranks as THREADS of one process sharing one GPU (backend "threads").

    RCCL refuses two processes on one device, so the one-GPU test box cannot run the RCCL transport
    across processes; with every rank a thread of one process, each on its own HIP stream, the
    native pumps run their comm mode over a real RCCL path (parallel/transport.py "rccl-self",
    csrc/runtime/comm.cpp RcclSelfLoop).  Collectives are in-process: broadcast hands every rank the
    SAME object (so the self-loop communicator is shared), the others copy nothing either.
    """
    group: Any = None

    def barrier(self) -> None:
        self.group.wait()

    def broadcast_object(self, obj, src: int = 0):
        g = self.group
        if self.rank == src:
            g.slots[src] = obj
        g.wait()
        out = g.slots[src]
        g.wait()
        return out

    def allreduce_max(self, x: float) -> float:
        g = self.group
        g.slots[self.rank] = float(x)
        g.wait()
        m = max(g.slots)
        g.wait()
        return m

    def gather_objects(self, obj) -> Optional[List[Any]]:
        g = self.group
        g.slots[self.rank] = obj
        g.wait()
        out = list(g.slots) if self.rank == 0 else None
        g.wait()
        return out

    def shutdown(self) -> None:
        pass


def run_thread_ranks(world: int, fn, timeout: float = 300.0) -> List[Any]:
    """Run ``fn(env)`` on ``world`` thread-ranks of this process (cuda:0, one stream per rank);
    returns their results in rank order, or raises the first failure (the group is broken so no
    rank waits forever)."""
    import threading

    group = ThreadGroup(world, timeout)
    out: List[Any] = [None] * world
    errs: List[BaseException] = []

    def body(rank: int) -> None:
        try:
            torch.cuda.set_device(0)
            env = ThreadEnv(rank=rank, world=world, local_rank=rank, device=torch.device("cuda", 0),
                            backend="threads", group=group)
            with torch.cuda.stream(torch.cuda.Stream()):
                out[rank] = fn(env)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)
            group.abort()

    ths = [threading.Thread(target=body, args=(r,), name=f"eh-rank{r}") for r in range(world)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout + 60.0)
    if any(t.is_alive() for t in ths):
        raise TimeoutError("thread ranks did not finish")
    if errs:
        raise errs[0]
    return out


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
