"""Python facade over the native arrival collector (csrc/runtime/collector.{h,cpp}).

GPU mode: probes are HIP events (torch.cuda.Event) recorded behind an RCCL receive or
behind the local gradient kernel; the poll loop, virtual straggler delays and stop rule
all run in C++ with the GIL released (``wait``/``drain``).
Host mode (CPU tensors, gloo): gloo's p2p ``Work`` objects only complete inside
``wait()`` (``is_completed()`` never flips), so one waiter thread per source rank waits
on that rank's receives in FIFO order and reports the completion time; local CPU
compute completes immediately.  The same native state machine decides arrival order
and the stop.
"""
from __future__ import annotations

import math
import queue
import threading
import time
from typing import Dict, List, Sequence, Tuple

from .._ext import native
from ..codes.schemes import Arrival


class ArrivalCollector:
    def __init__(self, n_workers: int, group_of: Sequence[int], n_groups: int, gpu: bool, tie_seed: int = -1):
        C = native()
        self._C = C
        self.c = C.Collector(int(n_workers), [int(g) for g in group_of], int(n_groups))
        self.c.set_tie_seed(int(tie_seed))  # simultaneous arrivals: seeded per-round worker permutation
        self.gpu = gpu
        self._keep: Dict[int, object] = {}  # probe -> event (kept alive until arrival)
        self._pending_host = 0
        self._done: "queue.Queue[Tuple[int, float]]" = queue.Queue()
        self._waiters: Dict[int, "queue.Queue"] = {}
        self.round = -1

    def _waiter(self, q: "queue.Queue") -> None:
        while True:
            item = q.get()
            if item is None:
                return
            pid, work = item
            try:
                work.wait()
            finally:
                self._done.put((pid, self.now()))

    def close(self) -> None:
        for q in self._waiters.values():
            q.put(None)
        self._waiters.clear()

    @staticmethod
    def now() -> float:
        return native().Collector.now()

    def set_shards(self, n_shards) -> None:
        """{(worker, part): n} — messages computed as n partition shards (arrive with the last one)."""
        for (w, p), n in n_shards.items():
            if n != 1:
                self.c.set_shards(int(w), int(p), int(n))

    def set_skip_stale(self, on: bool) -> None:
        """Drain "lazy": a worker still busy with an earlier round when the next one begins skips it
        (csrc/runtime/collector.h, stale-round skipping); off = lag carries, every round is delivered."""
        self.c.set_skip_stale(bool(on))

    @property
    def skipped(self) -> int:
        """Virtual probes skipped as stale so far."""
        return int(self.c.skipped)

    @property
    def stale_arrivals(self) -> int:
        """Messages that arrived after their round ended (never decoded)."""
        return int(self.c.stale_arrivals)

    def begin_round(self, i: int, t_start: float, rule: int, k: int) -> None:
        self.round = i
        self.c.begin_round(int(i), float(t_start), int(rule), int(k))

    def add_event(self, worker: int, part: int, i: int, event, delay: float, physical: bool = False) -> int:
        """physical: a really late rank's message; its completion time is its arrival (no carry-over)."""
        pid = self.c.add_event_probe(int(worker), int(part), int(i), int(event.cuda_event), float(delay), bool(physical))
        self._keep[pid] = event
        return pid

    def add_flag(self, worker: int, part: int, i: int, addr: int, value: int, delay: float,
                 physical: bool = False) -> int:
        """IPC mailbox probe: arrived when the shared-host counter at ``addr`` reaches ``value``."""
        return self.c.add_flag_probe(int(worker), int(part), int(i), int(addr), int(value), float(delay), bool(physical))

    def add_work(self, worker: int, part: int, i: int, work, delay: float, src: int = 0,
                 t_seen: float = None, physical: bool = False) -> int:
        """Host probe completed when ``work`` finishes (None = already complete at ``t_seen``, default now)."""
        pid = self.c.add_host_probe(int(worker), int(part), int(i), float(delay), bool(physical))
        if work is None:
            self.c.mark_seen(pid, self.now() if t_seen is None else float(t_seen))
        else:
            q = self._waiters.get(src)
            if q is None:
                q = self._waiters[src] = queue.Queue()
                threading.Thread(target=self._waiter, args=(q,), daemon=True).start()
            self._pending_host += 1
            q.put((pid, work))
        return pid

    def _poll_host(self) -> None:
        while True:
            try:
                pid, t = self._done.get_nowait()
            except queue.Empty:
                return
            self._pending_host -= 1
            self.c.mark_seen(pid, t)

    def _arrivals(self) -> List[Arrival]:
        out = []
        for a in self.c.arrivals():
            out.append(Arrival(a.worker, a.part, a.t_rel))
            self._keep.pop(a.probe, None)
        return out

    def wait(self, timeout: float) -> Tuple[List[Arrival], bool]:
        """Block until the round's stop rule holds (True) or the timeout elapses (False)."""
        if self._pending_host == 0 and self.gpu:
            ok = self.c.wait(float(timeout))
            return self._arrivals(), ok
        t0 = time.perf_counter()
        while True:
            self._poll_host()
            if self.c.step():
                return self._arrivals(), True
            if time.perf_counter() - t0 > timeout:
                return self._arrivals(), False
            time.sleep(2e-5 if self.gpu else 1e-4)

    def drain(self, i: int, timeout: float = math.inf) -> bool:
        """Wait until every probe of rounds <= i arrived (the reference's Waitall)."""
        if self._pending_host == 0 and self.gpu:
            ok = self.c.drain(int(i), float(min(timeout, 1e9)))
        else:
            t0 = time.perf_counter()
            ok = True
            while self.c.pending_upto(int(i)) > 0:
                self._poll_host()
                self.c.step()
                if time.perf_counter() - t0 > timeout:
                    ok = False
                    break
                time.sleep(1e-4)
        if self.c.pending() == 0:
            self._keep.clear()
        return ok

    def wait_seen(self, i: int, timeout: float = math.inf) -> bool:
        """Wait until the data of every message of rounds <= i has landed (mailbox slot reuse)."""
        if self._pending_host == 0 and self.gpu:
            return self.c.wait_seen(int(i), float(min(timeout, 1e9)))
        t0 = time.perf_counter()
        while True:
            self._poll_host()
            if self.c.wait_seen(int(i), 0.0):
                return True
            if time.perf_counter() - t0 > timeout:
                return False
            time.sleep(1e-4)

    def late(self) -> List[Arrival]:
        return [Arrival(a.worker, a.part, a.t_rel) for a in self.c.late_arrivals(self.round)]
