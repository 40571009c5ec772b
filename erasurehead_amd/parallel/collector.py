"""Python facade over the native arrival collector (csrc/runtime/collector.{h,cpp}).

GPU mode: probes are HIP events (torch.cuda.Event) recorded behind an RCCL receive or
behind the local gradient kernel; the poll loop, virtual straggler delays and stop rule
all run in C++ with the GIL released (``wait``/``drain``).
Host mode (CPU tensors, gloo): probes are completed from Python when the gloo ``Work``
reports completion (or immediately for synchronous CPU compute) and the same native
state machine decides arrival order and the stop.
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional, Sequence, Tuple

from .._ext import native
from ..codes.schemes import Arrival


class ArrivalCollector:
    def __init__(self, n_workers: int, group_of: Sequence[int], n_groups: int, gpu: bool):
        C = native()
        self._C = C
        self.c = C.Collector(int(n_workers), [int(g) for g in group_of], int(n_groups))
        self.gpu = gpu
        self._keep: Dict[int, object] = {}  # probe -> event (kept alive until arrival)
        self._host: Dict[int, Tuple[object, int]] = {}  # probe -> (work or None, round)
        self.round = -1

    @staticmethod
    def now() -> float:
        return native().Collector.now()

    def begin_round(self, i: int, t_start: float, rule: int, k: int) -> None:
        self.round = i
        self.c.begin_round(int(i), float(t_start), int(rule), int(k))

    def add_event(self, worker: int, part: int, i: int, event, delay: float) -> int:
        pid = self.c.add_event_probe(int(worker), int(part), int(i), int(event.cuda_event), float(delay))
        self._keep[pid] = event
        return pid

    def add_work(self, worker: int, part: int, i: int, work, delay: float) -> int:
        """Host probe completed when ``work.is_completed()`` (None = already complete now)."""
        pid = self.c.add_host_probe(int(worker), int(part), int(i), float(delay))
        if work is None:
            self.c.mark_seen(pid, self.now())
        else:
            self._host[pid] = (work, i)
        return pid

    def _poll_host(self) -> None:
        if not self._host:
            return
        done = []
        t = self.now()
        for pid, (w, _) in self._host.items():
            if w.is_completed():
                self.c.mark_seen(pid, t)
                done.append(pid)
        for pid in done:
            del self._host[pid]

    def _arrivals(self) -> List[Arrival]:
        out = []
        for a in self.c.arrivals():
            out.append(Arrival(a.worker, a.part, a.t_rel))
            self._keep.pop(a.probe, None)
        return out

    def wait(self, timeout: float) -> Tuple[List[Arrival], bool]:
        """Block until the round's stop rule holds (True) or the timeout elapses (False)."""
        if not self._host and self.gpu:
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
        if not self._host and self.gpu:
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

    def late(self) -> List[Arrival]:
        return [Arrival(a.worker, a.part, a.t_rel) for a in self.c.late_arrivals(self.round)]
