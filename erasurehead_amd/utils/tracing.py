"""Phase timers and an env-gated roctx range API.

The reference only records wall-clock stamps (per-round master time, per-worker arrival,
total).  The engine keeps those and adds per-phase host timers (send, compute launch,
wait-for-k, decode, update) plus roctx ranges visible in ``rocprofv3 --marker-trace``
when ``ERASUREHEAD_TRACE=1`` (or RunConfig.trace).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List

_ENABLED = os.environ.get("ERASUREHEAD_TRACE", "0") not in ("0", "", "false")


def enable(flag: bool = True) -> None:
    """Turn roctx ranges on for the Python engine and (via the environment, read once) the
    native executors in csrc/runtime/engine.cpp."""
    global _ENABLED
    _ENABLED = flag
    if flag:
        os.environ["ERASUREHEAD_TRACE"] = "1"


@contextlib.contextmanager
def range_(name: str):
    if not _ENABLED:
        yield
        return
    try:
        import torch

        torch.cuda.nvtx.range_push(name)  # roctx on ROCm builds
        pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            import torch

            torch.cuda.nvtx.range_pop()


class PhaseTimer:
    """Accumulates host wall time per named phase."""

    def __init__(self):
        self.t: Dict[str, List[float]] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        with range_(name):
            yield
        self.t[name].append(time.perf_counter() - t0)

    def add(self, name: str, dt: float) -> None:
        self.t[name].append(dt)

    def summary(self) -> Dict[str, Dict[str, float]]:
        out = {}
        for k, v in self.t.items():
            if v:
                s = sorted(v)
                out[k] = {"n": len(v), "mean_us": 1e6 * sum(v) / len(v), "p50_us": 1e6 * s[len(s) // 2],
                          "max_us": 1e6 * s[-1]}
        return out
