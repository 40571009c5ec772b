"""erasurehead_amd — MI355X-native straggler-tolerant distributed gradient descent with gradient codes.

Capabilities of Distributed-Deep-Learning/ErasureHead (uncoded, cyclic-MDS, fractional
repetition, approximate gradient coding, ignore-stragglers, partial hybrids; logistic and
least-squares models; GD/AGD) rebuilt on PyTorch-ROCm + gfx950 HIP kernels + RCCL.
"""
import os as _os

__version__ = "0.1.0"

# Hardware queues per process.  HIP maps streams onto at most GPU_MAX_HW_QUEUES in-order hardware
# queues (default 4) and streams beyond that share one.  The master's p2p transports (RCCL /
# loopback, parallel/transport.py CommTransport) keep one receive and one send stream per worker
# rank; a receive blocked on a straggler would otherwise stall another worker's receive queued
# behind it on the same hardware queue, and the master could no longer take the fastest k.  Read
# by the HIP runtime when it initialises, so it is raised here, before anything touches the GPU
# (to at least 16; a larger setting in the environment is kept).
MIN_HW_QUEUES = 16
try:
    _q = int(_os.environ.get("GPU_MAX_HW_QUEUES", "0"))
except ValueError:
    _q = 0
# What the HIP runtime of this process actually uses: the value from before the override when HIP
# was already initialised (torch touched the GPU before this package was imported), else ours.
# parallel/transport.py warns on it and Trainer.rank_report records it.
_HIP_WAS_UP = False
try:
    import sys as _sys

    _t = _sys.modules.get("torch")
    _HIP_WAS_UP = bool(_t is not None and _t.cuda.is_initialized())
except Exception:  # noqa: BLE001 - torch half-imported: treat as not initialised
    _HIP_WAS_UP = False
if _q < MIN_HW_QUEUES and not _HIP_WAS_UP:
    _os.environ["GPU_MAX_HW_QUEUES"] = str(MIN_HW_QUEUES)
HW_QUEUES = (_q or 4) if _HIP_WAS_UP else max(_q, MIN_HW_QUEUES)

from .config import RunConfig  # noqa: E402
