"""Compute-precision modes of the worker path.

  fp64  X fp64, accumulate fp64 — bit-compatible math with the reference's NumPy float64
  fp32  X fp32, accumulate fp32
  bf16  X stored bf16 (half the HBM bytes of fp32), accumulate fp32

beta, u and the betaset history are always fp64 on the master (update kernel), the
per-round worker copy of beta and the gradient messages use the accumulator type.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class Precision:
    name: str
    code: int  # kernel dtype code
    storage: torch.dtype
    acc: torch.dtype
    vec: int  # elements per 16-byte vector load

    @property
    def storage_bytes(self) -> int:
        return 16 // self.vec

    def ld(self, d: int) -> int:
        """Leading dimension: d rounded up to the 16-byte vector width."""
        return ((d + self.vec - 1) // self.vec) * self.vec


PRECISIONS = {
    "fp64": Precision("fp64", 0, torch.float64, torch.float64, 2),
    "fp32": Precision("fp32", 1, torch.float32, torch.float32, 4),
    "bf16": Precision("bf16", 2, torch.bfloat16, torch.float32, 8),
}


def get_precision(name: str) -> Precision:
    try:
        return PRECISIONS[name]
    except KeyError:
        raise ValueError(f"unknown precision {name!r}; choose from {sorted(PRECISIONS)}") from None
