"""Host reference of the IPC message integrity tags (csrc/kernels/integrity.h).

Every tagged put writes, per payload row, a 16-byte tag ``{round + 1: u32, sender rank: u32,
checksum: u64}`` next to the receiver's buffer before it signals the round counter; the receiver
recomputes the checksum over the row it reads.  The checksum of a row of n elements (fp64 or
fp32 bit patterns, zero-extended to 64 bits) is

    sum_j bits_j * (2 j + 1)   mod 2^64

so single corrupted or moved elements and stale rows change it.  This module recomputes it on
the host (tests, diagnostics) and parses tag bytes.  The reference has no equivalent: it
relies on MPI's per-source message ordering (ref src/naive.py:66-79).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

TAG_BYTES = 16


def row_checksum(row: np.ndarray) -> int:
    """Checksum of one payload row (float64 or float32) exactly as the kernels compute it."""
    a = np.ascontiguousarray(row)
    if a.dtype.itemsize == 8:
        bits = a.view(np.uint64)
    elif a.dtype.itemsize == 4:
        bits = a.view(np.uint32).astype(np.uint64)
    else:
        raise ValueError("rows are float64 or float32")
    j = np.arange(bits.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return int(np.sum(bits * (np.uint64(2) * j + np.uint64(1)), dtype=np.uint64))


def parse_tags(raw: bytes) -> List[Tuple[int, int, int]]:
    """(round + 1, rank, checksum) of every 16-byte tag in ``raw``."""
    a = np.frombuffer(raw, dtype=np.uint8)
    if a.size % TAG_BYTES:
        raise ValueError("tag bytes must be a multiple of 16")
    out = []
    for k in range(a.size // TAG_BYTES):
        t = a[k * TAG_BYTES:(k + 1) * TAG_BYTES]
        r1, rank = (int(x) for x in t[:8].view(np.uint32))
        out.append((r1, rank, int(t[8:].view(np.uint64)[0])))
    return out
