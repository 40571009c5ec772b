"""Cyclic MDS gradient code (Tandon et al.) — encoding matrix and online decode.

Reference behaviour:
  * ``getB(n_workers, n_stragglers)``  ref src/util.py:64-83
      1. H ~ N(0,1) of shape s x (W-1); append a last column so every row of H sums to 0.
      2. Row i of B has support {i, ..., i+s} mod W with B[i, i] = 1.
      3. The other s entries solve H[:, S_i \\ i] v = -H[:, i].
    Any W - s rows of B then span the all-ones vector.
  * online decode  ``A_row[F] = lstsq(B[F,:].T, ones)``; ``g = A_row . msgBuffers``
      ref src/coded.py:147-149, src/partial_coded.py:192-194
  * ``getA`` / ``calculate_indexA`` (all C(W, s) patterns, unused in the reference,
    ref src/util.py:85-134) are revived here as :class:`DecodeCache` keyed by the
    straggler bitmask, so the fp64 solve runs once per pattern instead of per round.

B is rank-deficient by construction (cond ~ 1e17), so every solve is done on the host
in float64; only the resulting W coefficients travel to the GPU.
"""
from __future__ import annotations

import itertools
from typing import Dict, Iterable, Optional, Sequence

import numpy as np


def cyclic_support(n_workers: int, n_stragglers: int) -> np.ndarray:
    """Ssets[i] = (i, i+1, ..., i+s) mod W  (ref src/util.py:69-73)."""
    base = np.arange(n_workers)[:, None] + np.arange(n_stragglers + 1)[None, :]
    return base % n_workers


def make_cyclic_B(n_workers: int, n_stragglers: int, rng: Optional[np.random.RandomState] = None) -> np.ndarray:
    """Cyclic-MDS encoding matrix with the reference's construction (ref src/util.py:64-83)."""
    W, s = int(n_workers), int(n_stragglers)
    if not 0 <= s < W:
        raise ValueError(f"need 0 <= n_stragglers < n_workers, got s={s}, W={W}")
    rng = rng if rng is not None else np.random.mtrand._rand
    B = np.zeros((W, W))
    if s == 0:
        np.fill_diagonal(B, 1.0)
        return B
    Htemp = rng.normal(0, 1, [s, W - 1])
    H = np.hstack([Htemp, -Htemp.sum(axis=1, keepdims=True)])
    S = cyclic_support(W, s)
    for i in range(W):
        B[i, S[i, 0]] = 1.0
        v = -np.linalg.solve(H[:, S[i, 1:]], H[:, S[i, 0]])
        B[i, S[i, 1:]] = v
    return B


def decode_vector(B: np.ndarray, completed: Sequence[int]) -> np.ndarray:
    """a with a[F] = lstsq(B[F,:]^T, 1), zeros elsewhere (ref src/coded.py:147-148)."""
    W = B.shape[0]
    F = np.asarray(sorted(int(w) for w in completed), dtype=np.int64)
    a = np.zeros(W)
    if F.size == 0:
        return a
    sol = np.linalg.lstsq(B[F, :].T, np.ones(B.shape[1]), rcond=-1)[0]
    a[F] = sol
    return a


class DecodeCache:
    """Decode vectors keyed by the completion bitmask (the reference's getA, revived)."""

    def __init__(self, B: np.ndarray):
        self.B = np.asarray(B, dtype=np.float64)
        self._cache: Dict[int, np.ndarray] = {}

    def __call__(self, completed: Iterable[int]) -> np.ndarray:
        mask = 0
        for w in completed:
            mask |= 1 << int(w)
        a = self._cache.get(mask)
        if a is None:
            a = decode_vector(self.B, [w for w in range(self.B.shape[0]) if mask >> w & 1])
            self._cache[mask] = a
        return a

    def precompute_all(self, n_stragglers: int) -> np.ndarray:
        """All C(W, s) straggler patterns, rows ordered like the reference's getA."""
        W = self.B.shape[0]
        rows = []
        for pos in itertools.combinations(range(W), n_stragglers):
            done = [w for w in range(W) if w not in pos]
            rows.append(self(done))
        return np.array(rows)


def decode_error(B: np.ndarray, completed: Sequence[int]) -> float:
    """max |a . B - 1| for a completion set (the exact-recovery property)."""
    a = decode_vector(B, completed)
    return float(np.max(np.abs(a @ B - 1.0)))


def pattern_index(completed_mask: Sequence[bool]) -> int:
    """Combinatorial index of a completion pattern (ref src/util.py:123-134 calculate_indexA)."""
    from math import comb

    l = len(completed_mask)
    ctr = 0
    ind = 0
    for j in range(l - 1, -1, -1):
        if completed_mask[j]:
            ctr += 1
            ind += comb(l - 1 - j, ctr)
    return int(ind)
