"""Master decode-combine + GD/AGD update (K5/K7/K8; csrc/kernels/update.hip).

``combine_update`` computes g = sum_m coef_m * msg_m and applies the reference update
(ref src/naive.py:112-122) to the fp64 master state in one launch, also writing the
betaset history row and the worker-precision copy of the new beta.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._ext import native


def combine_update(msgs: Sequence[torch.Tensor], coefs: Sequence[float], beta: torch.Tensor, u: torch.Tensor,
                   d: int, decay: float, gm: float, l2: float, theta: float, rule: int,
                   hist: Optional[torch.Tensor] = None, beta_w: Optional[torch.Tensor] = None,
                   g_out: Optional[torch.Tensor] = None) -> None:
    if beta.is_cuda:
        C = native()
        if len(msgs) > C.MAX_MSGS:
            raise ValueError(f"at most {C.MAX_MSGS} messages per combine")
        C.combine_update(list(msgs), [float(c) for c in coefs], beta, u, hist, beta_w, g_out, int(d),
                         float(decay), float(gm), float(l2), float(theta), int(rule))
        return
    g = torch.zeros(d, dtype=torch.float64)
    for m, c in zip(msgs, coefs):
        g += float(c) * m[:d].double()
    b = beta[:d]
    if rule == 0:
        nb = decay * b - gm * g
    else:
        yt = (1.0 - theta) * b + theta * u[:d]
        nb = yt - gm * g - l2 * b
        u[:d] = b + (nb - b) * (1.0 / theta)
    beta[:d] = nb
    if hist is not None:
        hist[:d] = nb
    if beta_w is not None:
        beta_w.zero_()
        beta_w[:d] = nb.to(beta_w.dtype)
    if g_out is not None:
        g_out[:d] = g
