"""Worker-gradient execution plans (device side of K1-K4/K13).

A *plan* is built once per run for all logical workers hosted on one GPU: every
message (worker, part) is a list of segments (partition, label coefficient).  Each
round the plan is executed with one launch set:

  dense  -> ``grad_dense`` (fused single pass over X, slab reduction)   csrc/kernels/grad_dense.hip
            ``grad_dense_wide`` (a workgroup per row) when d > 2048 fp64       (same file)
            ``grad_dense_twopass`` beyond 8192 fp64 / 16384 fp32 columns
  sparse -> ``grad_sparse`` (ELL / CSR row pass + deterministic CSC tiles)  csrc/kernels/grad_sparse.hip

On CPU tensors the same plans run a float64/float32 torch implementation of the
identical math (the test path and the gloo multi-process path); on GPU tensors the
native kernels are mandatory (:func:`erasurehead_amd._ext.native` raises if absent).
"""
from __future__ import annotations

import collections
import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .._ext import native
from ..models.losses import LOGISTIC
from .precision import Precision

_SEG = struct.Struct("<QQdq")  # csrc Segment {const void* X; const void* y; double coef; long long nrows}
MAX_CPL = 32
DEFAULT_TASKS = 2048
REPLICA_TASKS = 4096
MAX_BUNDLE = 8  # replica task slots (waves) per workgroup of grad_dense_staged
MIN_ROWS_PER_TASK = 32
SLAB_SPLITS = 16  # csrc/kernels/grad_dense.hip kSplits
N_CUS = 256  # MI355X compute units (8 XCDs x 32)
# A rank streams in the "long-stream" regime when each CU reads at least this many distinct rows per
# round: there the gradient is HBM-bound with fewer, longer bundles (their per-bundle beta load,
# fold and slab write amortise over more rows), below it the grid must fill every wave slot.  The
# measured crossover lies between 500k and 1e6 rows of 1000 columns on 256 CUs (N = 2 vs N = 1 of
# the headline, profiles/round2/s2_multi, round2/s2_epi); 2900 rows per CU (~742k rows) sits in between.
LONG_STREAM_ROWS_PER_CU = 2900

KIND_IDS = {"fused": 0, "multi": 1, "staged": 2, "mfma": 3, "wide": 4, "twopass": -1}


@dataclass(frozen=True)
class KernelChoice:
    """The dense-gradient kernel a plan launches (csrc/kernels/grad_dense.h KernelChoice).

    kind     fused    a wave per row, ``rows`` rows in flight (2: the interleaved pair kernel),
                      beta in registers or LDS (``beta_lds``); distinct rows, or replicas with the
                      replica-interleaved dispatch (``interleave``)
             multi    one-wave replica bundles: each row loaded once into registers, every one of the
                      ``replicas`` co-located messages computed from it (``fold``: 4 bundles of one
                      partition per workgroup folded through LDS; ``lane_epi``: reduce-scatter
                      epilogue with one lane per replica; ``pair``: two rows per reduce-scatter,
                      narrow rows)
             staged   replica bundles streamed through an LDS ring, a wave per replica (``pair``: two
                      rows per step share one reduction; ``wpr`` waves per replica)
             mfma     bf16 replica bundles on the matrix cores
             wide     a workgroup per row (2048 < d <= 8192 fp64 / 16384 fp32); ``replicas`` > 1: replica
                      bundles of 256-thread rows (one row load, every replica's dot product and gradient)
             twopass  wider rows / bf16 beyond the one-pass kernels: two passes over X
    bundle_rows  rows per bundle task (bundle kinds)
    fill         folded one-wave bundles: split every partition evenly so the plan has exactly
                 ``fill`` workgroups (fill_splits; 0 = fixed ``bundle_rows``-row bundles)
    """
    kind: str
    replicas: int = 1
    bundle_rows: int = 0
    fold: bool = False
    lane_epi: bool = False
    pair: bool = False
    wpr: int = 0
    rows: int = 2
    beta_lds: bool = False
    interleave: bool = False
    fill: int = 0

    @property
    def bundled(self) -> bool:
        return self.kind in ("multi", "staged", "mfma") or (self.kind == "wide" and self.replicas > 1)

    def native(self):
        """The C++ struct (csrc/kernels/grad_dense.h) passed to the launchers."""
        return native().KernelChoice(kind=KIND_IDS[self.kind], replicas=self.replicas, fold=int(self.fold),
                                     lane_epi=int(self.lane_epi), pair=int(self.pair), wpr=self.wpr,
                                     rows=self.rows, beta_lds=int(self.beta_lds))

    def label(self) -> str:
        name = {"fused": "fused", "multi": "one-wave bundles", "staged": "LDS-staged bundles", "mfma": "MFMA bundles",
                "wide": "wide rows", "twopass": "two-pass"}[self.kind]
        opts = [o for o, on in (("folded", self.fold), ("lane epilogue", self.lane_epi), ("pair", self.pair),
                                ("interleaved", self.interleave)) if on]
        out = name + (f" ({', '.join(opts)})" if opts else "")
        if self.bundled and self.fill:
            out += f", R={self.replicas}, partitions split evenly over {self.fill} workgroups"
        elif self.bundled:
            out += f", R={self.replicas}, {self.bundle_rows}-row bundles"
        elif self.kind == "fused":
            out += f", {self.rows} rows in flight" + (", beta in LDS" if self.beta_lds else "")
        return out


def multi_slots(distinct_rows: int, fp32: bool = False, n_cus: int = N_CUS, cpl: int = 16) -> int:
    """Resident one-wave bundles of grad_dense_multi on the chip (4 per folded workgroup).  ``fp32``
    selects the 12 / 8-per-CU rule measured for fp32 in round 3; since round 5 it sizes bf16 distinct
    rows and fp32 rows narrower than 16 columns per lane only, while fp32 rows of 16 columns per lane
    take the fp64 rule (choose_kernel; profiles/round5/shapes/fp32_*)."""
    long_stream = distinct_rows >= LONG_STREAM_ROWS_PER_CU * n_cus
    # fp64: one workgroup (4 bundles) per CU.  Since a step waits for its own row only (the label
    # load behind the row), 4 waves with the next row in flight keep a CU's share of HBM busy, and
    # half as many slab rows, betas and folds are paid (profiles/round3/rows_prefetch: 1024 / 512 /
    # 256 / 128-row bundles at 1e6 / 500k / 250k / 125k rows: 1.142 / 0.587 / 0.304 / 0.160 ms vs
    # 1.185-1.218 / 0.611 / 0.320 / 0.171 at two workgroups per CU)
    per_cu = (12 if not long_stream else 8) if fp32 else 4
    per_cu *= max(1, 16 // cpl)
    return per_cu * n_cus


def multi_bundle_rows(distinct_rows: int, fp32: bool = False, n_cus: int = N_CUS, cpl: int = 16,
                      part_rows: Optional[Sequence[int]] = None) -> int:
    """Rows per one-wave bundle of grad_dense_multi: the shortest multiple of 32 rows whose folded
    workgroups (4 bundles of one partition each, the last one per partition padded) all fit the
    chip's resident slots at once, so every bundle starts in the first dispatch round and no CU is
    left with a second, partial round of equal-length bundles (the tail that costs a whole bundle).

    Resident one-wave bundles per CU: 8 fp64 (244 VGPRs, 2 waves per SIMD), 12 fp32 (155 VGPRs,
    3 per SIMD); narrower rows (cpl < 16 columns per lane) hold proportionally fewer registers, so
    16 / cpl times as many fit.  In the long-stream regime fp32 fills 8 per CU too (1e6 rows, lane
    epilogue: 512-row bundles 0.631 ms vs 352 rows 0.693 / 256 rows 0.644 with the wave epilogue;
    profiles/round3/choices_nt/agc.jsonl).  part_rows: row counts of the distinct partitions (default: the
    rows split evenly over 8).  With the non-temporal X stream (common.h kStreamAux) every slot
    filled once wins at every rank shape (profiles/round3/nt_rows): fp64 1e6 / 500k / 250k / 125k
    distinct rows -> 512 / 256 / 128 / 64-row bundles, 1.195 / 0.600 / 0.312 / 0.169 ms (768 rows,
    the default before nt: 1.26 ms; 384: 1.42 = a second partial round); fp32 -> 352 / 192 / 96 /
    64 rows (192: 0.333 vs 256: 0.341-0.350 ms at 500k; 96: 0.177 vs 128: 0.186 at 250k)."""
    slots = multi_slots(distinct_rows, fp32, n_cus, cpl)
    parts = [int(r) for r in part_rows if r > 0] if part_rows else [distinct_rows / 8.0] * 8
    per = distinct_rows / slots
    # small problems: bundles down to 8 rows (a wave with one row ahead streams ~1.4 us per row, so a
    # 32-row bundle alone is ~45 us: 4000 x 1000 fp64 rows over 2 ranks took 46 us per gradient)
    # granularity: 128 rows for long bundles (fp64 1e6 rows: 1024-row bundles 1.198 ms vs 992-row 1.214,
    # the same box, profiles/round3/rows_prefetch/rows5_fp64.jsonl: one padded workgroup less per
    # partition), 32 for mid-size ones, 8 for small problems
    gran = 128 if per > 128 else 32 if per > 16 else 8
    base = max(8, gran * int(np.ceil(per / gran)))

    def fits(rows: int) -> bool:
        return sum(4 * int(np.ceil(np.ceil(p / rows) / 4)) for p in parts) <= slots

    rows = base
    while not fits(rows) and rows < max(parts):
        rows += gran
    return rows if fits(rows) else base  # more partitions than slots: short bundles keep the tail short


def fill_splits(part_rows: Dict[int, int], wgs: int, per_wg: int = 4) -> Optional[Dict[int, List[int]]]:
    """Row boundaries of the bundles of every partition so the folded plan has exactly ``wgs``
    workgroups of ``per_wg`` bundles (one partition per workgroup): workgroups are apportioned to
    the partitions by row count (largest remainder, at least one each) and each partition is cut into
    per_wg * (its workgroups) bundles whose lengths differ by at most one row.  Fixed-length bundles
    leave CUs idle whenever the rows do not divide evenly (125k rows in 128-row bundles: 245
    workgroups on 256 CUs, 1e6 rows in 1024-row bundles: 245 too).  None when there are more
    partitions than workgroups."""
    parts = sorted(p for p, n in part_rows.items() if n > 0)
    total = sum(part_rows[p] for p in parts)
    if not parts or len(parts) > wgs:
        return None
    quota = {p: part_rows[p] * wgs / total for p in parts}
    w = {p: max(1, int(quota[p])) for p in parts}
    while sum(w.values()) < wgs:
        p = max(parts, key=lambda q: (quota[q] - w[q], -q))
        w[p] += 1
    while sum(w.values()) > wgs:
        p = max((q for q in parts if w[q] > 1), key=lambda q: (w[q] - quota[q], q))
        w[p] -= 1
    out = {}
    for p in parts:
        n = part_rows[p]
        k = min(per_wg * w[p], n)
        out[p] = [(n * j) // k for j in range(k + 1)]
    return out


def pair_bundle_rows(distinct_rows: int, n_cus: int = N_CUS, fp32: bool = False, cpl: int = 8) -> int:
    """Rows per narrow-row (cpl <= 8) one-wave bundle with the pair-row epilogue: about 16 bundles
    (4 folded workgroups) per CU, 64 for fp32 rows of <= 4 columns per lane (1 KB rows: far fewer
    registers, so more waves per SIMD), the power of two nearest to that, 8..512 rows.  Measured
    (profiles/round3/choices/choices_pair_rows.jsonl, round3/choices_nt/narrow*.jsonl): d = 256
    fp64 1e6 rows 256-row bundles 5.3 TB/s (128: 5.3, 512: 4.7), 1e5 rows 32-row 4.1; fp32 d = 256
    1e6 rows 64-row 5.05 (128: 5.1, 256: 4.5), 1e5 8 / 16 / 32 rows equal; fp32 d = 512 1e6 rows
    256-row 5.9 (64: 5.2)."""
    per = max(1.0, distinct_rows / ((64 if fp32 and cpl <= 4 else 16) * n_cus))
    return int(min(512, max(8 if fp32 and cpl <= 4 else 32, 2 ** round(np.log2(per)))))


def mfma_bundle_rows(distinct_rows: int, n_cus: int = N_CUS, part_rows: Optional[Sequence[int]] = None) -> int:
    """Rows per bf16 MFMA bundle: one 8-wave workgroup per CU (150 KB of LDS); the shortest power of two
    from 256 rows whose bundles (one per workgroup, per partition) all start in the first dispatch
    round.  Measured with the nt stream (profiles/round3/nt_rows/bf16.jsonl), rank gradient ms by
    bundle rows: 500k distinct rows 2048: 0.200 (1024: 0.208, 4096: 0.302 = a second round);
    250k 1024: 0.097 (512: 0.112, 2048: 0.159); 125k 512: 0.054 (256: 0.062, 1024: 0.086); 1e6 rows
    4096: 0.375 = 2048: 0.378."""
    parts = [int(r) for r in part_rows if r > 0] if part_rows else [distinct_rows / 8.0] * 8
    rows = 256
    while rows < 8192 and sum(int(np.ceil(p / rows)) for p in parts) > n_cus:
        rows *= 2
    return rows


def staged_bundle_rows(distinct_rows: int, n_cus: int = N_CUS, fp32: bool = False, cpl: int = 16) -> int:
    """Rows per LDS-staged bundle.  Long streams: 512, 384 for fp32 rows of 32 columns per lane (4
    replicas at d = 1000 fp32: 496-512 rows 0.78-0.80 ms vs 384 0.80-0.84); short streams: 256 for
    fp64 rows of 32 columns per lane (d = 1025..2048, 16 KB rows), else 128.  Measured with the nt stream, pair form
    (profiles/round3/choices_nt/staged.jsonl, d = 2048, 3 replicas): fp64 1e6 rows 512: 2.676 ms
    (496: 2.624, 1024: 2.629; the old non-pair default 2.751), fp32 1e6 384: 1.377 (512: 1.485),
    fp64 1e5 256: 0.326 (128: 0.334-0.376); d = 1000 ranks (round 2, profiles/round2/s1_shapes):
    128 at N = 8 (0.238 vs 0.415 ms at 512)."""
    if distinct_rows >= LONG_STREAM_ROWS_PER_CU * n_cus:
        # fp32 rows of 32 columns per lane (d = 2048): 1024 rows 1.223 ms vs 384 1.402 with the clock
        # warmed before every candidate (profiles/round4/r4i/choices.jsonl; the round-3 sweep that
        # picked 384 timed the first candidates on the clock ramp)
        return 1024 if fp32 and cpl >= 32 else 512
    return 256 if cpl >= 32 and not fp32 else 128  # 16 KB rows (fp64 d > 1024); fp32 2048 at 1e5: 128 rows 0.169 vs 256 0.194 ms


def choose_kernel(prec_code: int, ld: int, cpl: Optional[int], max_rep: int, distinct_rows: int,
                  n_cus: int = N_CUS, part_rows: Optional[Sequence[int]] = None) -> KernelChoice:
    """The measured default kernel of a plan (a pure function; tests/test_plan_tables.py pins the table).

    prec_code: 0 fp64, 1 fp32, 2 bf16 storage.  max_rep: most co-located messages reading one
    partition (1 = distinct rows only).  distinct_rows: rows of the distinct partitions per round.
    Measured choices (docs/PERF_NOTES.md):
      * distinct rows (naive, message-placed ranks): one-wave bundles of one replica at 16 columns per
        lane (profiles/round3/choices_nt/naive.jsonl: fp64 1e6 rows 1.160 vs 1.197-1.213 ms fused,
        fp32 0.581 vs 0.639, fp64 375k rows 0.447-0.456 vs 0.491; bf16, six rows in flight per wave:
        0.302 vs 0.367, profiles/round5/bf16); otherwise the fused kernel, fp64 the interleaved pair
        kernel, fp32 4 rows, bf16 1 row;
      * replicas, 3 per bundle, narrow rows (<= 8 columns per lane, d <= 512 fp64 / 1024 fp32):
        one-wave bundles with two rows per reduce-scatter (d = 256: 5.2 vs 2.3 TB/s before);
      * replicas, fp64 / fp32, 2 or 3 per bundle (AGC / cyclic s = 2, FRC s = 1): one-wave bundles,
        folded, lane epilogue (with the nt stream, profiles/round3/choices_nt: AGC fp64 1e6 rows
        1.165 vs 1.199-1.217 ms wave-uniform; FRC s = 1 fp64 1.157 vs 1.315 ms LDS-staged, fp32
        0.615 vs 0.666, 250k rows 0.303 vs 0.370);
      * replicas otherwise (R > 3, or rows of 32 columns per lane): LDS-staged bundles, pair form
        (two rows per reduction; with the nt stream it wins everywhere: d = 2048 fp64 2.676 vs 2.751
        ms, 4 replicas at d = 1000 fp64 1.532-1.542 vs 1.668; one-wave bundles of 4 replicas need
        276 registers, 1 wave per SIMD, and measured 1.76 ms: profiles/round3/choices_nt/frc4.jsonl);
      * bf16 replicas: MFMA bundles (d <= 1024, d % 8 == 0; one-wave bundles of 3 bf16 replicas are
        VALU-bound: 0.367 vs 0.321 ms, profiles/round5/bf16/choices_agc.jsonl), else the fused kernel
        interleaved;
      * 2048 < d (fp64, 4096 fp32): the wide kernel; fp64 replicas at 1024 < d <= 2048 too (its half-width
        instance); beyond 8192 / 16384 or cpl unknown: two passes.
    """
    if cpl is None:
        return KernelChoice("twopass")
    shared = max_rep > 1
    if cpl >= 256:
        if shared and cpl == 256 and max_rep <= 3:
            return KernelChoice("wide", replicas=max_rep,
                                bundle_rows=wide_bundle_rows(distinct_rows, n_cus, part_rows,
                                                             wide_slots_per_cu(prec_code, ld, max_rep)))
        return KernelChoice("wide", interleave=shared)
    if not shared:
        if 8 < cpl <= 16:  # distinct rows of 16 columns per lane: bundles of one
            # (bf16: six rows in flight per wave, grad_dense.hip kMultiDepth; 1e6 x 1000 rows 0.302 ms vs
            # 0.367 on the fused kernel, profiles/round5/bf16/choices_naive.jsonl; sized with the 12 / 8 per CU
            # rule: 1024-row bundles 0.350.  fp32 sized like fp64: 250k rows 152.2 us with 256-row bundles
            # vs 161.3 with 96, 1e6 rows 577.0 vs 579.4, profiles/round5/shapes/fp32_naive_choices.jsonl)
            return KernelChoice("multi", replicas=1,
                                bundle_rows=multi_bundle_rows(distinct_rows, prec_code == 2, n_cus, cpl, part_rows),
                                fold=True)
        return KernelChoice("fused", rows={0: 2, 1: 4, 2: 1}[prec_code])
    long_stream = distinct_rows >= LONG_STREAM_ROWS_PER_CU * n_cus
    if prec_code == 2:
        if ld <= 1024 and ld % 8 == 0 and max_rep <= 16:
            return KernelChoice("mfma", replicas=min(max_rep, MAX_BUNDLE),
                                bundle_rows=mfma_bundle_rows(distinct_rows, n_cus, part_rows))
        return KernelChoice("fused", rows=1, interleave=True)
    if cpl <= 8 and max_rep == 3:  # narrow rows: two rows per reduce-scatter
        return KernelChoice("multi", replicas=3, bundle_rows=pair_bundle_rows(distinct_rows, n_cus, prec_code == 1, cpl),
                            fold=True,
                            pair=True)
    if cpl == 32 and max_rep <= 3 and (prec_code == 0 or (prec_code == 1 and not long_stream)):
        # (fp32 d = 2048 short streams: the quarter-width instance, 1e5 rows 0.152 vs 0.158 ms staged,
        # profiles/round4/r4o/choices.jsonl; long fp32 streams keep the staged bundles)
        # fp64 rows of 32 columns per lane (1024 < d <= 2048): 256-thread wide-row bundles (the
        # half-width instance) over the LDS-staged pair form: d = 2048 1e6 rows 2.466 vs 2.719 ms, 1e5
        # rows 0.268 vs 0.335 (profiles/round4/r4i/choices.jsonl)
        return KernelChoice("wide", replicas=max_rep,
                            bundle_rows=wide_bundle_rows(distinct_rows, n_cus, part_rows,
                                                         wide_slots_per_cu(prec_code, ld, max_rep)))
    if cpl <= 16 and max_rep in (2, 3):
        # fp32 rows of 16 columns per lane size their replica bundles like fp64 (one folded workgroup per
        # CU): AGC R = 3 at the 1 / 2 / 4 / 8-GPU rank shapes 586.7 / 299.0 / 155.5 / 86.3 us vs 587.6 /
        # 303.4 / 170.6 / 87.4 with the 12-per-CU fp32 sizing (profiles/round5/shapes/fp32_rows_*.jsonl)
        return KernelChoice("multi", replicas=max_rep,
                            bundle_rows=multi_bundle_rows(distinct_rows, prec_code == 1 and cpl < 16, n_cus, cpl,
                                                          part_rows),
                            fold=True, lane_epi=True)
    # more replicas than a workgroup's task slots: bundles of MAX_BUNDLE (and the remainder, padded)
    return KernelChoice("staged", replicas=min(max_rep, MAX_BUNDLE),
                        bundle_rows=staged_bundle_rows(distinct_rows, n_cus, prec_code == 1, cpl),
                        pair=True, wpr=0 if long_stream else 1)


def wide_slots_per_cu(prec_code: int, ld: int, replicas: int) -> int:
    """Resident wide-row bundles per CU (grad_dense.hip launch_wide): rows that fit half of the
    kernel's vectors at 256 threads (fp32 d <= 4096, bf16 <= 4096) take the NV / 2 instance, two or
    more per CU (fp32 d <= 2048: the NV / 4 instance, counted as four); full-width replica rows (fp64
    d > 2048, fp32 > 4096) run 512-thread workgroups of about 150 VGPRs, one per CU."""
    vec = {0: 2, 1: 4, 2: 8}[prec_code]
    half = 256 * (WIDE_EPT[vec] // 2) >= ld
    quarter = prec_code == 1 and 256 * (WIDE_EPT[vec] // 4) >= ld  # fp32 d <= 2048: the quarter instance
    return 4 if quarter else 2 if replicas <= 1 or half else 1


def wide_bundle_rows(distinct_rows: int, n_cus: int = N_CUS, part_rows: Optional[Sequence[int]] = None,
                     per_cu: int = 2) -> int:
    """Rows per wide-row replica bundle (one workgroup per bundle, ``per_cu`` resident per CU): the
    shortest multiple of 16 rows whose bundles (per partition) all start in the first dispatch round,
    the rule of multi_bundle_rows.  The earlier "about 4 bundles per CU" sizing put 1032 bundles of
    976 rows on 1024 slot-rounds at 1e6 rows (a third, near-empty round) and 1042 of 96 rows at 1e5."""
    slots = per_cu * n_cus
    parts = [int(r) for r in part_rows if r > 0] if part_rows else [distinct_rows / 8.0] * 8
    base = max(16, 16 * int(np.ceil(distinct_rows / slots / 16)))

    def fits(rows: int) -> bool:
        return sum(int(np.ceil(p / rows)) for p in parts) <= slots

    rows = base
    while not fits(rows) and rows < max(parts):
        rows += 16
    return rows if fits(rows) else base


WIDE_EPT = {2: 16, 4: 32, 8: 32}  # elements per thread per row of grad_dense_wide (by vector width)


def choose_cpl(ld: int, vec: int) -> Optional[int]:
    """Kernel selector of the single-pass dense gradient.

    2..32       grad_dense_fused: a wave owns a row, ``cpl`` columns per lane (64 * cpl >= ld)
    256, 512    grad_dense_wide: a workgroup of that many threads owns a row (wide d)
    None        two-pass path (rows wider than 8192 fp64 / 16384 fp32, bf16 elements)
    """
    for c in (2, 4, 8, 16, 32):
        if c % vec == 0 and 64 * c >= ld:
            return c
    for bs in (256, 512):
        if bs * WIDE_EPT[vec] >= ld:
            return bs
    return None


XCDS = 8  # MI355X: workgroups are dealt round-robin over the 8 XCDs (block b -> XCD b % 8)


def replica_dispatch_order(keys: Sequence[Tuple[int, int]], stride: int = 0) -> List[int]:
    """Dispatch order of the gradient tasks that co-schedules replicas on one XCD.

    Co-located logical workers of a replicated scheme read identical rows: every member of an
    FRC/AGC group holds the same partitions, cyclic neighbours share s of their s+1.  In
    message-major order those reads are hundreds of workgroups apart and each streams the rows
    from HBM again.  Here the tasks that read the same (partition, row range) — a *bundle* —
    are placed 8 dispatch slots apart, so (blocks being dealt round-robin over the XCDs) they
    start together on the same XCD and walk the same rows in step: one HBM read feeds the
    others from that XCD's L2 / the Infinity Cache.  Every task still runs in full; only the
    order changes, and slab rows stay message-major, so results are bitwise unchanged.

    keys[i] = (partition, first row) of task i (message-major order).  Returns a permutation.
    stride: dispatch distance between bundle members (default XCDS: same XCD).
    """
    stride = stride or XCDS
    bundles: Dict[Tuple[int, int], List[int]] = {}
    for i, k in enumerate(keys):
        bundles.setdefault(k, []).append(i)
    by_size: Dict[int, List[List[int]]] = {}
    for b in bundles.values():  # first-appearance order
        by_size.setdefault(len(b), []).append(b)
    order: List[int] = []
    for size in sorted(by_size, reverse=True):
        group = by_size[size]
        for c in range(0, len(group), stride):
            chunk = group[c:c + stride]
            for m in range(size):  # member m of bundle j at offset m * len(chunk) + j
                order.extend(b[m] for b in chunk)
    return order


def _residual_torch(kind: int, z, y, coef):
    if kind == LOGISTIC:
        return -(coef * y) * torch.sigmoid(-(y * z))
    return -2.0 * coef * (y - z)


class DenseGradPlan:
    """Gradient of every local message over dense partitions.

    partitions: {partition_index: (X [rows, ld] storage dtype, y [rows] acc dtype)}
    messages:   sequence of (segments) where segments = [(partition_index, coef), ...]
    """

    def __init__(self, messages: Sequence[Sequence[Tuple[int, float]]],
                 partitions: Dict[int, Tuple[torch.Tensor, torch.Tensor]], prec: Precision, loss: int, d: int,
                 target_tasks: Optional[int] = None, choice: Optional[KernelChoice] = None):
        """choice: the kernel to launch (tests / sweeps); default: :func:`choose_kernel`'s measured pick."""
        self.prec = prec
        self.loss = loss
        self.d = d
        self.ld = prec.ld(d)
        self.messages = [list(m) for m in messages]
        self.partitions = partitions
        self.nslots = len(self.messages)
        any_t = next(iter(partitions.values()))[0] if partitions else torch.empty(0)
        self.device = any_t.device
        for p, (X, y) in partitions.items():
            if X.dim() != 2 or X.shape[1] != self.ld or X.dtype != prec.storage or not X.is_contiguous():
                raise ValueError(f"partition {p}: X must be contiguous [rows, {self.ld}] {prec.storage}")
            if y.shape[0] != X.shape[0] or y.dtype != prec.acc:
                raise ValueError(f"partition {p}: y must be [{X.shape[0]}] {prec.acc}")
        self.total_rows = sum(partitions[p][0].shape[0] for m in self.messages for p, _ in m)
        self.cpl = choose_cpl(self.ld, prec.vec)
        # co-located replicas: a partition read by several local messages
        self.max_rep = max(collections.Counter(p for m in self.messages for p, _ in m).values(), default=0)
        part_rows = [partitions[p][0].shape[0] for p in sorted({p for m in self.messages for p, _ in m})]
        distinct_rows = sum(part_rows)
        self.choice = choice or choose_kernel(prec.code, self.ld, self.cpl, self.max_rep, distinct_rows,
                                              part_rows=part_rows)
        c = self.choice
        if c.kind == "twopass" and self.cpl is not None:
            raise ValueError("the two-pass kernel is for rows wider than the one-pass kernels")
        if c.kind in ("multi", "staged", "mfma") and (self.cpl is None or self.cpl > MAX_CPL):
            raise ValueError(f"{c.kind} bundles need d <= {64 * MAX_CPL} columns per vector width")
        if c.kind == "multi" and (self.cpl > 16 or self.max_rep > 3):
            raise ValueError("one-wave bundles hold at most 3 replicas of rows of <= 16 columns per lane")
        if c.kind == "multi" and c.pair and (self.cpl > 8 or not c.fold):
            raise ValueError("pair-row one-wave bundles need <= 8 columns per lane and the fold")
        if c.kind == "wide" and c.replicas > 1 and (self.cpl not in (32, 256) or c.replicas > 3):
            raise ValueError("wide-row bundles are 256-thread rows (32 or 256 columns per lane) of at most 3 replicas")
        if c.kind == "mfma" and (prec.code != 2 or self.ld > 1024 or self.ld % 8 or self.max_rep > 16):
            raise ValueError("MFMA bundles are bf16, d <= 1024, d % 8 == 0, at most 16 replicas")
        self.bundle_rows = c.bundle_rows if c.bundled else 0
        if target_tasks is None:  # measured: smaller tasks keep interleaved replicas in step
            target_tasks = REPLICA_TASKS if c.interleave else DEFAULT_TASKS
        if self.bundle_rows:
            target_tasks = max(1, -(-self.total_rows // self.bundle_rows))
        if self.device.type == "cuda":
            self._native_choice = c.native()
            self._build_tables(target_tasks)

    # ---- device tables ----------------------------------------------------------------
    def _build_tables(self, target_tasks: int):
        segs = bytearray()
        tasks: List[Tuple[int, int, int, int]] = []
        slot_begin = [0]
        rows_per_task = max(MIN_ROWS_PER_TASK, -(-self.total_rows // max(1, target_tasks)))
        splits = None
        if self.choice.fill and self.choice.kind == "multi" and self.choice.fold:
            splits = fill_splits({p: self.partitions[p][0].shape[0] for m in self.messages for p, _ in m},
                                 self.choice.fill)
        seg_id = 0
        keys = []  # (partition, first row) of every task: equal keys read identical rows
        for slot, m in enumerate(self.messages):
            for p, coef in m:
                X, y = self.partitions[p]
                n = X.shape[0]
                segs += _SEG.pack(X.data_ptr(), y.data_ptr(), float(coef), n)
                bounds = splits[p] if splits else list(range(0, n, rows_per_task)) + [n]
                for r0, r1 in zip(bounds[:-1], bounds[1:]):
                    tasks.append((slot, seg_id, r0, r1, len(tasks)))
                    keys.append((p, r0))
                seg_id += 1
            slot_begin.append(len(tasks))
        if self.bundle_rows:
            tasks, folded_begin = self._bundle_table(tasks, keys)
            if folded_begin is not None:  # one slab row per (workgroup, replica): see _fold_table
                slot_begin = folded_begin
        elif self.choice.interleave:
            tasks = [tasks[i] for i in replica_dispatch_order(keys)]
        dev = self.device
        self.segs = torch.tensor(list(bytes(segs) or b"\0" * 32), dtype=torch.uint8).to(dev)
        self.ntasks = len(tasks)
        t = np.asarray(tasks, dtype=np.int32).reshape(-1, 5)
        self.tasks = torch.from_numpy(t).to(dev)
        self.slot_task_begin = torch.tensor(slot_begin, dtype=torch.int32, device=dev)
        self.slab = torch.empty((max(1, self.ntasks), self.ld), dtype=self.prec.acc, device=dev)
        # slab partial sums [nslots, SLAB_SPLITS, ld] (csrc/kernels/launchers.h slab_part_bytes)
        self.part = torch.zeros(max(1, self.nslots) * SLAB_SPLITS * self.ld, dtype=self.prec.acc, device=dev)
        if self.cpl is None:
            off = np.zeros(max(1, self.ntasks), dtype=np.int64)
            if self.ntasks:
                off[1:] = np.cumsum(t[:, 3] - t[:, 2])[:-1]
            if off.size and off[-1] + (t[-1, 3] - t[-1, 2] if self.ntasks else 0) >= 2 ** 31:
                raise ValueError("two-pass plan exceeds int32 row offsets")
            self.task_row_off = torch.from_numpy(off.astype(np.int32)).to(dev)
            self.rbuf = torch.empty(max(1, int(self.total_rows)), dtype=self.prec.acc, device=dev)

    def _bundle_table(self, tasks, keys):
        """Replica-bundle layout: R task slots per bundle (one wave each, or all in one wave for multi)."""
        bundles: Dict[Tuple[int, int], List[int]] = {}
        for i, k in enumerate(keys):
            bundles.setdefault(k, []).append(i)
        groups: List[List[int]] = []
        for b in bundles.values():
            groups += [b[i:i + MAX_BUNDLE] for i in range(0, len(b), MAX_BUNDLE)]
        R = max(len(g) for g in groups)
        if R != self.choice.replicas:
            raise ValueError(f"the plan's bundles hold {R} replicas, the kernel choice {self.choice.replicas}")
        pad = (0, -1, 0, 0, 0)
        table = []
        for g in groups:
            table += [tasks[i] for i in g] + [pad] * (R - len(g))
        if self.choice.kind == "multi" and self.choice.fold:
            return self._fold_table(groups, tasks, keys, R, pad)
        return table, None

    def _fold_table(self, groups, tasks, keys, R: int, pad):
        """Bundle table of the folded one-wave kernel (variant 70 + R): workgroups of 4 bundles of one
        partition, padded at a partition's end, so replica slot q is the same message in all four.
        Wave 0 writes one slab row per (workgroup, replica), numbered message by message; returns
        the table and the per-message slab row ranges that replace the message-major ones."""
        aligned: List[Optional[List[int]]] = []
        cur = None
        for g in groups:
            p = keys[g[0]][0]
            if p != cur and len(aligned) % 4:
                aligned += [None] * (4 - len(aligned) % 4)
            cur = p
            aligned.append(g)
        if len(aligned) % 4:
            aligned += [None] * (4 - len(aligned) % 4)
        per_slot: Dict[int, List[Tuple[int, int]]] = collections.defaultdict(list)
        for w in range(len(aligned) // 4):
            for q, ti in enumerate(aligned[4 * w]):  # a workgroup starts with a real bundle
                per_slot[tasks[ti][0]].append((w, q))
        slab_of: Dict[Tuple[int, int], int] = {}
        slot_begin = [0]
        for slot in range(self.nslots):
            for wq in per_slot[slot]:
                slab_of[wq] = len(slab_of)
            slot_begin.append(len(slab_of))
        table = []
        for b, g in enumerate(aligned):
            for q in range(R):
                if g is None or q >= len(g):
                    table.append(pad)
                    continue
                t = tasks[g[q]]
                table.append((t[0], t[1], t[2], t[3], slab_of[(b // 4, q)] if b % 4 == 0 else t[4]))
        return table, slot_begin

    def out_buffer(self, n: int = 1) -> torch.Tensor:
        """Message buffer(s) [n, nslots, ld] in the accumulator dtype."""
        return torch.zeros((n, self.nslots, self.ld), dtype=self.prec.acc, device=self.device)

    # ---- execution -------------------------------------------------------------------
    def run(self, beta: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
        """G[slot] = gradient of message slot at beta (beta: [ld] acc dtype)."""
        if G.shape != (self.nslots, self.ld):
            raise ValueError(f"G must be [{self.nslots}, {self.ld}]")
        if self.device.type == "cuda":
            C = native()
            if self.cpl is not None:
                C.grad_dense(self.prec.code, self.loss, self.cpl, self.segs, self.tasks, beta, self.slab,
                             self.slot_task_begin, self.part, G, self.ld, self._native_choice)
            else:
                C.grad_dense_twopass(self.prec.code, self.loss, self.segs, self.tasks, beta, self.task_row_off,
                                     self.rbuf, self.slab, self.slot_task_begin, self.part, G, self.ld)
            return G
        return self._run_torch(beta, G)

    def native_launcher(self):
        """C++ GradLauncher for the native round executors (csrc/runtime/engine.cpp)."""
        if self.device.type != "cuda":
            raise RuntimeError("native launchers need GPU tensors")
        C = native()
        if self.cpl is not None:
            return C.GradLauncher.dense(self.prec.code, self.loss, self.cpl, self.segs, self.tasks, self.slab,
                                        self.slot_task_begin, self.part, self.ld, choice=self._native_choice)
        return C.GradLauncher.dense(self.prec.code, self.loss, 0, self.segs, self.tasks, self.slab,
                                    self.slot_task_begin, self.part, self.ld, self.task_row_off, self.rbuf)

    def _run_torch(self, beta, G):
        acc = self.prec.acc
        b = beta.to(acc)
        for slot, m in enumerate(self.messages):
            g = torch.zeros(self.ld, dtype=acc)
            for p, coef in m:
                X, y = self.partitions[p]
                Xa = X.to(acc)
                z = Xa @ b
                r = _residual_torch(self.loss, z, y, torch.tensor(coef, dtype=acc))
                g += Xa.t() @ r
            G[slot].copy_(g)
        return G

    @property
    def bytes_per_round(self) -> int:
        """Bytes of X the messages read per round (every message's rows; replicas counted each time)."""
        es = torch.tensor([], dtype=self.prec.storage).element_size()
        return int(self.total_rows) * self.ld * es

    @property
    def distinct_bytes(self) -> int:
        """Bytes of the distinct partitions behind those rows (the HBM floor when replicas share reads)."""
        es = torch.tensor([], dtype=self.prec.storage).element_size()
        rows = sum(self.partitions[p][0].shape[0] for p in {p for m in self.messages for p, _ in m})
        return int(rows) * self.ld * es


class SparseGradPlan:
    """Gradient of every local message over CSR partitions (one-hot / pattern-only aware).

    partitions: {partition_index: (scipy.sparse.csr_matrix, y ndarray float64)}

    GPU (csrc/kernels/grad_sparse.hip): every DISTINCT partition of the local messages is read once
    with coefficient 1 -- row pass (ELL with 16-bit window offsets, or CSR) -> u, a deterministic
    column pass over 512-entry CSC tiles -> Gb[partition] -- and the launcher's device encoding forms
    G[message] = sum coef * Gb[partition] (the label encoding is linear in the coefficient), so
    co-located replicas (FRC / AGC groups, cyclic neighbours) share one read of their partitions
    (the reference repeats it per worker: ref src/replication.py:63-68).  No float atomics: the
    result is bitwise reproducible.  CPU: scipy per message (the reference's own arithmetic).
    """

    TILE = 512  # grad_sparse.hip kTileEntries
    ROW_BLOCK_ROWS = 4096  # residuals of one column-pass sub-block, staged in LDS
    # tiles per column-pass workgroup (wave w takes w, w + 16, ...): a fixed count (<= grad_sparse.hip
    # kMaxWgTiles), or None -- balanced chunks sized to the chip (csc_tables slots): at most WG_SLOTS
    # workgroups (256 CUs x 2 resident), chunks of 16 tiles when there are few.  Fixed 16 / 32 / 48 / 64 at
    # covtype-shaped naive: 57.0 / 54.5 / 53.2 / 51.7 us (64: 680 workgroups, a second partial dispatch round);
    # kc_house / amazon (0.6k / 2.3k tiles) want 16 (13.7 / 21.3 us; 22.8 / 35.8 at 64); profiles/round5/sparse/
    WG_TILES = None
    MAX_WG_TILES = 128
    WG_SLOTS = 512
    # column-aligned workgroup chunks (csc_tables wg_spans): the crossing columns are summed inside the
    # column pass's workgroups, no csc_spans launch and no head / tail round trip
    WG_SPANS = True  # (False: the csc_spans launch; tools/bench_kernels.py --no-wg-spans, for A/B)
    # beta bytes the ELL row pass stages in LDS (grad_sparse.hip kEllLdsBytes).  ELL rows pay off there
    # (covtype-shaped, 124 KB of fp64 beta: 54.7 vs 105.3 us with CSR rows); a beta that does not fit
    # leaves ELL one row per thread gathering from L2, which the CSR pass (8 lanes per row since round 6) beats on
    # the real shapes (amazon 33.1 vs 37.9 us, kc_house 18.4 vs 18.9: profiles/round4/r5a/breakdown.txt)
    ELL_LDS_BYTES = 148 * 1024
    # FRC / AGC units: a group's replicas all send the SAME message (the sum of the group's partitions,
    # coefficient 1: ref src/replication.py:56-68), so the device stacks the group's partitions into one
    # unit and the column pass writes the unit's sums straight into every member's message row
    # (SparseArgs::dst) -- no per-partition rows and no encoding launch, the naive plan's work.  Units
    # up to this many rows are staged whole (grad_sparse.hip csc_tiles_lds UNITS); larger ones keep the
    # partition basis and the encoding.
    UNIT_ROWS = 8192
    MAX_DST = 4  # grad_sparse.hip kSparseMaxDst: replicas per unit

    def __init__(self, messages: Sequence[Sequence[Tuple[int, float]]], partitions: Dict[int, Tuple[object, np.ndarray]],
                 prec: Precision, loss: int, d: int, device="cpu", use_ell="auto"):
        import scipy.sparse as sps

        if prec.name == "bf16":
            raise ValueError("sparse data uses fp64 or fp32 values (bf16 has no benefit for one-hot data)")
        self.prec, self.loss, self.d = prec, loss, d
        self.ld = prec.ld(d)
        self.messages = [list(m) for m in messages]
        self.nslots = len(self.messages)
        self.device = torch.device(device)
        self.basis = sorted({p for m in self.messages for p, _ in m})  # distinct partitions
        pos = {p: j for j, p in enumerate(self.basis)}
        self.blocks = []
        for p in self.basis:
            A, y = partitions[p]
            A = sps.csr_matrix(A)
            if A.shape[1] > d:
                raise ValueError("partition has more columns than d")
            A = sps.csr_matrix((A.data, A.indices, A.indptr), shape=(A.shape[0], d))
            A.sort_indices()
            self.blocks.append((A, np.asarray(y, dtype=np.float64)))
        X = sps.vstack([b[0] for b in self.blocks], format="csr") if self.blocks else sps.csr_matrix((0, d))
        X = sps.csr_matrix((X.data, X.indices, X.indptr), shape=(X.shape[0], d))
        X.sort_indices()
        self.nrows = X.shape[0]  # distinct rows
        self.nnz = X.nnz
        self.msg_rows = sum(self.blocks[pos[p]][0].shape[0] for m in self.messages for p, _ in m)
        self.pattern_only = bool(X.nnz == 0 or np.all(X.data == 1.0))
        # encoding: message slot -> (distinct partition, coefficient) in message order
        ptr, idx, coef = [0], [], []
        for m in self.messages:
            for p, c in m:
                idx.append(pos[p])
                coef.append(float(c))
            ptr.append(len(idx))
        self._enc = (ptr, idx, coef)
        self.ell = False
        self.idx16 = False
        self.row16 = False
        self.identity = False  # set by _build_device: messages are the distinct partitions themselves
        self.units = None  # set on the GPU for FRC / AGC groups (UNIT_ROWS): the message sets, stacked
        if self.device.type == "cuda":
            self.units = self._merge_units()
            if self.units is not None:  # the device's rows in unit order: each unit's partitions stacked
                dev_blocks = []
                for u in self.units:
                    mats = [self.blocks[pos[p]] for p in u]
                    Au = sps.vstack([m[0] for m in mats], format="csr")
                    Au = sps.csr_matrix((Au.data, Au.indices, Au.indptr), shape=(Au.shape[0], d))
                    Au.sort_indices()
                    dev_blocks.append((Au, np.concatenate([m[1] for m in mats])))
                X = sps.vstack([b[0] for b in dev_blocks], format="csr")
                X = sps.csr_matrix((X.data, X.indices, X.indptr), shape=(X.shape[0], d))
                X.sort_indices()
            else:
                dev_blocks = self.blocks
            self._build_device(X, use_ell, dev_blocks)

    def _merge_units(self):
        """The FRC / AGC message sets as device units (see UNIT_ROWS), or None: every coefficient 1, some
        set used by several messages, any two sets identical or disjoint, at most MAX_DST messages per
        set, and every unit at most UNIT_ROWS rows."""
        sets = [tuple(sorted(p for p, _ in m)) for m in self.messages]
        if not sets or any(float(c) != 1.0 for m in self.messages for _, c in m) or len(set(sets)) == len(sets):
            return None
        units = sorted(set(sets))
        seen = set()
        for u in units:
            if seen & set(u) or sets.count(u) > self.MAX_DST:
                return None
            seen |= set(u)
        pos = {p: j for j, p in enumerate(self.basis)}
        if max(sum(self.blocks[pos[p]][0].shape[0] for p in u) for u in units) > self.UNIT_ROWS:
            return None
        return units

    # ---- device tables ----------------------------------------------------------------------
    def _build_device(self, X, use_ell: bool, dev_blocks):
        """dev_blocks: the device's (matrix, labels) units in row order -- the distinct partitions, or the
        merged FRC / AGC units (self.units)."""
        dev, acc = self.device, self.prec.acc
        npacc = np.float64 if acc == torch.float64 else np.float32
        ys = np.concatenate([b[1] for b in dev_blocks]) if dev_blocks else np.zeros(0)
        self.y = torch.from_numpy(ys.astype(npacc)).to(dev)
        self.u = torch.zeros(max(1, self.nrows), dtype=acc, device=dev)
        nnz_row = np.diff(X.indptr)
        self.ell_idx = self.ell_lo = self.row_ptr = self.col_idx = self.vals = None
        self.csr_fixed = 0
        beta_lds = self.d * torch.tensor([], dtype=acc).element_size() <= self.ELL_LDS_BYTES
        if use_ell == "auto":
            use_ell = beta_lds
        if use_ell and self.nrows and np.all(nnz_row == nnz_row[0]) and nnz_row[0] > 0 and self.nrows < 2 ** 31:
            m = int(nnz_row[0])
            idx = X.indices.reshape(self.nrows, m).T  # [m, rows]; sorted rows -> the k-th smallest column
            lo = idx.min(axis=1).astype(np.int64)
            width = idx.max(axis=1) - lo + 1
            self.ell, self.ell_m = True, m
            # an even row stride: the LDS row pass loads a row pair's field at once (grad_sparse.hip
            # ell_rows_lds); the padding row points at each window's first column with value 0
            pad = self.nrows % 2

            def padded(x):
                return np.ascontiguousarray(np.pad(x, ((0, 0), (0, pad))) if pad else x)

            if int(width.max()) <= 65536:  # 16-bit offsets into each feature's category window
                self.idx16 = True
                off = (idx - lo[:, None]).astype(np.uint16).view(np.int16)
                self.ell_idx = torch.from_numpy(padded(off)).to(dev)
                self.ell_lo = torch.from_numpy(lo.astype(np.int32)).to(dev)
            else:
                self.ell_idx = torch.from_numpy(padded(idx.astype(np.int32))).to(dev)
            if not self.pattern_only:
                self.vals = torch.from_numpy(padded(X.data.reshape(self.nrows, m).T.astype(npacc))).to(dev)
        else:
            self.row_ptr = torch.from_numpy(X.indptr.astype(np.int64)).to(dev)
            self.col_idx = torch.from_numpy(X.indices.astype(np.int32)).to(dev)
            # one-hot rows: the same nnz everywhere, so the row pass skips its row_ptr load
            if self.nrows and np.all(nnz_row == nnz_row[0]) and nnz_row[0] > 0:
                self.csr_fixed = int(nnz_row[0])
            if not self.pattern_only:
                self.vals = torch.from_numpy(X.data.astype(npacc)).to(dev)
        # residual sub-blocks staged in LDS by the column pass: 4096 rows (32 KB fp64, 16 KB fp32; four
        # staged values per thread of its 1024-thread workgroups, grad_sparse.hip kStageRegs)
        rb = self.ROW_BLOCK_ROWS
        wgt = self.WG_TILES
        self.wg_tiles = wgt or self.MAX_WG_TILES
        if self.units is not None:  # a unit is one sub-block of up to UNIT_ROWS rows (csc_tiles_lds UNITS)
            rb = max(rb, max(b[0].shape[0] for b in dev_blocks))
        t = self.csc_tables([b[0] for b in dev_blocks], self.d, self.TILE, row_block=rb, wg_tiles=self.wg_tiles,
                            wg_spans=self.WG_SPANS, slots=0 if wgt else self.WG_SLOTS)
        self.row_block = rb
        self.nsub = t["nsub"]
        self.row16 = t["row16"]
        self.crow = torch.from_numpy(t["crow"]).to(dev)
        self.cvals = None if self.pattern_only else torch.from_numpy(t["cvals"].astype(npacc)).to(dev)
        self.col_ptr = torch.from_numpy(t["col_ptr"]).to(dev)
        self.tiles = torch.from_numpy(t["tiles"]).to(dev)
        self.part_entry0 = torch.from_numpy(t["part_entry0"]).to(dev)
        self.part_row0 = torch.from_numpy(t["part_row0"]).to(dev)
        self.part_nnz = torch.from_numpy(t["part_nnz"]).to(dev)
        self.span = torch.from_numpy(t["span"]).to(dev)
        self.empty = torch.from_numpy(t["empty"]).to(dev)
        nt = max(1, len(t["tiles"]))
        self.head = torch.zeros(nt, dtype=acc, device=dev)
        self.tail = torch.zeros(nt, dtype=acc, device=dev)
        self.Gb = torch.zeros((max(1, len(self.basis)), self.ld), dtype=acc, device=dev)
        self.wg = torch.from_numpy(t["wg"]).to(dev)
        self.runs = torch.from_numpy(t["runs"]).to(dev)
        self.tkeys = torch.from_numpy(t["tkeys"]).to(dev)
        self.u_lds = int(t["wg"][:, 3].max()) if len(t["wg"]) else 1
        self.wg_spans = bool(t["wg_spans"]) and len(t["wg"]) > 0
        self.wspan = torch.from_numpy(t["wspan"]).to(dev) if self.wg_spans else None
        self.wspan_ptr = torch.from_numpy(t["wspan_ptr"]).to(dev) if self.wg_spans else None
        blocked = self.nsub != len(dev_blocks)  # some partition spans several sub-blocks
        self.sub_begin = torch.from_numpy(t["sub_begin"]).to(dev) if blocked else None
        self.Gs = torch.zeros((self.nsub, self.ld), dtype=acc, device=dev) if blocked else None
        ptr, idx, coef = self._enc
        # identity encoding (naive: message i is distinct partition i with coefficient 1, no sub-blocks):
        # the column pass writes the messages themselves, no Gb and no encode launch (amazon-shaped
        # naive: 15.5 MB read + 15.5 MB written per round).  Two kinds of G columns are then never
        # written: the columns empty in a partition (native_launcher hands the kernels no empty-column
        # list) and the padding columns [d, ld).  Both stay as the caller's G holds them, so an identity
        # plan needs a G that is zero there -- every buffer the plans and the trainer allocate is
        # (out_buffer, the trainer's G ring); run() checks it the first time it sees a buffer.
        self.identity = (not blocked and len(self.messages) == len(self.basis)
                         and all(m == [(self.basis[i], 1.0)] for i, m in enumerate(self.messages)))
        self.dst = None
        if self.units is not None:
            if blocked:
                raise AssertionError("a merged unit must be one sub-block")
            sets = [tuple(sorted(p for p, _ in m)) for m in self.messages]
            dst = np.full((len(self.units), self.MAX_DST), -1, dtype=np.int32)
            for j, u in enumerate(self.units):
                rows = [i for i, s in enumerate(sets) if s == u]
                dst[j, : len(rows)] = rows
            self.dst = torch.from_numpy(dst).to(dev)
            self.identity = True  # the column pass writes the messages themselves
        self.enc_ptr = torch.tensor(ptr, dtype=torch.int32, device=dev)
        self.enc_idx = torch.tensor(idx or [0], dtype=torch.int32, device=dev)[: len(idx)]
        self.enc_coef = torch.tensor(coef or [0.0], dtype=torch.float64, device=dev)[: len(coef)]
        self._launcher = None
        self._zero_checked = set()  # G buffers run() has seen zero in the padding columns

    @staticmethod
    def csc_tables(blocks, d: int, tile: int = 512, row_block: int = 0, wg_tiles: int = 16,
                   wg_spans: bool = False, slots: int = 0) -> dict:
        """Host tables of the deterministic column pass (grad_sparse.hip csc_tiles / csc_spans): per
        partition a CSC twin (rows sorted by (column, row), padded to whole tiles), its column
        pointers, the tiles (partition, base entry, column of the base entry, span flags: 1 = the
        first column began in an earlier tile, 2 = the last goes on in a later one), the columns that
        cross tiles (partition, column, first tile, last tile) and the empty columns.

        Every row index carries a run-start flag in its top bit (bit 15 of 16-bit rows, so those need
        <= 32768 rows; bit 31 otherwise): set on the first entry of each column and of each tile.
        runs / tkeys: every tile's run columns in order, and per tile (first run, n | runs << 10 |
        span flags << 20, partition, first column) -- the keyed column pass reads a tile's columns
        from there instead of walking the column pointers.

        row_block > 0: every partition is cut into sub-blocks of at most that many rows and the tables
        are built per sub-block (the "partitions" of the kernels are then the sub-blocks; sub_begin[j]
        lists partition j's).  A workgroup takes up to wg_tiles tiles of ONE sub-block and stages
        that sub-block's residuals in LDS (wg: first row of the sub-block, first tile, tiles, rows),
        so the column pass's gathers never leave the CU; the sub-block sums are added per partition
        afterwards.

        wg_spans (with row_block > 0): a workgroup's chunk of tiles ends on a column boundary -- its
        last tile is cut short (padded) before the first column that would not fit -- so no column
        crosses workgroups and the workgroup adds its own crossing columns from LDS after its tiles
        (wspan: sub-block, column, first and last tile relative to the chunk; wspan_ptr: each
        workgroup's range).  No csc_spans launch, no head / tail round trip through memory.  Tile t's
        entries still sit at crow[tile * t ...]; its entry count is tkeys' n (< tile for a cut tile).
        Falls back to whole chunks (span = the global list) when a column is longer than a chunk.

        slots > 0 (with wg_spans): balanced chunks sized to the chip -- sub-block s (T_s tiles of T in
        all) is cut into n_s = max(1, min(ceil(T_s / 16), floor(T_s * slots / T))) chunks of about
        T_s / n_s tiles (at most wg_tiles), so at most `slots` workgroups (one dispatch round of the
        column pass's 2 per CU) when the tiles are many, and chunks of 16 when they are few."""
        import scipy.sparse as sps

        sub_begin = None
        if row_block > 0:
            subs, sub_begin = [], [0]
            for A in blocks:
                n = A.shape[0]
                for r in range(0, max(n, 1), row_block):
                    subs.append(sps.csr_matrix(A[r:min(n, r + row_block)]))
                sub_begin.append(len(subs))
            blocks = subs
        cuts = wg_spans and row_block > 0
        cscs = []
        for A in blocks:
            C = A.tocsc()
            C.sort_indices()
            cscs.append(C)
            if cuts and C.nnz and int(np.diff(C.indptr).max()) > tile * wg_tiles:
                cuts = False  # a column longer than a chunk: whole chunks and the global spans
        total_tiles = sum(-(-C.nnz // tile) for C in cscs)
        row16 = all(A.shape[0] <= 32768 for A in blocks)
        flag = np.int64(1 << 15) if row16 else np.int64(1 << 31)
        rows_l, vals_l, cps, tiles, spans, empty = [], [], [], [], [], []
        runs_l, tkeys = [], []
        wg, wspan, wspan_ptr = [], [], [0]
        n_runs = 0
        entry0, row0, nnzs = [], [], []
        e_off = r_off = n_tiles = 0
        for j, (A, C) in enumerate(zip(blocks, cscs)):
            cp = C.indptr.astype(np.int64)
            nnz = int(cp[-1])
            r = C.indices.astype(np.int64)
            col_of = np.repeat(np.arange(d, dtype=np.int64), np.diff(cp))  # each entry's column
            nonempty = np.nonzero(cp[1:] > cp[:-1])[0]
            cstart = cp[nonempty]  # first entry of every non-empty column
            # tiles [bases, ends) and the chunks of tiles (first tile, tiles) of this block
            if cuts:
                bl, chunks, pos = [], [], 0
                per = tile * wg_tiles  # entries per chunk
                if slots > 0 and nnz:
                    ts = -(-nnz // tile)
                    n_s = max(1, min(-(-ts // 16), (ts * slots) // max(1, total_tiles)))
                    per = min(per, -(-nnz // n_s))
                while pos < nnz:
                    lim = pos + per
                    end = nnz if lim >= nnz else int(cstart[np.searchsorted(cstart, lim, side="right") - 1])
                    chunks.append((len(bl), -(-(end - pos) // tile)))
                    bl.extend(range(pos, end, tile))
                    pos = end
                bases = np.asarray(bl, dtype=np.int64)
                ends = np.minimum(bases + tile, np.append(bases[1:], nnz)) if bases.size else bases
            else:
                bases = np.arange(0, nnz, tile, dtype=np.int64)
                ends = np.minimum(bases + tile, nnz)
                chunks = [(t0, min(wg_tiles, bases.size - t0)) for t0 in range(0, bases.size, wg_tiles)]
            nt = bases.size
            start = np.zeros(nnz, dtype=bool)  # run starts: first entry of a column or of a tile
            start[cstart] = True
            start[bases] = True
            r = np.where(start, r | flag, r)
            # tile k's entries at slots [tile * k, tile * k + (ends - bases)), the rest zero padding
            slot = np.zeros(nnz, dtype=np.int64)
            if nnz:
                tof = np.searchsorted(bases, np.arange(nnz), side="right") - 1
                slot = tof * tile + (np.arange(nnz) - bases[tof])
            rr = np.zeros(nt * tile, dtype=np.int64)
            vv = np.zeros(nt * tile)
            rr[slot] = r
            vv[slot] = C.data.astype(np.float64)
            rows_l.append(rr)
            vals_l.append(vv)
            cps.append(cp.astype(np.int32))
            entry0.append(e_off)
            row0.append(r_off)
            nnzs.append(nnz)
            t_first = n_tiles
            if nt:
                c0 = np.searchsorted(cp, bases, side="right") - 1
                c_last = np.searchsorted(cp, ends - 1, side="right") - 1
                flags = (cp[c0] < bases).astype(np.int64) | 2 * (cp[c_last + 1] > ends).astype(np.int64)
                tiles.append(np.stack([np.full(nt, j), bases, c0, flags], axis=1))
                n_tiles += nt
                sidx = np.nonzero(start)[0]
                runs_l.append(col_of[sidx])
                r_first = np.searchsorted(sidx, bases)  # runs before each tile
                r_cnt = np.diff(np.append(r_first, sidx.size))
                ns = ends - bases
                tkeys.append(np.stack([n_runs + r_first, ns | (r_cnt << 10) | (flags << 20),
                                       np.full(nt, j), c0], axis=1))
                n_runs += sidx.size
            t1 = np.searchsorted(bases, cp[nonempty], side="right") - 1
            t2 = np.searchsorted(bases, cp[nonempty + 1] - 1, side="right") - 1
            cross = t2 > t1
            if row_block > 0:
                for k, (c_t0, c_nt) in enumerate(chunks):
                    wg.append((r_off, t_first + c_t0, c_nt, A.shape[0]))
                    if cuts:
                        inside = cross & (t1 >= c_t0) & (t1 < c_t0 + c_nt)
                        assert np.all(t2[inside] < c_t0 + c_nt) and inside.sum() < wg_tiles  # one per boundary
                        if inside.any():
                            wspan.append(np.stack([np.full(int(inside.sum()), j), nonempty[inside],
                                                   t1[inside] - c_t0, t2[inside] - c_t0], axis=1))
                        wspan_ptr.append(wspan_ptr[-1] + int(inside.sum()))
            if cross.any() and not cuts:
                spans.append(np.stack([np.full(int(cross.sum()), j), nonempty[cross], t_first + t1[cross],
                                       t_first + t2[cross]], axis=1))
            ec = np.nonzero(cp[1:] == cp[:-1])[0]
            if ec.size:
                empty.append(np.stack([np.full(ec.size, j), ec], axis=1))
            e_off += nt * tile
            r_off += A.shape[0]
        crow = np.concatenate(rows_l) if rows_l else np.zeros(tile, dtype=np.int64)
        crow = crow.astype(np.uint16).view(np.int16) if row16 else crow.astype(np.uint32).view(np.int32)
        extra = {"sub_begin": np.asarray(sub_begin, dtype=np.int32) if sub_begin is not None else None,
                 "wg": np.asarray(wg, dtype=np.int32).reshape(-1, 4), "nsub": len(blocks),
                 "row_block": int(row_block), "wg_spans": bool(cuts),
                 "wspan": (np.concatenate(wspan) if wspan else np.zeros((0, 4))).astype(np.int32).reshape(-1, 4),
                 "wspan_ptr": np.asarray(wspan_ptr if cuts else [0], dtype=np.int32)}
        return {**extra, "row16": row16, "crow": np.ascontiguousarray(crow),
                "cvals": np.concatenate(vals_l) if vals_l else np.zeros(tile),
                "col_ptr": np.ascontiguousarray(np.stack(cps)) if cps else np.zeros((1, d + 1), dtype=np.int32),
                "tiles": (np.concatenate(tiles) if tiles else np.zeros((0, 4))).astype(np.int32).reshape(-1, 4),
                "part_entry0": np.asarray(entry0 or [0], dtype=np.int64),
                "part_row0": np.asarray(row0 or [0], dtype=np.int64),
                "part_nnz": np.asarray(nnzs or [0], dtype=np.int32),
                "span": (np.concatenate(spans) if spans else np.zeros((0, 4))).astype(np.int32).reshape(-1, 4),
                "empty": (np.concatenate(empty) if empty else np.zeros((0, 2))).astype(np.int32).reshape(-1, 2),
                "runs": (np.concatenate(runs_l) if runs_l else np.zeros(1)).astype(np.int32),
                "tkeys": (np.concatenate(tkeys) if tkeys else np.zeros((0, 4))).astype(np.int32).reshape(-1, 4)}

    def out_buffer(self, n: int = 1) -> torch.Tensor:
        return torch.zeros((n, self.nslots, self.ld), dtype=self.prec.acc, device=self.device)

    def native_launcher(self):
        if self.device.type != "cuda":
            raise RuntimeError("native launchers need GPU tensors")
        if self._launcher is None:
            # the column pass writes into this plan's own zero-initialised Gs / Gb (the device encoding
            # set below always follows it) and never into a column that is empty in its (sub-)block,
            # so those zeros stay: the per-round zero writes are skipped (amazon-shaped data: 1.9M
            # of them, 242k columns x 8 partitions)
            empty = self.empty[:0]
            L = native().GradLauncher.sparse(self.loss, self.y, self.u, self.ell_idx, self.ell_lo, self.row_ptr,
                                             self.col_idx, self.vals, self.crow, self.cvals, self.col_ptr, self.tiles,
                                             self.part_entry0, self.part_row0, self.part_nnz, self.head, self.tail,
                                             self.span, empty, self.nsub, self.d, self.ld,
                                             wg=self.wg if len(self.wg) else None, u_lds=self.u_lds, Gs=self.Gs,
                                             sub_begin=self.sub_begin, runs=self.runs, tkeys=self.tkeys,
                                             wspan=self.wspan, wspan_ptr=self.wspan_ptr, dst=self.dst,
                                             csr_fixed=self.csr_fixed)
            if not self.identity:
                L.set_encode(self.enc_ptr, self.enc_idx, self.enc_coef, self.Gb)
            self._launcher = L
        return self._launcher

    @property
    def stream_bytes(self) -> int:
        """Index / value bytes one gradient streams from HBM (row pass + CSC tiles; beta and u gathers
        hit L2)."""
        if self.device.type != "cuda":
            return 0
        n = sum(t.numel() * t.element_size() for t in (self.ell_idx, self.row_ptr, self.col_idx, self.vals, self.crow,
                                                       self.cvals, self.y) if t is not None)
        return int(n + 2 * self.u.numel() * self.u.element_size())

    def run(self, beta: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
        """G [nslots, ld]: the messages.  An identity plan (see _build_device) leaves the columns empty
        in a partition and the padding columns [d, ld) as G holds them: pass a G that is zero there."""
        if G.shape != (self.nslots, self.ld):
            raise ValueError(f"G must be [{self.nslots}, {self.ld}]")
        if self.device.type == "cuda":
            if self.identity and self.ld > self.d and G.data_ptr() not in self._zero_checked:
                if bool((G[:, self.d:] != 0).any()):  # once per buffer (a host sync), off the round path
                    raise ValueError("identity sparse plan: G's padding columns [d, ld) must be zero")
                self._zero_checked.add(G.data_ptr())
            self.native_launcher().launch(beta, G)
            return G
        b = beta.detach().cpu().double().numpy()[: self.d]
        G.zero_()
        pos = {p: j for j, p in enumerate(self.basis)}
        for slot, m in enumerate(self.messages):
            g = np.zeros(self.d)
            for p, c in m:
                A, y = self.blocks[pos[p]]
                z = A.dot(b)
                if self.loss == LOGISTIC:
                    r = -(c * y) * (1.0 / (1.0 + np.exp(np.clip(y * z, -700, 700))))
                else:
                    r = -2.0 * c * (y - z)
                g += np.asarray(A.T.dot(r)).ravel()
            G[slot, : self.d] = torch.from_numpy(g).to(G.dtype)
        return G


class SharedGradPlan:
    """Distinct partitions once, then device encoding of every local message (``--share-partitions``).

    Logical workers placed on one GPU share partitions: all members of an FRC/AGC group hold
    the same (s+1) partitions (ref src/replication.py:56-68) and cyclic neighbours overlap in s
    of them (ref src/coded.py:31-50).  The faithful plans above compute every message from its
    own rows, streaming (s+1)-replicated X; this plan streams each distinct partition once
    (coefficient 1) into ``Gb`` and encodes ``G = E . Gb`` (csrc/kernels/encode.hip), E being
    the [messages x partitions] matrix of label-encoding coefficients.  The residual is linear
    in the coefficient, so every message is the same sum (up to fp rounding order).

    ``make_inner(messages)`` builds the dense or sparse plan over the basis messages.
    """

    def __init__(self, messages: Sequence[Sequence[Tuple[int, float]]], make_inner):
        self.messages = [list(m) for m in messages]
        self.nslots = len(self.messages)
        self.basis = sorted({p for m in self.messages for p, _ in m})
        pos = {p: j for j, p in enumerate(self.basis)}
        self.inner = make_inner([[(p, 1.0)] for p in self.basis])
        self.prec, self.loss, self.d, self.ld = self.inner.prec, self.inner.loss, self.inner.d, self.inner.ld
        self.device = self.inner.device
        ptr, idx, coef = [0], [], []
        for m in self.messages:
            for p, c in m:
                idx.append(pos[p])
                coef.append(float(c))
            ptr.append(len(idx))
        if idx and (min(idx) < 0 or max(idx) >= len(self.basis)):
            raise ValueError("encoding index out of range")
        self.E = torch.zeros((self.nslots, len(self.basis)), dtype=torch.float64)
        for s in range(self.nslots):
            for k in range(ptr[s], ptr[s + 1]):
                self.E[s, idx[k]] += coef[k]
        dev = self.device
        self.enc_ptr = torch.tensor(ptr, dtype=torch.int32, device=dev)
        self.enc_idx = torch.tensor(idx or [0], dtype=torch.int32, device=dev)[: len(idx)]
        self.enc_coef = torch.tensor(coef or [0.0], dtype=torch.float64, device=dev)[: len(coef)]
        self.Gb = self.inner.out_buffer()[0]

    @staticmethod
    def worthwhile(messages: Sequence[Sequence[Tuple[int, float]]], rows_of) -> bool:
        """True when the local messages stream some partition more than once."""
        total = sum(rows_of(p) for m in messages for p, _ in m)
        distinct = sum(rows_of(p) for p in {p for m in messages for p, _ in m})
        return distinct < total

    def out_buffer(self, n: int = 1) -> torch.Tensor:
        return torch.zeros((n, self.nslots, self.ld), dtype=self.prec.acc, device=self.device)

    @property
    def bytes_per_round(self) -> int:
        return getattr(self.inner, "bytes_per_round", 0)

    @property
    def distinct_bytes(self) -> int:
        return getattr(self.inner, "distinct_bytes", 0)

    def run(self, beta: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
        if G.shape != (self.nslots, self.ld):
            raise ValueError(f"G must be [{self.nslots}, {self.ld}]")
        self.inner.run(beta, self.Gb)
        if self.device.type == "cuda":
            native().encode_messages(self.Gb, self.enc_ptr, self.enc_idx, self.enc_coef, G)
        else:
            G.copy_((self.E.to(self.Gb.dtype) @ self.Gb).to(G.dtype))
        return G

    def native_launcher(self):
        L = self.inner.native_launcher()
        L.set_encode(self.enc_ptr, self.enc_idx, self.enc_coef, self.Gb)
        return L
