"""Worker-gradient execution plans (device side of K1-K4/K13).

A *plan* is built once per run for all logical workers hosted on one GPU: every
message (worker, part) is a list of segments (partition, label coefficient).  Each
round the plan is executed with one launch set:

  dense  -> ``grad_dense`` (fused single pass over X, slab reduction)   csrc/kernels/grad_dense.hip
            ``grad_dense_wide`` (a workgroup per row) when d > 2048 fp64       (same file)
            ``grad_dense_twopass`` beyond 8192 fp64 / 16384 fp32 columns
  sparse -> ``grad_sparse`` (CSR row pass + sorted-COO column pass)      csrc/kernels/grad_sparse.hip

On CPU tensors the same plans run a float64/float32 torch implementation of the
identical math (the test path and the gloo multi-process path); on GPU tensors the
native kernels are mandatory (:func:`erasurehead_amd._ext.native` raises if absent).
"""
from __future__ import annotations

import collections
import os
import struct
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
MAX_BUNDLE = 8  # replica task slots (waves) per workgroup of grad_dense_bundle / _staged
STAGED_ROWS = 512  # rows per bundle task of grad_dense_staged (measured: 512 > 256, 1024; 2048 leaves CUs idle)
SHARD_STAGED_ROWS = 128  # rows per bundle task when a rank holds < SHARD_ROWS distinct rows (multi-GPU shards)


def multi_bundle_rows(distinct_rows: int, fp32: bool = False) -> int:
    """Rows per one-wave bundle of grad_dense_multi, in multiples of 64 (tools/sweep_multi_rows.sh,
    profiles/r3_multi).  fp64 (244 VGPRs, 2 waves per SIMD): about 2000 bundles, 1300 at the
    one-GPU headline (N=1 768 rows 1.330 ms vs 512 1.36 / 640 1.37 / 1024 1.54; N=2 256 rows 0.708;
    N=4 128 rows 0.370 vs 96 0.45 / 160 0.40; N=8 64 rows 0.206 vs 48 0.25 / 80 0.22).  fp32
    (155 VGPRs, 3 waves per SIMD): about 2600 bundles, just under the 3072 wave slots (N=1 384
    rows 0.692 ms; 320 rows = 3125 bundles needs a second pass: 0.95)."""
    waves = 2600 if fp32 else 1300 if distinct_rows >= 750_000 else 1953
    return max(64, 64 * int(round(distinct_rows / waves / 64)))
SHARD_ROWS = 800_000
MIN_ROWS_PER_TASK = 32
SLAB_SPLITS = 16  # csrc/kernels/grad_dense.hip kSplits


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
    stride: dispatch distance between bundle members (default XCDS: same XCD; 1: adjacent
    slots, i.e. different XCDs sharing through the Infinity Cache — A/B runs only).
    """
    stride = stride or int(os.environ.get("ERASUREHEAD_REPLICA_STRIDE", XCDS))
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
                 target_tasks: Optional[int] = None, interleave: Optional[bool] = None):
        # replica-interleaved dispatch (see replica_dispatch_order); ERASUREHEAD_NO_INTERLEAVE=1 for A/B runs
        self.interleave = (not os.environ.get("ERASUREHEAD_NO_INTERLEAVE")) if interleave is None else interleave
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
        # co-located replicas (a partition in several local messages) read shared rows
        self.replicated = len({p for m in self.messages for p, _ in m}) < sum(len(m) for m in self.messages)
        shared = self.replicated and self.interleave
        if target_tasks is None:  # measured: smaller tasks keep interleaved replicas in step
            target_tasks = REPLICA_TASKS if shared else DEFAULT_TASKS
        # grad_dense_fused variant (csrc/kernels/grad_dense.hip fused_rows), measured per case:
        # one row in flight for interleaved replicas (L2-fed) in every precision; for distinct
        # rows the interleaved pair kernel (fp64), 4 rows (fp32), 1 row (bf16)
        self.variant = 1 if shared else {0: 2, 1: 4, 2: 1}[prec.code]
        # Replica bundles: the tasks that read the same rows run in one workgroup, one wave per
        # replica.  Default for fp64/fp32 replicas: grad_dense_staged streams each bundle's rows
        # from HBM once through LDS and every replica wave computes its own message from there
        # (measured 1.58 vs 1.80 ms fp64, 0.89 vs 0.99 ms fp32 at the headline; bf16 rows are
        # too short to pay for the staging: 0.70 vs 0.66 ms, docs/PERF_NOTES.md).
        # ERASUREHEAD_STAGED=0 / 1 / pair overrides (pair: two rows share one reduction and one
        # residual evaluation; the default for fp32 and sharded ranks, see below).
        staged_env = os.environ.get("ERASUREHEAD_STAGED", "")
        staged_ok = shared and self.cpl is not None and self.cpl <= MAX_CPL
        # One-wave bundles (grad_dense_multi, the fp64 default): one wave computes every replica of
        # its bundle from rows double-buffered in registers, with no LDS staging and no barrier.
        # R <= 3 replicas, d <= 1024.  Measured against the LDS-staged bundles, fp64
        # (profiles/r3_multi, r3_fold; with the workgroup fold): one-GPU headline 1.33 vs 1.45 ms,
        # 2/4/8-GPU rank shapes 0.70 / 0.36 / 0.195 vs 0.78 / 0.41-0.43 / 0.21-0.23 ms.  fp32: the one-GPU headline
        # (0.692 vs 0.740 ms); sharded fp32 ranks stay on the staged pair bundles (N=8 0.115-0.122
        # vs 0.129 ms).  ERASUREHEAD_STAGED=multi forces it for fp32.
        max_rep = max(collections.Counter(p for m in self.messages for p, _ in m).values(), default=0)
        multi_ok = staged_ok and self.cpl <= 16 and max_rep <= 3
        distinct_rows = sum(partitions[p][0].shape[0] for p in {p for m in self.messages for p, _ in m})
        # default only for bundles of 3 (AGC / cyclic with s = 2): with 2 replicas (FRC s = 1) the
        # staged bundles with two waves per replica stay ahead (1.36 vs 1.40 ms, profiles/r3_fold)
        self.multi = multi_ok and ((staged_env == "multi" and prec.code in (0, 1)) or (
            staged_env == "" and max_rep == 3 and (prec.code == 0 or (prec.code == 1 and distinct_rows >= 750_000))))
        self.staged = staged_ok and not self.multi and (
            staged_env in ("1", "pair") or (staged_env == "" and prec.code in (0, 1)))
        # two rows per step sharing one reduction: the fp32 default (0.790 vs 0.862 ms at the
        # headline, profiles/r2_fp32) and the default on sharded ranks of a multi-GPU run, where it
        # also wins for fp64 with one wave per replica (N=8 rank 0.213 vs 0.238 ms, N=4 0.407 vs
        # 0.429, profiles/r2_rank_sweep); slower for the one-GPU fp64 headline
        sharded = distinct_rows < SHARD_ROWS
        self.staged_pair = self.staged and (staged_env == "pair" or (staged_env == "" and (prec.code == 1 or sharded)))
        self.staged_wpr = 1 if (self.staged and sharded and staged_env == "") else 0  # 0: kernel default
        # bf16 replica bundles on the matrix cores (csrc/kernels/grad_mfma.hip): the R replicas of a
        # bundle are the M dimension of X·beta and Xᵀ·r per 32-row LDS stage.  ERASUREHEAD_MFMA=0
        # keeps the VALU kernels (A/B runs).
        self.mfma = (prec.code == 2 and staged_ok and self.ld <= 1024 and self.ld % 8 == 0
                     and os.environ.get("ERASUREHEAD_MFMA", "1") != "0")
        # rows per bundle task: 512 at the one-GPU headline (1e6 distinct rows); a rank holding the
        # partition shards of an N-GPU run (500k / 250k / 125k rows at N = 2 / 4 / 8) is fastest with
        # 128-row bundles (profiles/r2_shapes: N=8 0.238 vs 0.415 ms, N=2 0.80 vs 0.99 ms at 512)
        staged_rows = STAGED_ROWS if distinct_rows >= SHARD_ROWS else SHARD_STAGED_ROWS
        if self.mfma:
            # MFMA bundles run one 8-wave workgroup per CU (150 KB of LDS): long bundles amortise its
            # prologue (profiles/r2_mfma_ab2: 512 / 1024 / 2048 rows -> 0.458 / 0.440 / 0.430 ms at
            # the bf16 headline); about two bundles per CU, 256..2048 rows
            staged_rows = 256
            while staged_rows < 2048 and staged_rows * 512 < distinct_rows:
                staged_rows *= 2
        if self.multi:
            staged_rows = multi_bundle_rows(distinct_rows, fp32=prec.code == 1)
        default_rows = str(staged_rows) if (self.staged or self.mfma or self.multi) else "0"
        self.bundle_rows = int(os.environ.get("ERASUREHEAD_BUNDLE_ROWS", default_rows)) if (
            shared and self.cpl is not None and self.cpl <= MAX_CPL) else 0
        if self.bundle_rows:
            target_tasks = max(1, -(-self.total_rows // self.bundle_rows))
        if self.device.type == "cuda":
            self._build_tables(target_tasks)

    # ---- device tables ----------------------------------------------------------------
    def _build_tables(self, target_tasks: int):
        segs = bytearray()
        tasks: List[Tuple[int, int, int, int]] = []
        slot_begin = [0]
        rows_per_task = max(MIN_ROWS_PER_TASK, -(-self.total_rows // max(1, target_tasks)))
        seg_id = 0
        keys = []  # (partition, first row) of every task: equal keys read identical rows
        for slot, m in enumerate(self.messages):
            for p, coef in m:
                X, y = self.partitions[p]
                n = X.shape[0]
                segs += _SEG.pack(X.data_ptr(), y.data_ptr(), float(coef), n)
                for r0 in range(0, n, rows_per_task):
                    tasks.append((slot, seg_id, r0, min(n, r0 + rows_per_task), len(tasks)))
                    keys.append((p, r0))
                seg_id += 1
            slot_begin.append(len(tasks))
        if self.bundle_rows:
            tasks, folded_begin = self._bundle_table(tasks, keys)
            if folded_begin is not None:  # one slab row per (workgroup, replica): see _fold_table
                slot_begin = folded_begin
        elif self.interleave and self.cpl is not None:
            tasks = [tasks[i] for i in replica_dispatch_order(keys)]
        dev = self.device
        self.segs = torch.tensor(list(bytes(segs) or b"\0" * 32), dtype=torch.uint8).to(dev)
        self.ntasks = len(tasks)
        t = np.asarray(tasks, dtype=np.int32).reshape(-1, 5)
        self.tasks = torch.from_numpy(t).to(dev)
        self.slot_task_begin = torch.tensor(slot_begin, dtype=torch.int32, device=dev)
        self.slab = torch.empty((max(1, self.ntasks), self.ld), dtype=self.prec.acc, device=dev)
        # partial sums [nslots, SLAB_SPLITS, ld], then 16 zeroed bytes: the staged kernels' persistent-grid
        # ticket (csrc/kernels/launchers.h slab_part_bytes)
        es = torch.tensor([], dtype=self.prec.acc).element_size()
        self.part = torch.zeros(max(1, self.nslots) * SLAB_SPLITS * self.ld + 16 // es, dtype=self.prec.acc, device=dev)
        if self.cpl is None:
            off = np.zeros(max(1, self.ntasks), dtype=np.int64)
            if self.ntasks:
                off[1:] = np.cumsum(t[:, 3] - t[:, 2])[:-1]
            if off.size and off[-1] + (t[-1, 3] - t[-1, 2] if self.ntasks else 0) >= 2 ** 31:
                raise ValueError("two-pass plan exceeds int32 row offsets")
            self.task_row_off = torch.from_numpy(off.astype(np.int32)).to(dev)
            self.rbuf = torch.empty(max(1, int(self.total_rows)), dtype=self.prec.acc, device=dev)

    def _bundle_table(self, tasks, keys):
        """Replica-bundle layout for grad_dense_bundle: R task slots per workgroup, one wave each."""
        bundles: Dict[Tuple[int, int], List[int]] = {}
        for i, k in enumerate(keys):
            bundles.setdefault(k, []).append(i)
        groups: List[List[int]] = []
        for b in bundles.values():
            groups += [b[i:i + MAX_BUNDLE] for i in range(0, len(b), MAX_BUNDLE)]
        R = max(len(g) for g in groups)
        pad = (0, -1, 0, 0, 0)
        table = []
        for g in groups:
            table += [tasks[i] for i in g] + [pad] * (R - len(g))
        if self.mfma and R > 16:
            raise ValueError("MFMA bundles hold at most 16 replicas")
        if self.multi and R > 3:
            raise ValueError("one-wave bundles (ERASUREHEAD_STAGED=multi) hold at most 3 replicas")
        self.fold = self.multi and os.environ.get("ERASUREHEAD_MULTI_FOLD", "1") != "0"
        # epilogue of the folded one-wave kernel: replicas 0/1 reduce-scattered and one lane per
        # replica evaluating its residual (csrc variant 90 + R) wins on sharded ranks (N=2/4/8
        # 0.677-0.684 / 0.353-0.354 / 0.188-0.190 vs 0.689-0.699 / 0.365-0.368 / 0.194-0.197 ms);
        # the wave-uniform one (70 + R) on the one-GPU headline (1.316-1.334 vs 1.40-1.43 ms),
        # profiles/r3_epi.  ERASUREHEAD_MULTI_EPI=wave|lane overrides.
        epi = os.environ.get("ERASUREHEAD_MULTI_EPI", "")
        distinct = sum(self.partitions[p][0].shape[0] for p in {p for m in self.messages for p, _ in m})
        self.lane_epi = self.fold and (epi == "lane" or (epi == "" and distinct < 750_000))
        self.variant = (40 if self.mfma else (90 if self.lane_epi else 70 if self.fold else 60) if self.multi
                        else 30 if self.staged_pair else 20 if self.staged else 10) + R
        if self.staged and self.staged_wpr:
            self.variant += 100 * self.staged_wpr  # csrc: variant / 100 % 10 = waves per replica
        # persistent staged workgroups (csrc: variant >= 1000): as many workgroups as fit, each taking
        # bundles from an atomic ticket until none is left; ERASUREHEAD_PERSISTENT=1 (read per plan)
        self.persistent = bool(self.staged and os.environ.get("ERASUREHEAD_PERSISTENT", "0") == "1")
        if self.persistent:
            self.variant += 1000
        if self.fold:
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
                             self.slot_task_begin, self.part, G, self.ld, self.variant)
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
                                        self.slot_task_begin, self.part, self.ld, variant=self.variant)
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
    """

    def __init__(self, messages: Sequence[Sequence[Tuple[int, float]]], partitions: Dict[int, Tuple[object, np.ndarray]],
                 prec: Precision, loss: int, d: int, device="cpu", use_ell: bool = True):
        import scipy.sparse as sps

        if prec.name == "bf16":
            raise ValueError("sparse data uses fp64 or fp32 values (bf16 has no benefit for one-hot data)")
        self.prec, self.loss, self.d = prec, loss, d
        self.ld = prec.ld(d)
        self.messages = [list(m) for m in messages]
        self.nslots = len(self.messages)
        self.device = torch.device(device)
        blocks, ys, coefs, slots = [], [], [], []
        for slot, m in enumerate(self.messages):
            for p, coef in m:
                A, y = partitions[p]
                A = sps.csr_matrix(A)
                if A.shape[1] > d:
                    raise ValueError("partition has more columns than d")
                blocks.append(A)
                ys.append(np.asarray(y, dtype=np.float64))
                coefs.append(np.full(A.shape[0], float(coef)))
                slots.append(np.full(A.shape[0], slot, dtype=np.int64))
        X = sps.vstack(blocks, format="csr") if blocks else sps.csr_matrix((0, d))
        X = sps.csr_matrix((X.data, X.indices, X.indptr), shape=(X.shape[0], d))
        X.sort_indices()
        self.nrows = X.shape[0]
        self.nnz = X.nnz
        row_slot = np.concatenate(slots) if slots else np.zeros(0, dtype=np.int64)
        self.pattern_only = bool(X.nnz == 0 or np.all(X.data == 1.0))
        # COO sorted by key = slot * ld + col (the CSC twin across all local messages)
        coo = X.tocoo()
        keys = row_slot[coo.row] * self.ld + coo.col.astype(np.int64)
        order = np.argsort(keys, kind="stable")
        acc = prec.acc
        npacc = np.float64 if acc == torch.float64 else np.float32
        dev = self.device
        self.row_ptr = torch.from_numpy(X.indptr.astype(np.int64)).to(dev)
        self.col_idx = torch.from_numpy(X.indices.astype(np.int32)).to(dev)
        self.vals = None if self.pattern_only else torch.from_numpy(X.data.astype(npacc)).to(dev)
        self.y = torch.from_numpy((np.concatenate(ys) if ys else np.zeros(0)).astype(npacc)).to(dev)
        self.coef = torch.from_numpy((np.concatenate(coefs) if coefs else np.zeros(0)).astype(npacc)).to(dev)
        self.keys = torch.from_numpy(keys[order]).to(dev)
        self.rows = torch.from_numpy(coo.row[order].astype(np.int32)).to(dev)
        self.cvals = None if self.pattern_only else torch.from_numpy(coo.data[order].astype(npacc)).to(dev)
        self.rbuf = torch.empty(max(1, self.nrows), dtype=acc, device=dev)
        self._row_slot = torch.from_numpy(row_slot).to(dev)
        self._X_cpu = X if dev.type == "cpu" else None
        self.ell = False
        if dev.type == "cuda" and use_ell:
            self._build_ell(X, row_slot, npacc, slots)

    ELL_CHUNK = 4096  # rows per column-pass block

    def _build_ell(self, X, row_slot, npacc, slots):
        """Column-major ELL twin when every row has the same nnz (one-hot data)."""
        nnz_row = np.diff(X.indptr)
        if self.nrows == 0 or not np.all(nnz_row == nnz_row[0]) or nnz_row[0] == 0 or self.nrows >= 2 ** 31:
            return
        m = int(nnz_row[0])
        idx = X.indices.reshape(self.nrows, m).T  # [m, nrows]; rows are sorted -> k-th smallest column
        lo = idx.min(axis=1).astype(np.int32)
        width = (idx.max(axis=1) - lo + 1).astype(np.int32)
        chunks = []
        r = 0
        for slot in range(self.nslots):
            n = int(np.sum(row_slot == slot))
            for r0 in range(r, r + n, self.ELL_CHUNK):
                chunks.append((r0, min(r + n, r0 + self.ELL_CHUNK), slot, 0))
            r += n
        dev = self.device
        self.ell = True
        self.ell_m = m
        self.ell_idx = torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int32)).to(dev)
        self.ell_vals = None if self.pattern_only else torch.from_numpy(
            np.ascontiguousarray(X.data.reshape(self.nrows, m).T, dtype=npacc)).to(dev)
        self.ell_lo = torch.from_numpy(lo).to(dev)
        self.ell_width = torch.from_numpy(width).to(dev)
        self.ell_max_width = int(width.max())
        self.ell_chunks = torch.from_numpy(np.asarray(chunks, dtype=np.int32).reshape(-1, 4)).to(dev)

    def out_buffer(self, n: int = 1) -> torch.Tensor:
        return torch.zeros((n, self.nslots, self.ld), dtype=self.prec.acc, device=self.device)

    def native_launcher(self):
        if self.device.type != "cuda":
            raise RuntimeError("native launchers need GPU tensors")
        if self.ell:
            return native().GradLauncher.ell(self.loss, self.ell_idx, self.ell_vals, self.y, self.coef, self.rbuf,
                                             self.ell_chunks, self.ell_lo, self.ell_width, self.ell_max_width,
                                             self.nslots, self.ld)
        return native().GradLauncher.sparse(self.loss, self.row_ptr, self.col_idx, self.vals, self.y, self.coef,
                                            self.rbuf, self.keys, self.rows, self.cvals, self.nslots, self.ld)

    def run(self, beta: torch.Tensor, G: torch.Tensor) -> torch.Tensor:
        if G.shape != (self.nslots, self.ld):
            raise ValueError(f"G must be [{self.nslots}, {self.ld}]")
        if self.device.type == "cuda" and self.ell:
            native().grad_ell(self.loss, self.ell_idx, self.ell_vals, self.y, self.coef, beta, self.rbuf,
                              self.ell_chunks, self.ell_lo, self.ell_width, self.ell_max_width, G, self.ld)
            return G
        if self.device.type == "cuda":
            native().grad_sparse(self.loss, self.row_ptr, self.col_idx, self.vals, self.y, self.coef, beta,
                                 self.rbuf, self.keys, self.rows, self.cvals, G, self.ld)
            return G
        X = self._X_cpu
        b = beta.detach().cpu().double().numpy()[: self.d]
        z = X.dot(b)
        y = self.y.double().numpy()
        c = self.coef.double().numpy()
        if self.loss == LOGISTIC:
            r = -(c * y) * (1.0 / (1.0 + np.exp(np.clip(y * z, -700, 700))))
        else:
            r = -2.0 * c * (y - z)
        G.zero_()
        rs = self._row_slot.numpy()
        for slot in range(self.nslots):
            sel = rs == slot
            g = X[sel].T.dot(r[sel]) if sel.any() else np.zeros(self.d)
            G[slot, : self.d] = torch.from_numpy(np.asarray(g).ravel()).to(G.dtype)
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
