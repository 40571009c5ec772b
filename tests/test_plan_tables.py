"""Host-side layout of the dense gradient plans (no GPU): the folded one-wave bundle table."""
import types

from erasurehead_amd.ops.grad import DenseGradPlan, multi_bundle_rows


def _headline_like(rows_per_part=(5, 5, 3), messages=((0, 1), (0, 1), (0, 1), (2,), (2,))):
    """Tasks in message-major order as DenseGradPlan._build_tables makes them: (slot, seg, r0, r1, slab)."""
    tasks, keys = [], []
    seg = 0
    for slot, parts in enumerate(messages):
        for p in parts:
            for c in range(rows_per_part[p]):
                tasks.append((slot, seg, 64 * c, 64 * c + 64, len(tasks)))
                keys.append((p, 64 * c))
            seg += 1
    bundles = {}
    for i, k in enumerate(keys):
        bundles.setdefault(k, []).append(i)
    return tasks, keys, list(bundles.values()), len(messages)


def test_fold_table_groups_one_partition_per_workgroup():
    tasks, keys, groups, nslots = _headline_like()
    R = max(len(g) for g in groups)
    pad = (0, -1, 0, 0, 0)
    table, slot_begin = DenseGradPlan._fold_table(types.SimpleNamespace(nslots=nslots), groups, tasks, keys, R, pad)
    assert R == 3 and len(table) % (4 * R) == 0
    nb = len(table) // R
    part_of = {t[:4]: keys[i][0] for i, t in enumerate(tasks)}  # (slot, seg, r0, r1) -> partition
    seen = set()
    for w in range(nb // 4):
        lead = table[4 * w * R: 4 * w * R + R]
        assert lead[0][1] >= 0, "a workgroup starts with a real bundle"
        parts = {part_of[t[:4]] for b in range(4) for t in table[(4 * w + b) * R:(4 * w + b + 1) * R] if t[1] >= 0}
        assert len(parts) == 1, f"workgroup {w} mixes partitions {parts}"
        for b in range(4):  # replica slot q is the same message in every bundle of the workgroup
            for q in range(R):
                t = table[(4 * w + b) * R + q]
                if t[1] >= 0:
                    assert t[0] == lead[q][0]
        for q in range(R):
            if lead[q][1] >= 0:
                s = lead[q][4]
                assert slot_begin[lead[q][0]] <= s < slot_begin[lead[q][0] + 1] and s not in seen
                seen.add(s)
    assert seen == set(range(slot_begin[-1]))  # every slab row written exactly once
    # partition 0 and 1 (5 chunks each -> 2 workgroups each), partition 2 (3 chunks -> 1): 5 workgroups;
    # messages 0-2 read partitions 0 and 1 (4 workgroups each), messages 3-4 partition 2 (1 each)
    assert nb // 4 == 5 and [b - a for a, b in zip(slot_begin, slot_begin[1:])] == [4, 4, 4, 1, 1]


def test_multi_bundle_rows_table():
    # every folded workgroup resident at once (profiles/round3/nt_rows)
    assert [multi_bundle_rows(n) for n in (1_000_000, 500_000, 250_000, 125_000)] == [1024, 512, 256, 128]
    assert [multi_bundle_rows(n, fp32=True) for n in (1_000_000, 500_000, 250_000, 125_000)] == [512, 256, 96, 64]
    assert multi_bundle_rows(1000) == 8 and multi_bundle_rows(12_000) == 16 and multi_bundle_rows(4_000_000) == 3968
    # per-partition fold padding pushes a bundle length up until the workgroups fit the slots
    assert multi_bundle_rows(260_000) == 256 and multi_bundle_rows(260_000, part_rows=[2600] * 100) == 384
    assert multi_bundle_rows(260_000, part_rows=[100] * 2600) == 256  # can never fit: the plain length


def test_kernel_selection_table():
    """choose_kernel (ops/grad.py): every default reachable without environment variables, one row
    per regime (precision x replication x rows per CU x row width)."""
    from erasurehead_amd.ops.grad import KernelChoice, choose_cpl, choose_kernel

    def pick(prec, d, rep, rows):
        vec = {0: 2, 1: 4, 2: 8}[prec]
        ld = -(-d // vec) * vec
        return choose_kernel(prec, ld, choose_cpl(ld, vec), rep, rows)

    # the headline (AGC W=8 s=2: bundles of 3 replicas), one GPU (1e6 distinct rows): long stream
    assert pick(0, 1000, 3, 1_000_000) == KernelChoice("multi", replicas=3, bundle_rows=1024, fold=True, lane_epi=True)
    # (fp32 replica bundles sized like fp64: one folded workgroup per CU, profiles/round5/shapes/fp32_rows_*)
    assert pick(1, 1000, 3, 1_000_000) == KernelChoice("multi", replicas=3, bundle_rows=1024, fold=True, lane_epi=True)
    assert pick(2, 1000, 3, 1_000_000) == KernelChoice("mfma", replicas=3, bundle_rows=4096)
    # bf16 MFMA bundles: every workgroup (one per CU) in the first dispatch round
    assert [pick(2, 1000, 3, n).bundle_rows for n in (500_000, 250_000, 125_000, 10_000)] == [2048, 1024, 512, 256]
    # the 8-GPU partition-shard rank (125k rows): fill every wave slot, lane epilogue
    assert pick(0, 1000, 3, 125_000) == KernelChoice("multi", replicas=3, bundle_rows=128, fold=True, lane_epi=True)
    assert pick(1, 1000, 3, 125_000) == KernelChoice("multi", replicas=3, bundle_rows=128, fold=True, lane_epi=True)
    assert pick(1, 1000, 3, 500_000).bundle_rows == 512 and pick(1, 1000, 3, 250_000).bundle_rows == 256
    # FRC s=1 (bundles of 2): one-wave bundles too, one GPU / a sharded rank
    assert pick(0, 1000, 2, 1_000_000) == KernelChoice("multi", replicas=2, bundle_rows=1024, fold=True, lane_epi=True)
    assert pick(0, 1000, 2, 250_000) == KernelChoice("multi", replicas=2, bundle_rows=256, fold=True, lane_epi=True)
    # more than 3 co-located replicas: LDS-staged bundles
    assert pick(0, 1000, 4, 1_000_000) == KernelChoice("staged", replicas=4, bundle_rows=512, pair=True)
    assert pick(1, 1000, 4, 1_000_000) == KernelChoice("staged", replicas=4, bundle_rows=512, pair=True)
    assert pick(0, 1000, 4, 250_000) == KernelChoice("staged", replicas=4, bundle_rows=128, pair=True, wpr=1)
    # more co-located replicas than task slots per workgroup (a cyclic W = 9 table on one rank): bundles of 8
    assert pick(0, 1000, 9, 1_000_000).replicas == 8 and pick(2, 1000, 9, 1_000_000).replicas == 8
    # distinct rows (naive): one-wave bundles of one replica (fp32 sized like fp64, bf16 with the 12 / 8 per CU rule)
    assert [pick(p, 1000, 1, 1_000_000) for p in (0, 1, 2)] == [
        KernelChoice("multi", replicas=1, bundle_rows=1024, fold=True),
        KernelChoice("multi", replicas=1, bundle_rows=1024, fold=True),
        KernelChoice("multi", replicas=1, bundle_rows=512, fold=True)]
    assert pick(1, 1000, 1, 250_000).bundle_rows == 256
    assert pick(0, 256, 1, 1_000_000) == KernelChoice("fused", rows=2)  # narrow distinct rows: fused
    # d = 2048: fp64 replicas on 256-thread wide-row bundles, fp32 on LDS-staged bundles (pair form,
    # 1024 rows in the long stream); 4096 takes the wide kernel
    assert pick(0, 2048, 3, 1_000_000) == KernelChoice("wide", replicas=3, bundle_rows=1968)
    assert pick(1, 2048, 3, 1_000_000) == KernelChoice("staged", replicas=3, bundle_rows=1024, pair=True)
    assert pick(0, 2048, 3, 100_000) == KernelChoice("wide", replicas=3, bundle_rows=208)
    assert pick(1, 2048, 3, 100_000) == KernelChoice("wide", replicas=3, bundle_rows=112)  # quarter-width rows
    # fp64 full-width replica rows run 512-thread workgroups, one resident per CU (wide_slots_per_cu)
    assert pick(0, 4096, 3, 1_000_000) == KernelChoice("wide", replicas=3, bundle_rows=3920)
    assert pick(1, 4096, 2, 100_000) == KernelChoice("wide", replicas=2, bundle_rows=208)
    assert pick(0, 8192, 3, 1_000_000) == KernelChoice("wide", interleave=True)  # 512-thread rows: no bundles
    # narrow rows: one-wave bundles with two rows per reduce-scatter, ~16 bundles per CU
    assert pick(0, 256, 3, 1_000_000) == KernelChoice("multi", replicas=3, bundle_rows=256, fold=True, pair=True)
    assert pick(1, 256, 3, 1_000_000) == KernelChoice("multi", replicas=3, bundle_rows=64, fold=True, pair=True)
    assert pick(1, 256, 3, 100_000).bundle_rows == 8
    assert pick(0, 512, 3, 1_000_000).pair and pick(1, 512, 3, 1_000_000).pair  # cpl 8
    assert pick(1, 512, 3, 1_000_000).bundle_rows == 256
    assert pick(0, 256, 3, 100_000).bundle_rows == 32 and pick(0, 256, 3, 4_000_000).bundle_rows == 512
    assert not pick(1, 1000, 3, 1_000_000).pair  # cpl 16: four row buffers would not fit
    assert pick(0, 4096, 1, 1_000_000) == KernelChoice("wide")
    assert pick(0, 10000, 3, 100_000) == KernelChoice("twopass")
    # bf16 beyond the MFMA tile: the fused kernel, replica-interleaved
    assert pick(2, 2000, 3, 1_000_000) == KernelChoice("fused", rows=1, interleave=True)
    # the regime boundary is a rows-per-CU rule, not a row count: 4x the CUs -> 4x the rows
    assert pick(0, 1000, 4, 700_000).wpr == 1 and pick(0, 1000, 4, 800_000).wpr == 0
    assert choose_kernel(0, 1000, 16, 4, 2_800_000, n_cus=1024).wpr == 1
    # fp32 replica bundles of 16 columns per lane: 4 per CU like fp64 at every size; narrower fp32 rows keep
    # the 12-per-CU sizing below the long-stream regime, 8 in it
    assert pick(1, 1000, 3, 700_000).bundle_rows == 768 and pick(1, 1000, 3, 800_000).bundle_rows == 896


def test_no_tuning_env_knobs_left():
    """The kernel selection reads no environment variable (round-2 verdict: 28 knobs -> <= 10, all of
    them runtime policy, test hooks or build plumbing)."""
    import glob
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    knobs = set()
    for pat in ("erasurehead_amd/**/*.py", "csrc/**/*.cpp", "csrc/**/*.hip", "csrc/**/*.h", "bench.py"):
        for f in glob.glob(os.path.join(root, pat), recursive=True):
            knobs |= set(re.findall(r"ERASUREHEAD_[A-Z0-9_]+", open(f).read()))
    assert len(knobs) <= 10, sorted(knobs)
    assert not any(k.startswith(("ERASUREHEAD_STAGE", "ERASUREHEAD_MULTI", "ERASUREHEAD_BUNDLE", "ERASUREHEAD_MFMA",
                                 "ERASUREHEAD_PERSISTENT", "ERASUREHEAD_GRAD")) for k in knobs), sorted(knobs)


def test_fill_splits_fill_every_workgroup_slot():
    """fill_splits (ops/grad.py): exactly `wgs` folded workgroups, bundle lengths within one row."""
    import numpy as np

    from erasurehead_amd.ops.grad import fill_splits

    for parts, wgs in (({0: 125_000}, 256), ({p: 125_000 for p in range(8)}, 256), ({0: 125_000, 1: 125_000, 2: 125_000}, 256),
                       ({0: 1000, 1: 300_000, 2: 7}, 512)):
        s = fill_splits(parts, wgs)
        assert sum(-(-(len(b) - 1) // 4) for b in s.values()) == wgs
        for p, b in s.items():
            d = np.diff(b)
            assert b[0] == 0 and b[-1] == parts[p] and d.min() >= 1 and d.max() - d.min() <= 1
    assert fill_splits({p: 10 for p in range(300)}, 256) is None
