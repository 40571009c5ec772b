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
    assert [multi_bundle_rows(n) for n in (1_000_000, 500_000, 250_000, 125_000)] == [768, 256, 128, 64]
    assert multi_bundle_rows(1_000_000, fp32=True) == 384 and multi_bundle_rows(1000) == 64
