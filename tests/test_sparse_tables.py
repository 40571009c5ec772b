"""Host tables of the deterministic sparse column pass (ops/grad.py SparseGradPlan.csc_tables), checked
by a NumPy emulation of csrc/kernels/grad_sparse.hip (csc_tiles + csc_spans): every column of every
partition is written exactly once -- inside one tile by the lane holding its last entry, across tiles
as tail + heads in tile order, or 0 when empty -- and the result is X_p^T u_p."""
import numpy as np
import pytest
import scipy.sparse as sps

from erasurehead_amd.ops.grad import SparseGradPlan

TILE = 512


def rows_and_flags(t):
    """CSC row indices and their run-start flags (the top bit)."""
    if t["row16"]:
        raw = t["crow"].view(np.uint16).astype(np.int64)
        return raw & 0x7FFF, raw >> 15
    raw = t["crow"].view(np.uint32).astype(np.int64)
    return raw & 0x7FFFFFFF, raw >> 31


def tile_keys(t, ti, flag):
    """The keyed column pass's columns of tile ti (grad_sparse.hip csc_tiles_lds): the run list read at
    the wave prefix of the run-start flags."""
    r0, packed, p, c0 = (int(x) for x in t["tkeys"][ti])
    n, nruns, flags = packed & 1023, (packed >> 10) & 1023, packed >> 20
    f = flag[TILE * ti:TILE * ti + TILE]
    assert f[0] == 1 and int(f[:n].sum()) == nruns and not f[n:].any()
    ridx = np.cumsum(f) - 1
    keys = t["runs"][r0 + ridx].astype(np.int64)
    assert keys[0] == c0
    return keys[:n], n, p, c0, flags


def emulate(t, u_parts, d, keyed=False):
    nparts = len(u_parts)
    G = np.full((nparts, d), np.nan)
    head, tail = {}, {}
    crow, flag = rows_and_flags(t)
    for ti, (p, base, c0, flags) in enumerate(t["tiles"]):
        cp = t["col_ptr"][p].astype(np.int64)
        nnz = int(t["part_nnz"][p])
        cut = bool(t.get("wg_spans"))  # column-aligned chunks: a tile's entry count is tkeys' n
        n = int(t["tkeys"][ti][1]) & 1023 if cut else min(TILE, nnz - base)
        e0 = TILE * ti if cut else int(t["part_entry0"][p]) + base
        assert e0 % 8 == 0
        cnt = np.zeros(TILE, dtype=np.int64)
        c = c0 + 1
        while c <= d and cp[c] < base + n:  # the wave's boundary walk
            cnt[cp[c] - base] += 1
            c += 1
        keys = c0 + np.cumsum(cnt)[:n]
        assert keys[0] == c0 and np.all(cp[keys] <= base + np.arange(n)) and np.all(base + np.arange(n) < cp[keys + 1])
        assert e0 == TILE * ti  # the kernels address tile ti's entries directly
        if keyed:
            k2, n2, p2, c02, f2 = tile_keys(t, ti, flag)
            assert (n2, p2, c02, f2) == (n, p, c0, flags)
            np.testing.assert_array_equal(k2, keys)
            keys = k2
        v = u_parts[p][crow[e0:e0 + n]] * t["cvals"][e0:e0 + n]
        start = 0
        for q in range(n):
            if q != n - 1 and keys[q + 1] == keys[q]:
                continue
            val = 0.0
            for x in v[start:q + 1]:
                val += x
            key = int(keys[q])
            has_head = key == c0 and bool(flags & 1)
            has_tail = q == n - 1 and bool(flags & 2)
            if has_head:
                head[ti] = val
            if has_tail:
                tail[ti] = val
            if not has_head and not has_tail:
                assert np.isnan(G[p, key]), "column written twice"
                G[p, key] = val
            start = q + 1
    for p, c, t1, t2 in t["span"]:
        assert np.isnan(G[p, c])
        G[p, c] = tail[t1] + sum(head[t] for t in range(t1 + 1, t2 + 1))
    if t.get("wg_spans"):  # each workgroup's own crossing columns, chunk-relative tiles (from LDS)
        assert len(t["span"]) == 0 and len(t["wspan_ptr"]) == len(t["wg"]) + 1
        for k, (_, t0, nt, _) in enumerate(t["wg"]):
            for p, c, t1, t2 in t["wspan"][t["wspan_ptr"][k]:t["wspan_ptr"][k + 1]]:
                assert np.isnan(G[p, c]) and 0 <= t1 < t2 < nt
                G[p, c] = tail[t0 + t1] + sum(head[t0 + t] for t in range(t1 + 1, t2 + 1))
    for p, c in t["empty"]:
        assert np.isnan(G[p, c])
        G[p, c] = 0.0
    assert not np.any(np.isnan(G)), "a column was never written"
    return G


def _onehot(rng, n, windows):
    cols, lo = [], 0
    for w in windows:
        p = rng.dirichlet(np.ones(w) * 0.3)
        cols.append(lo + rng.choice(w, n, p=p))
        lo += w
    cols = np.stack(cols, axis=1)
    return sps.csr_matrix((np.ones(cols.size), cols.ravel(), np.arange(0, cols.size + 1, len(windows))), shape=(n, lo))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_tables_emulate_to_the_transposed_product(seed):
    rng = np.random.RandomState(seed)
    d = 3000
    blocks = [
        _onehot(rng, 2000, [2, 40, 700, 1200]),       # a binary feature: columns span many tiles
        _onehot(rng, 333, [1, 900, 5, 1000]),          # partition smaller than a tile, empty columns
        sps.random(900, d - 1, density=0.01, format="csr", random_state=rng),  # valued, ragged rows
        sps.csr_matrix((70000, 2948)),                 # no entries at all (and > 65536 rows)
    ]
    blocks = [sps.csr_matrix((b.data, b.indices, b.indptr), shape=(b.shape[0], d)) for b in blocks]
    t = SparseGradPlan.csc_tables(blocks, d, TILE)
    assert not t["row16"]  # one partition has more than 65536 rows
    u = [rng.randn(b.shape[0]) for b in blocks]
    got = emulate(t, u, d, keyed=True)
    for p, b in enumerate(blocks):
        np.testing.assert_allclose(got[p], b.T.dot(u[p]), rtol=1e-12, atol=1e-12)
    assert len(t["span"]) > 0 and len(t["empty"]) > 0


def test_sixteen_bit_rows_and_tile_alignment():
    rng = np.random.RandomState(5)
    blocks = [_onehot(rng, 1500, [3, 50, 400]), _onehot(rng, 700, [3, 50, 400])]
    d = blocks[0].shape[1]
    t = SparseGradPlan.csc_tables(blocks, d, TILE)
    assert t["row16"] and t["crow"].dtype == np.int16
    assert all(e % TILE == 0 for e in t["part_entry0"])
    u = [rng.randn(b.shape[0]) for b in blocks]
    got = emulate(t, u, d, keyed=True)
    for p, b in enumerate(blocks):
        np.testing.assert_allclose(got[p], b.T.dot(u[p]), rtol=1e-12, atol=1e-12)


def test_cpu_plan_matches_scipy_per_message():
    """The CPU plan (the reference's arithmetic) with replicas sharing partitions."""
    import torch

    from erasurehead_amd.models.losses import LOGISTIC, logistic_grad
    from erasurehead_amd.ops import get_precision

    rng = np.random.RandomState(3)
    parts = {p: (_onehot(rng, 300, [2, 30, 60]), rng.choice([-1.0, 1.0], 300)) for p in range(3)}
    d = parts[0][0].shape[1]
    msgs = [[(0, 1.0), (1, 1.0)], [(1, 0.5), (2, -1.0)], [(0, 2.0)]]
    prec = get_precision("fp64")
    plan = SparseGradPlan(msgs, parts, prec, LOGISTIC, d)
    assert plan.basis == [0, 1, 2] and plan.nrows == 900 and plan.msg_rows == 1500
    b = rng.randn(d) * 0.1
    beta = torch.zeros(plan.ld, dtype=torch.float64)
    beta[:d] = torch.from_numpy(b)
    G = plan.out_buffer()[0]
    plan.run(beta, G)
    for s, m in enumerate(msgs):
        ref = sum(logistic_grad(parts[p][0], parts[p][1], b, c) for p, c in m)
        np.testing.assert_allclose(G[s, :d].numpy(), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("row_block,wg_spans", [(64, False), (700, False), (4096, False), (64, True), (700, True),
                                                (4096, True)])
def test_row_blocked_tables_sum_to_the_transposed_product(row_block, wg_spans):
    """Row-blocked tables (SparseGradPlan.csc_tables(row_block=...)): every partition cut into
    sub-blocks of at most row_block rows; the emulated sub-block sums, added per partition in
    sub-block order (grad_sparse.hip sub_reduce), are X_p^T u_p; the workgroup table covers every
    tile of every sub-block exactly once, never mixing sub-blocks.  wg_spans: chunks end on column
    boundaries and every crossing column is summed inside its workgroup."""
    rng = np.random.RandomState(7)
    d = 2500
    blocks = [_onehot(rng, 1800, [2, 40, 700, 1200]), _onehot(rng, 333, [1, 900, 5, 1000]),
              sps.csr_matrix((0, 2403))]
    blocks = [sps.csr_matrix((b.data, b.indices, b.indptr), shape=(b.shape[0], d)) for b in blocks]
    t = SparseGradPlan.csc_tables(blocks, d, TILE, row_block=row_block, wg_tiles=16, wg_spans=wg_spans)
    assert t["wg_spans"] == wg_spans
    if wg_spans and row_block > 512:  # (64-row sub-blocks fit one tile each)
        assert len(t["wspan"]) > 0
    sb = t["sub_begin"]
    assert len(sb) == len(blocks) + 1 and sb[-1] == t["nsub"]
    u = [rng.randn(b.shape[0]) for b in blocks]
    u_sub = []
    for j, b in enumerate(blocks):
        for r in range(0, max(b.shape[0], 1), row_block):
            u_sub.append(u[j][r:r + row_block])
    assert len(u_sub) == t["nsub"]
    got = emulate(t, u_sub, d, keyed=True)
    seen = []
    for row0, t0, nt, rows in t["wg"]:
        s = int(t["tiles"][t0][0])
        assert row0 == t["part_row0"][s] and 1 <= nt <= 16 and rows == len(u_sub[s])
        assert all(t["tiles"][k][0] == s for k in range(t0, t0 + nt))
        seen += list(range(t0, t0 + nt))
    assert sorted(seen) == list(range(len(t["tiles"])))
    for j, b in enumerate(blocks):
        acc = np.zeros(d)
        for s in range(sb[j], sb[j + 1]):
            acc = acc + got[s]
        np.testing.assert_allclose(acc, b.T.dot(u[j]), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("slots", [4, 16, 512])
def test_chip_sized_chunks(slots):
    """csc_tables(slots=...): balanced column-aligned chunks, at most `slots` workgroups when the tiles are
    many (and at least one per sub-block), chunks of about 16 tiles when they are few; every chunk at most
    wg_tiles tiles; the emulated sums still give X_p^T u_p."""
    rng = np.random.RandomState(11)
    d = 2500
    blocks = [_onehot(rng, 3000, [2, 40, 700, 1200]), _onehot(rng, 2500, [1, 900, 5, 1000])]
    blocks = [sps.csr_matrix((b.data, b.indices, b.indptr), shape=(b.shape[0], d)) for b in blocks]
    t = SparseGradPlan.csc_tables(blocks, d, TILE, row_block=1000, wg_tiles=128, wg_spans=True, slots=slots)
    assert t["wg_spans"]
    nsub = t["nsub"]
    ntiles = len(t["tiles"])
    assert len(t["wg"]) <= max(slots, nsub) and all(1 <= nt <= 128 for _, _, nt, _ in t["wg"])
    if slots >= 512:  # few tiles for the chip: chunks of about 16
        assert len(t["wg"]) >= ntiles // 17
    u = [rng.randn(b.shape[0]) for b in blocks]
    u_sub = [u[j][r:r + 1000] for j, b in enumerate(blocks) for r in range(0, b.shape[0], 1000)]
    got = emulate(t, u_sub, d, keyed=True)
    sb = t["sub_begin"]
    for j, b in enumerate(blocks):
        acc = np.zeros(d)
        for s_ in range(sb[j], sb[j + 1]):
            acc = acc + got[s_]
        np.testing.assert_allclose(acc, b.T.dot(u[j]), rtol=1e-12, atol=1e-12)
