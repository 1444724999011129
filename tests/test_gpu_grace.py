"""Grace hash join (HBM -> pinned host spill) vs the answer derived from the probe table."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _world():
    from dryad_amd.parallel.comm import World
    return World(0, 1, 0, torch.device("cuda", 0), None)


@pytest.mark.parametrize("budget,prune", [(None, False), (1 << 25, False), (1 << 20, False),   # in HBM / hybrid /
                                          (1 << 23, True), (1 << 18, True)])                 # all spilled
def test_grace_join_matches_expected(budget, prune):
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    cfg = HashJoinConfig(rows_r=300_000, rows_s=450_000, chunk_rows=100_000, hbm_budget=budget, prune=prune)
    job = HashJoinJob(_world(), cfg)
    res = job.step()
    assert res == job.expected()
    assert res[0] == 450_000
    total = (300_000 + 450_000) * (16 if prune else 64)
    if budget is None:
        assert job.last["in_hbm"] and job.last["spilled_bytes"] == 0
    elif budget in (1 << 25, 1 << 23):
        assert not job.last["in_hbm"] and 0 < job.last["spilled_bytes"] < total and job.last["buckets"] > 1
    else:
        assert job.last["spilled_bytes"] == total
    assert job.step() == res        # buffers re-created / released across steps


def test_sort_merge_join_pairs_many_to_many():
    from dryad_amd.ops import grace as G
    l = torch.zeros((6, 16), dtype=torch.uint8, device="cuda")
    r = torch.zeros((5, 16), dtype=torch.uint8, device="cuda")
    lk = [3, 1, 3, 7, 9, 1]
    rk = [1, 3, 3, 8, 1]
    for i, k in enumerate(lk):
        l[i, 0] = k
    for i, k in enumerate(rk):
        r[i, 0] = k
    oo, ii = G.sort_merge_join_pairs(l, r, 0, 8)
    got = sorted(zip(oo.tolist(), ii.tolist()))
    exp = sorted((a, b) for a in range(6) for b in range(5) if lk[a] == rk[b])
    assert got == exp


@pytest.mark.parametrize("ncols,dim", [(8, False), (8, True), (3, True), (5, False)])
def test_records64_rows_generator_matches_numpy_twin(ncols, dim):
    import numpy as np
    from dryad_amd.models.records_cpu import dim_multiplier, gen_columns
    from dryad_amd.ops import relational as R
    nkeys = 1_000_003 if dim else 977
    dm = dim_multiplier(nkeys) if dim else 0
    n = 20_011
    first = 500_000 if dim else 123
    rows = torch.empty((n, ncols), dtype=torch.int64, device="cuda")
    R.gen_records64_rows(rows, first, nkeys, 11, dm)
    ref = gen_columns(first, n, nkeys, 11, ncols=ncols, dim_mult=dm)
    for j in range(ncols):
        np.testing.assert_array_equal(rows[:, j].cpu().numpy(), ref[j])


@pytest.mark.parametrize("ncols,dim,n,skew", [(4, False, 20_011, 0), (1, False, 4096, 0), (8, False, 777, 1),
                                              (3, True, 5_003, 0), (5, False, 1, 0)])
def test_records64_columns_generator_matches_numpy_twin(ncols, dim, n, skew):
    """dr_gen_records64 (column stores: two rows per lane with 16-byte stores, the one-row path for
    columns that are not 16-byte aligned (``skew``) and odd counts) against the numpy twin."""
    import numpy as np
    from dryad_amd.models.records_cpu import dim_multiplier, gen_columns
    from dryad_amd.ops import relational as R
    nkeys = 1_000_003 if dim else 977
    dm = dim_multiplier(nkeys) if dim else 0
    first = 500_000 if dim else 123
    base = [torch.full((n + skew,), -7, dtype=torch.int64, device="cuda") for _ in range(ncols)]
    cols = [b[skew:] for b in base]
    R.gen_records64(cols, first, nkeys, 11, dm)
    ref = gen_columns(first, n, nkeys, 11, ncols=ncols, dim_mult=dm)
    for j in range(ncols):
        np.testing.assert_array_equal(cols[j].cpu().numpy(), ref[j])
        if skew:
            assert int(base[j][0]) == -7


def _rows(keys, stride=64, key_len=8):
    n = len(keys)
    r = torch.zeros((n, stride // 8), dtype=torch.int64)
    r[:, 0] = torch.tensor(keys, dtype=torch.int64)
    r[:, 1] = torch.arange(n, dtype=torch.int64) * 3 + 1
    return r.view(torch.uint8).reshape(n, stride).cuda()


def test_partition_rows_buckets_and_contiguous_tail():
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed(5)
    keys = torch.randint(0, 5000, (70_000,), generator=g).tolist()
    rows = _rows(keys)
    nb, cf, cap = 13, 9, 8000
    part = G.Partitioner(nb, rows.device)
    store = torch.zeros((cf * cap, 64), dtype=torch.uint8, device="cuda")
    tail = torch.zeros((70_000, 64), dtype=torch.uint8, device="cuda")
    part.ptrs.copy_(torch.tensor([store.data_ptr()] * cf + [tail.data_ptr()] * (nb - cf), dtype=torch.int64))
    part.fill.copy_(torch.tensor([b * cap for b in range(nb)], dtype=torch.int64))
    part.cap.copy_(torch.tensor([(b + 1) * cap for b in range(nb)], dtype=torch.int64))
    # two chunks: fills advance across calls, the tail restarts at row 0
    G.partition_rows(rows[:30_000], 0, 8, part, contig_from=cf)
    c1 = part.counts.tolist()
    G.partition_rows(rows[30_000:], 0, 8, part, contig_from=cf)
    c2 = part.counts.tolist()
    assert sum(c1) == 30_000 and sum(c2) == 40_000 and int(part.overflow.item()) == 0
    fill = part.fill.tolist()
    seen = {}
    for b in range(cf):
        got = store[b * cap: fill[b]].view(torch.int64).reshape(-1, 8)
        assert got.shape[0] == c1[b] + c2[b]
        for k, v in zip(got[:, 0].tolist(), got[:, 1].tolist()):
            seen.setdefault(k, set()).add(b)
            assert keys[(v - 1) // 3] == k
        # stable: row order within a bucket follows input order
        idx = ((got[:, 1] - 1) // 3).tolist()
        assert idx == sorted(idx)
    off = 0
    for b in range(cf, nb):
        got = tail[off: off + c2[b]].view(torch.int64).reshape(-1, 8)
        for k in got[:, 0].tolist():
            seen.setdefault(k, set()).add(b)
        off += c2[b]
    assert all(len(v) == 1 for v in seen.values())          # a key lives in exactly one bucket


def test_partition_overflow_is_flagged_not_written_past_cap():
    from dryad_amd.ops import grace as G
    rows = _rows([7] * 5000)                                  # every row hashes to one bucket
    part = G.Partitioner(4, rows.device)
    store = torch.zeros((4 * 1000 + 1, 64), dtype=torch.uint8, device="cuda")
    store[-1] = 0xAB
    part.ptrs.fill_(store.data_ptr())
    part.fill.copy_(torch.tensor([0, 1000, 2000, 3000], dtype=torch.int64))
    part.cap.copy_(torch.tensor([1000, 2000, 3000, 4000], dtype=torch.int64))
    G.partition_rows(rows, 0, 8, part)
    assert int(part.overflow.item()) == 1
    assert int(store[-1].min().item()) == 0xAB


@pytest.mark.parametrize("key_len", [8, 4, 12])
def test_hash_join_pairs_many_to_many(key_len):
    from collections import defaultdict
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed(9)
    # key = (field 0, low 4 bytes of field 1); field 0 also differs above bit 32 so a 4-byte key
    # merges keys that an 8-byte one separates
    bk = [(a + (b << 33), c) for a, b, c in zip(*(torch.randint(0, m, (4000,), generator=g).tolist()
                                                   for m in (300, 2, 3)))]
    pk = [(a + (b << 33), c) for a, b, c in zip(*(torch.randint(0, m, (5000,), generator=g).tolist()
                                                   for m in (400, 2, 3)))]

    def rows(keys):
        r = torch.zeros((len(keys), 8), dtype=torch.int64)
        r[:, 0] = torch.tensor([k for k, _ in keys])
        r[:, 1] = torch.tensor([c for _, c in keys])
        return r.view(torch.uint8).reshape(len(keys), 64).cuda()

    def norm(k):
        if key_len == 4:
            return k[0] & 0xFFFFFFFF
        return k[0] if key_len == 8 else k
    po, bo = G.hash_join_pairs(rows(bk), rows(pk), 0, key_len)
    got = sorted(zip(po.tolist(), bo.tolist()))
    idx = defaultdict(list)
    for j, k in enumerate(bk):
        idx[norm(k)].append(j)
    exp = sorted((i, j) for i, k in enumerate(pk) for j in idx.get(norm(k), []))
    assert got == exp
    assert po.tolist() == sorted(po.tolist())                # grouped by probe row, probe order


def test_join_sum_fused_aggregate():
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed(3)
    bk = torch.randperm(50_000, generator=g)[:30_000].tolist()
    pk = torch.randint(0, 60_000, (80_000,), generator=g).tolist()
    b, p = _rows(bk), _rows(pk)
    lc = G.ht_log_cap(len(bk))
    table = torch.empty((1 << lc) * 2, dtype=torch.int64, device="cuda")
    acc = torch.zeros(3, dtype=torch.int64, device="cuda")
    G.join_sum(b, p, 0, 8, 8, 8, acc, table, lc)
    pos = {k: j for j, k in enumerate(bk)}
    m = [(i, pos[k]) for i, k in enumerate(pk) if k in pos]
    assert acc.tolist() == [len(m), sum(3 * i + 1 for i, _ in m), sum(3 * j + 1 for _, j in m)]


@pytest.mark.parametrize("proj", [(0, 16), (8, 16), (4, 8)])
def test_partition_rows_projection(proj):
    """Column pruning in the partition pass: destination rows are bytes [po, po + ow) of the rows,
    bucketed exactly like the whole rows."""
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed(11)
    keys = torch.randint(0, 9000, (50_000,), generator=g).tolist()
    rows = _rows(keys)
    po, ow = proj
    nb = 7
    whole, pruned = G.Partitioner(nb, rows.device), G.Partitioner(nb, rows.device)
    a = torch.zeros((50_000, 64), dtype=torch.uint8, device="cuda")
    b = torch.zeros((50_000, ow), dtype=torch.uint8, device="cuda")
    whole.ptrs.fill_(a.data_ptr())
    pruned.ptrs.fill_(b.data_ptr())
    G.partition_rows(rows, 0, 8, whole, contig_from=0)
    G.partition_rows(rows, 0, 8, pruned, contig_from=0, proj=proj)
    assert whole.counts.tolist() == pruned.counts.tolist()
    assert torch.equal(a[:, po:po + ow], b)


@pytest.mark.parametrize("prune", [True, False])
def test_hash_join_job_pruned_columns(prune):
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    from dryad_amd.parallel.comm import World
    w = World(0, 1, 0, torch.device("cuda", 0), None)
    job = HashJoinJob(w, HashJoinConfig(rows_r=300_000, rows_s=500_000, chunk_rows=100_000, prune=prune))
    res = job.step()
    assert res == job.expected() and res[0] == 500_000
    job.release()


def _kv_rows(keys, vals):
    r = torch.stack([torch.tensor(keys, dtype=torch.int64), torch.tensor(vals, dtype=torch.int64)], 1)
    return r.view(torch.uint8).reshape(len(keys), 16).cuda()


@pytest.mark.parametrize("case", ["unique", "dups", "skew"])
def test_radix_join_sum_matches_global_table(case):
    """LDS radix join over segmented (gapped) stores == the global-table join_sum, including
    many-to-many keys, a key run too large for the LDS table and the empty-slot sentinel key."""
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed({"unique": 1, "dups": 2, "skew": 3}[case])
    nb_, np_ = 400_000, 600_000
    if case == "unique":
        bk = torch.randperm(2_000_000, generator=g)[:nb_]
    else:
        bk = torch.randint(0, 150_000, (nb_,), generator=g)
    pk = torch.randint(0, 2_000_000 if case == "unique" else 150_000, (np_,), generator=g)
    if case == "skew":
        bk[:9000] = 77                 # one key's build run > the LDS table
        pk[:50] = 77
        bk[9000] = -1                  # the LDS table's empty-slot sentinel as a real key
        pk[50:53] = -1
    bv = torch.randint(0, 1 << 40, (nb_,), generator=g)
    pv = torch.randint(0, 1 << 40, (np_,), generator=g)
    b, p = _kv_rows(bk.tolist(), bv.tolist()), _kv_rows(pk.tolist(), pv.tolist())
    lc = G.ht_log_cap(nb_)
    table = torch.empty((1 << lc) * 2, dtype=torch.int64, device="cuda")
    ref = torch.zeros(3, dtype=torch.int64, device="cuda")
    G.join_sum(b, p, 0, 8, 8, 8, ref, table, lc)
    # the same rows as 3 gapped segments per side, bucketed like the grace pass would not need to be
    # (any split works: partitions only have to agree between the sides through the hash digits)
    def segmented(rows, cuts, gap=1000):
        n = rows.shape[0]
        out = torch.zeros((n + gap * len(cuts), 16), dtype=torch.uint8, device="cuda")
        begins, lens, at, prev = [], [], 0, 0
        for c in list(cuts) + [n]:
            out[at:at + c - prev] = rows[prev:c]
            begins.append(at)
            lens.append(c - prev)
            at += c - prev + gap
            prev = c
        return out, (torch.tensor(begins, device="cuda"), torch.tensor(lens, device="cuda"))
    # segments must hold every occurrence of a key on one side (like grace buckets): split by key hash
    hb = (torch.tensor(bk.tolist()) * 0x9E3779B97F4A7C15) >> 62 & 3
    hp = (torch.tensor(pk.tolist()) * 0x9E3779B97F4A7C15) >> 62 & 3
    ob, op = torch.argsort(hb, stable=True), torch.argsort(hp, stable=True)
    cb = torch.bincount(hb, minlength=4).cumsum(0)[:-1].tolist()
    cp = torch.bincount(hp, minlength=4).cumsum(0)[:-1].tolist()
    bs, bseg = segmented(b[ob.cuda()], cb)
    ps, pseg = segmented(p[op.cuda()], cp)
    scratch = torch.empty((max(bs.shape[0], ps.shape[0]), 16), dtype=torch.uint8, device="cuda")
    acc = torch.zeros(3, dtype=torch.int64, device="cuda")
    n_ovf = G.radix_join_sum(bs, bseg, ps, pseg, 0, 8, 8, 8, acc, scratch)
    assert acc.tolist() == ref.tolist()
    assert (n_ovf > 0) == (case == "skew")


@pytest.mark.parametrize("radix", [True, False])
def test_hash_join_job_radix(radix):
    from dryad_amd.models.hashjoin import HashJoinConfig, HashJoinJob
    job = HashJoinJob(_world(), HashJoinConfig(rows_r=700_000, rows_s=900_000, chunk_rows=300_000, radix=radix))
    res = job.step()
    assert res == job.expected() and res[0] == 900_000
    assert job.step() == res
    job.release()


def test_partition_rows_unordered_matches_ordered_as_multisets():
    from dryad_amd.ops import grace as G
    g = torch.Generator().manual_seed(21)
    keys = torch.randint(0, 7000, (90_000,), generator=g).tolist()
    rows = _rows(keys)
    nb, cap = 9, 20_000
    outs = []
    for unordered in (False, True):
        part = G.Partitioner(nb, rows.device)
        store = torch.zeros((nb * cap, 16), dtype=torch.uint8, device="cuda")
        part.ptrs.fill_(store.data_ptr())
        part.fill.copy_(torch.tensor([b * cap for b in range(nb)], dtype=torch.int64))
        part.cap.copy_(torch.tensor([(b + 1) * cap for b in range(nb)], dtype=torch.int64))
        G.partition_rows(rows[:40_000], 0, 8, part, proj=(0, 16), unordered=unordered)
        G.partition_rows(rows[40_000:], 0, 8, part, proj=(0, 16), unordered=unordered)
        fill = part.fill.tolist()
        assert int(part.overflow.item()) == 0
        outs.append([sorted(map(tuple, store[b * cap: fill[b]].view(torch.int64).reshape(-1, 2).tolist()))
                     for b in range(nb)])
    assert outs[0] == outs[1]
