"""Device forms of the whole-partition aggregates (reduce.hip), the hash join and GroupJoin
(hashjoin.hip), keys wider than one sort entry (Rabin-64 fingerprints, verified byte for byte),
Zip / SelectMany / SlidingWindow and the keyed Fork: kernels against torch / Python references,
queries against the LocalDebug oracle, with checks that the ops stayed on the device."""
from collections import defaultdict

import pytest
import torch

import dryad_amd as D

pytestmark = pytest.mark.gpu


def _ctx(parts=1):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = parts
    return c


def _local():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _fallbacks(c):
    return c._get_executor().last_result["fallbacks"]


def _same(build, ordered=False, parts=1, device_ops=()):
    c = _ctx(parts)
    a = list(build(_local()))
    b = list(build(c))
    if ordered:
        assert a == b
    else:
        assert sorted(a, key=repr) == sorted(b, key=repr)
    fb = {op for _, op, _ in _fallbacks(c)}
    for op in device_ops:
        assert op not in fb, f"{op} fell back to the host: {_fallbacks(c)}"


INTS = [(i * 7919) % 100_003 - 50_000 for i in range(60_000)]
PAIRS = [(i % 101, float(i % 997) / 3) for i in range(50_000)]
BIG = 1 << 40


@pytest.mark.parametrize("n", [1, 777, 1 << 20, 3_000_001])
def test_reduce_kernel_matches_torch(n):
    from dryad_amd.ops import reduce as RD
    torch.manual_seed(n)
    a = torch.randint(-10**12, 10**12, (n,), dtype=torch.int64, device="cuda")
    f = torch.randn(n, dtype=torch.float64, device="cuda")
    m = (a % 3) == 0
    i32 = (a % 100_000).to(torch.int32)
    f32 = f.to(torch.float32)
    got = RD.reduce_multi(n, [(RD.SUM, a, None), (RD.MIN, f, None), (RD.MAX, i32, m), (RD.COUNT, None, m),
                              (RD.FIRST, None, m), (RD.LAST, None, m), (RD.SUM, f32, None), (RD.MAX, m, None),
                              (RD.SUM, f, m)], "cuda")
    idx = torch.nonzero(m).flatten().tolist()
    scale = max(1.0, float(f.abs().sum()))
    assert got[0] == int(a.sum())
    assert got[1] == float(f.min())
    assert got[2] == (int(i32[m].max()) if idx else -2**63)
    assert got[3] == len(idx)
    assert got[4] == (idx[0] if idx else None)
    assert got[5] == (idx[-1] if idx else None)
    assert abs(got[6] - float(f32.double().sum())) <= 1e-9 * scale
    assert got[7] == (1 if idx else 0)
    assert abs(got[8] - float(f[m].sum())) <= 1e-9 * scale


@pytest.mark.parametrize("parts", [1, 3])
def test_aggregates_on_device_match_localdebug(parts):
    cases = {
        "Count": lambda c: c.FromEnumerable(INTS).Count(lambda x: x % 7 == 0),
        "LongCount": lambda c: c.FromEnumerable(INTS).LongCount(),
        "Sum": lambda c: c.FromEnumerable(INTS).Sum(),
        "SumSelector": lambda c: c.FromEnumerable(PAIRS).Sum(lambda p: p[0] * 3),
        "Min": lambda c: c.FromEnumerable(INTS).Min(),
        "Max": lambda c: c.FromEnumerable(PAIRS).Max(lambda p: p[1]),
        "Average": lambda c: c.FromEnumerable(INTS).Average(),
        "Any": lambda c: c.FromEnumerable(INTS).Any(lambda x: x == INTS[12345]),
        "All": lambda c: c.FromEnumerable(INTS).All(lambda x: x > -60_000),
        "Contains": lambda c: c.FromEnumerable(INTS).Contains(INTS[4321]),
        "First": lambda c: c.FromEnumerable(PAIRS).First(lambda p: p[1] > 300),
        "Last": lambda c: c.FromEnumerable(INTS).Last(lambda x: x % 1000 == 1),
        "LastOrDefault": lambda c: c.FromEnumerable(INTS).LastOrDefault(lambda x: x > 10**9),
        "Single": lambda c: c.FromEnumerable(INTS).Single(lambda x: x == INTS[999]),
        "SumAsQuery": lambda c: list(c.FromEnumerable(PAIRS).SumAsQuery(lambda p: p[1]))[0],
    }
    for name, q in cases.items():
        c = _ctx(parts)
        exp, got = q(_local()), q(c)
        if isinstance(exp, float):
            assert got == pytest.approx(exp, rel=1e-12), name
        else:
            assert got == exp, name
        bad = [f for f in _fallbacks(c) if f[1].startswith("agg")]
        assert not bad, (name, bad)


@pytest.mark.parametrize("parts", [1, 3])
def test_user_aggregate_sum_fold_on_device(parts):
    """Aggregate(seed, func) whose step is acc + f(x), or a bitwise acc ^ / | / & f(x), folds on
    the device (one reduction);
    any other step still runs on the host and gives the oracle's answer."""
    cases = {
        "seed": (lambda c: c.FromEnumerable(INTS).Aggregate(5, lambda a, x: a + x * 3 - 1), True),
        "term_first": (lambda c: c.FromEnumerable(INTS).Aggregate(0, lambda a, x: (x % 11) + a), True),
        "minus": (lambda c: c.FromEnumerable(INTS).Aggregate(100, lambda a, x: a - x), True),
        "tuple_result": (lambda c: c.FromEnumerable(PAIRS).Aggregate(
            0.5, lambda a, p: a + p[1] * 2, lambda a: round(a, 6)), True),
        "seedless": (lambda c: c.FromEnumerable(INTS).Aggregate(lambda a, x: a + x), True),
        "bool_term": (lambda c: c.FromEnumerable(INTS).Aggregate(0, lambda a, x: a + (x > 0)), True),
        "xor": (lambda c: c.FromEnumerable(INTS).Aggregate(12345, lambda a, x: a ^ (x * 2654435761)), True),
        "or_term_first": (lambda c: c.FromEnumerable(INTS).Aggregate(0, lambda a, x: (x & 0xFF0) | a), True),
        "and_seedless": (lambda c: c.FromEnumerable(INTS).Aggregate(lambda a, x: a & (x | 1)), True),
        "mixed_host": (lambda c: c.FromEnumerable(INTS).Aggregate(0, lambda a, x: (a ^ x) + 1), False),
        "product_host": (lambda c: c.FromEnumerable(INTS[:50]).Aggregate(1, lambda a, x: a * (x % 3 + 1)), False),
        "max_host": (lambda c: c.FromEnumerable(INTS).Aggregate(0, lambda a, x: a if a > x else x), False),
    }
    for name, (q, on_device) in cases.items():
        c = _ctx(parts)
        exp, got = q(_local()), q(c)
        if isinstance(exp, float):
            assert got == pytest.approx(exp, rel=1e-9), name
        else:
            assert got == exp, name
        fb = {f[1] for f in _fallbacks(c)}
        assert ("aggregate_seq" not in fb) == on_device, (name, _fallbacks(c))


def test_hash_join_pairs_match_python_join():
    from dryad_amd.ops import relational as R
    torch.manual_seed(0)
    ko = torch.randint(0, 5000, (200_000,), device="cuda", dtype=torch.int64)
    ki = torch.randint(0, 5000, (30_000,), device="cuda", dtype=torch.int64)
    eo, _, lm = R.build_keys([ko])
    ei, _, _ = R.build_keys([ki])
    oo, ii, cnt = R.hash_join_pairs(eo, ei, lm)
    pos = defaultdict(list)
    for j, k in enumerate(ki.tolist()):
        pos[k].append(j)
    exp = [(o, j) for o, k in enumerate(ko.tolist()) for j in pos.get(k, ())]
    assert list(zip(oo.tolist(), ii.tolist())) == exp
    assert cnt.tolist() == [len(pos.get(k, ())) for k in ko.tolist()]
    # 96-bit composite keys (key material in the lo word) and inner keys that never match
    a = torch.randint(0, 40, (50_000,), device="cuda", dtype=torch.int64)
    b = torch.randint(0, 40, (50_000,), device="cuda", dtype=torch.int32)
    eo, _, lm = R.build_keys([a, b])
    ei, _, _ = R.build_keys([a[:700].clone() + 1000, b[:700].clone()])
    oo, _, _ = R.hash_join_pairs(eo, ei, lm)
    assert oo.numel() == 0
    ei, _, _ = R.build_keys([a[:700].clone(), b[:700].clone()])
    oo, ii, _ = R.hash_join_pairs(eo, ei, lm)
    ref = defaultdict(list)
    for j, kk in enumerate(zip(a[:700].tolist(), b[:700].tolist())):
        ref[kk].append(j)
    exp = [(o, j) for o, kk in enumerate(zip(a.tolist(), b.tolist())) for j in ref.get(kk, ())]
    assert list(zip(oo.tolist(), ii.tolist())) == exp


def test_join_and_group_join_keep_linq_order():
    dims = [(k, k * 10) for k in range(0, 101, 2)]
    _same(lambda c: c.FromEnumerable(PAIRS[:20_000]).Join(c.FromEnumerable(dims), lambda p: p[0], lambda d: d[0],
                                                          lambda p, d: (p[1], d[1])),
          ordered=True, device_ops=("hash_join",))
    customers = [(k, k * 3) for k in range(0, 200, 3)]
    orders = [(i % 150, float(i % 17)) for i in range(20_000)]
    _same(lambda c: c.FromEnumerable(customers).GroupJoin(
        c.FromEnumerable(orders), lambda cu: cu[0], lambda o: o[0],
        lambda cu, g: (cu[0], cu[1] + 1, g.Count(), g.Sum(lambda o: o[1]), g.Any(lambda o: o[1] > 15))),
        ordered=True, device_ops=("hash_group_join",))


def test_wide_keys_on_device():
    recs = [(BIG + i % 37, BIG + (i * 7) % 11, float(i % 5), i) for i in range(20_000)]
    _same(lambda c: c.FromEnumerable(recs).GroupBy(
        lambda r: (r[0], r[1], r[2]), lambda k, g: (k[0], k[1], k[2], g.Count(), g.Sum(lambda r: r[3]))), parts=2,
        device_ops=("group_partial", "group_final", "hash_partition"))
    _same(lambda c: c.FromEnumerable(recs).Select(lambda r: (r[0], r[1], r[2])).Distinct(), parts=2,
          device_ops=("distinct",))
    dims = [(BIG + k, BIG + j, k * 100 + j) for k in range(37) for j in range(11)]
    _same(lambda c: c.FromEnumerable(recs).Join(c.FromEnumerable(dims), lambda r: (r[0], r[1]),
                                                lambda d: (d[0], d[1]), lambda r, d: (r[3], d[2])),
          ordered=True, device_ops=("hash_join",))


def test_zip_selectmany_window_fork_on_device():
    _same(lambda c: c.FromEnumerable(INTS[:5000]).Zip(c.FromEnumerable(PAIRS[:4000]), lambda a, b: (a, b[1] * 2)),
          ordered=True, device_ops=("zip",))
    _same(lambda c: c.FromEnumerable(INTS[:3000]).SelectMany(lambda x: [x, x + 1, x * 2]), ordered=True,
          device_ops=("select_many",))
    _same(lambda c: c.FromEnumerable(PAIRS[:3000]).SelectMany(lambda p: (p[0], p[0] + 7), lambda p, y: (y, p[1])),
          ordered=True, device_ops=("select_many",))
    _same(lambda c: c.FromEnumerable(INTS[:4000]).SlidingWindow(lambda w: w[0] + w[1] * 2 - w[2], 3),
          ordered=True, device_ops=("sliding_window",))
    for parts in (1, 2):
        c, l = _ctx(parts), _local()
        kf = c.FromEnumerable(INTS[:9000]).Fork(lambda x: x % 5, keys=[0, 3, 4])
        kl = l.FromEnumerable(INTS[:9000]).Fork(lambda x: x % 5, keys=[0, 3, 4])
        for k in (0, 3, 4):
            assert sorted(kf[k]) == sorted(kl[k])
            assert "fork" not in {op for _, op, _ in _fallbacks(c)}, _fallbacks(c)


@pytest.mark.parametrize("parts", [1, 2])
def test_fork_tuple_mapper_on_device(parts):
    """Per-record ForkTuple mapper traced once: ports of different record types (scalar, tuple),
    a masked port and an unused slot, each consumed by a further device op."""
    def mapper(p):
        return D.ForkTuple(D.ForkValue(p[0] * 2, True), D.ForkValue((p[0], p[1] + 1.0), p[0] % 3 == 1),
                           D.ForkValue(None, False))
    c, l = _ctx(parts), _local()
    fc, fl = c.FromEnumerable(PAIRS[:20000]).Fork(mapper, per_record=True), \
        l.FromEnumerable(PAIRS[:20000]).Fork(mapper, per_record=True)
    assert sorted(fc.First.Where(lambda x: x > 10)) == sorted(fl.First.Where(lambda x: x > 10))
    assert "fork" not in {op for _, op, _ in _fallbacks(c)}, _fallbacks(c)
    assert sorted(fc.Second.Select(lambda t: (t[0], t[1] * 2))) == sorted(fl.Second.Select(lambda t: (t[0], t[1] * 2)))
    assert "fork" not in {op for _, op, _ in _fallbacks(c)}, _fallbacks(c)
    assert list(fc.Third) == list(fl.Third) == []
    # an untraceable mapper still answers correctly on the host
    hc = c.FromEnumerable(PAIRS[:500]).Fork(lambda p: D.ForkTuple(D.ForkValue(str(p[0]), True)), per_record=True)
    hl = l.FromEnumerable(PAIRS[:500]).Fork(lambda p: D.ForkTuple(D.ForkValue(str(p[0]), True)), per_record=True)
    assert sorted(hc.First) == sorted(hl.First)


@pytest.mark.parametrize("aos", [False, True])
def test_seg_reduce_aos_packing_matches_columns(aos, monkeypatch):
    from dryad_amd.ops import relational as R, sort as S
    monkeypatch.setattr(R, "AOS_MIN_ROWS", 0 if aos else 1 << 62)
    n = 400_003
    k = torch.randint(0, 70_000, (n,), device="cuda", dtype=torch.int64)
    vi = torch.randint(-10**6, 10**6, (n,), device="cuda", dtype=torch.int64)
    vf = torch.randn(n, device="cuda", dtype=torch.float64)
    e, b0, lo_mask = R.build_keys([k])
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    cnt, si, mx, sf = R.seg_reduce_multi(srt, seg, nseg, [("count", None, torch.int64), ("sum", vi, torch.int64),
                                                          ("max", vi, torch.int64), ("sum", vf, torch.float64)])
    uk, inv = torch.unique(k, return_inverse=True)
    assert torch.equal(cnt, torch.bincount(inv, minlength=uk.numel()))
    assert torch.equal(si, torch.zeros_like(uk).index_add_(0, inv, vi))
    assert torch.equal(mx, torch.full_like(uk, -2**62).scatter_reduce(0, inv, vi, "amax"))
    torch.testing.assert_close(sf, torch.zeros(uk.numel(), dtype=torch.float64, device="cuda").index_add_(0, inv, vf))
    # the group keys decoded from the sorted entries equal the gathered key column
    assert torch.equal(srt[:, 1].index_select(0, starts).bitwise_xor_(-(1 << 63)), uk)


@pytest.mark.parametrize("n,span", [(2, 8), (4097, 12), (5000, 1), (3_000_001, 30), (1 << 20, 20)])
def test_payload_sort_groups_match_torch(n, span):
    """E256 payload sort + sequential segmented reduction against a torch fp64/int64 reference."""
    from dryad_amd.ops import relational as R
    torch.manual_seed(n + span)
    key = torch.randint(-(1 << (span - 1)) if span > 1 else 0, 1 << (span - 1) if span > 1 else 2, (n,),
                        dtype=torch.int64, device="cuda")
    a = torch.randint(-10**9, 10**9, (n,), dtype=torch.int64, device="cuda")
    f = torch.randn(n, dtype=torch.float64, device="cuda")
    i32 = (a % 1000).to(torch.int32)
    specs = [("count", None, torch.int64), ("sum", a, torch.int64), ("min", f, torch.float64),
             ("max", f, torch.float64), ("max", i32, torch.int64), ("sum", a, torch.float64),
             ("min", a + 1, torch.int64)]
    assert R.payload_groups(key, specs) is None   # five distinct (column, dtype) payloads
    if n % 2:
        specs = specs[:6]   # four payloads: 40-byte E320 entries
    else:
        specs = specs[:5]   # three payloads: 32-byte E256 entries
    keys, outs = R.payload_groups(key, specs)
    uk, inv = torch.unique(key, sorted=True, return_inverse=True)
    assert torch.equal(keys, uk)
    g = uk.shape[0]
    cnt = torch.bincount(inv, minlength=g)
    s = torch.zeros(g, dtype=torch.int64, device="cuda").index_add_(0, inv, a)
    mn = torch.full((g,), float("inf"), dtype=torch.float64, device="cuda").scatter_reduce(0, inv, f, "amin")
    mx = torch.full((g,), float("-inf"), dtype=torch.float64, device="cuda").scatter_reduce(0, inv, f, "amax")
    mi = torch.full((g,), -2**63, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, i32.to(torch.int64), "amax")
    ref = [cnt, s, mn, mx, mi]
    if len(specs) == 6:
        ref.append(torch.zeros(g, dtype=torch.float64, device="cuda").index_add_(0, inv, a.to(torch.float64)))
    for j, (o, r) in enumerate(zip(outs, ref)):
        if j == 5:
            torch.testing.assert_close(o, r, rtol=1e-12, atol=1e-3)
        else:
            assert torch.equal(o, r)


def test_payload_sort_rejects_wide_key_span():
    from dryad_amd.ops import relational as R
    key = torch.tensor([0, 1 << 40, 5], dtype=torch.int64, device="cuda")
    assert R.payload_groups(key, [("count", None, torch.int64)]) is None


@pytest.mark.parametrize("parts", [1, 3])
def test_groupby_payload_path_matches_localdebug(parts, monkeypatch):
    from dryad_amd.gpu import ops as G
    from dryad_amd.ops import relational as R
    monkeypatch.setattr(R, "PAYLOAD_SORT_MIN_ROWS", 0)
    monkeypatch.setattr(G, "_fused_int64_groups", lambda *a: None)   # (the int64 key would take it first)
    calls = []
    orig = R.payload_groups
    monkeypatch.setattr(R, "payload_groups", lambda *a: calls.append(1) or orig(*a))
    _same(lambda c: c.FromEnumerable(PAIRS).GroupBy(
        lambda p: p[0] * 1000 - 7, lambda k, g: (k, g.Count(), g.Sum(lambda p: p[0]), g.Min(lambda p: p[1]),
                                                 g.Max(lambda p: p[0]), g.Average(lambda p: p[0]))),
        parts=parts, device_ops=("group_partial", "group_final", "group_by"))
    assert calls, "payload path not taken"


@pytest.mark.parametrize("n", [1, 4096, 4097, 1_000_003])
def test_fused_segment_ids_match_flag_scan(n):
    from dryad_amd.ops import relational as R
    from dryad_amd.ops import sort as S
    torch.manual_seed(n)
    k = torch.randint(0, max(2, n // 3), (n,), dtype=torch.int64, device="cuda")
    k2 = torch.randint(0, 3, (n,), dtype=torch.int32, device="cuda")
    e, b0, lm = R.build_keys([k, k2])
    srt = S.sort_entries_hybrid(e, b0)
    ids, nseg, starts = R.segment_ids(srt, lm)
    ref_ids, ref_n, ref_starts = R._ids_from_flags(R.segment_flags(srt, lm))
    assert nseg == ref_n
    assert torch.equal(ids, ref_ids)
    assert torch.equal(starts, ref_starts)


@pytest.mark.parametrize("ncols", [2, 3, 4, 5])
def test_seg_reduce_packed_rows_any_width(ncols, monkeypatch):
    """Packed value rows: 2-3 distinct columns -> 32-byte rows (vector loads), 4 -> 40-byte rows
    (strided loads), 5 -> not packed; every layout against a torch reference."""
    from dryad_amd.ops import relational as R, sort as S
    monkeypatch.setattr(R, "AOS_MIN_ROWS", 0)
    torch.manual_seed(ncols)
    n = 300_007
    k = torch.randint(0, 50_000, (n,), device="cuda", dtype=torch.int64)
    cols = [torch.randint(-10**6, 10**6, (n,), device="cuda", dtype=torch.int64) for _ in range(ncols)]
    e, b0, lo_mask = R.build_keys([k])
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, _ = R.segment_ids(srt, lo_mask)
    ops = ["sum", "min", "max", "sum", "max"]
    specs = [("count", None, torch.int64)] + [(ops[j], c, torch.int64) for j, c in enumerate(cols)] + \
        [("min", cols[0], torch.int64)]
    got = R.seg_reduce_multi(srt, seg, nseg, specs)
    uk, inv = torch.unique(k, return_inverse=True)
    g = uk.numel()
    assert torch.equal(got[0], torch.bincount(inv, minlength=g))
    red = {"sum": lambda c: torch.zeros(g, dtype=torch.int64, device="cuda").index_add_(0, inv, c),
           "min": lambda c: torch.full((g,), 2**62, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, c, "amin"),
           "max": lambda c: torch.full((g,), -2**62, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, c, "amax")}
    for j, c in enumerate(cols):
        assert torch.equal(got[1 + j], red[ops[j]](c)), j
    assert torch.equal(got[-1], red["min"](cols[0]))


@pytest.mark.parametrize("n,span,skew", [(1, 8, False), (513, 4, False), (5000, 1, False), (1_000_003, 30, False),
                                          (2_000_000, 24, True), (300_000, 12, False)])
def test_group_reduce_sorted_fused_ids_match_torch(n, span, skew):
    """GroupBy over int_key_sort entries with segment ids derived in the reduction (no id array):
    keys, Count, int64 Sum/Min, f64 Min/Max/Sum against torch, incl. groups spanning many chunks."""
    from dryad_amd.ops import relational as R
    torch.manual_seed(n * 7 + span)
    lo = -(1 << (span - 1)) if span > 1 else 0
    key = torch.randint(lo, max(lo + 2, 1 << (span - 1)), (n,), dtype=torch.int64, device="cuda")
    if skew:
        key[: n // 3] = 12345                        # one group over ~1300 chunks
    a = torch.randint(-10**9, 10**9, (n,), dtype=torch.int64, device="cuda")
    f = torch.randn(n, dtype=torch.float64, device="cuda")
    specs = [("count", None, torch.int64), ("sum", a, torch.int64), ("min", f, torch.float64),
             ("max", f, torch.float64), ("min", a, torch.int64)]
    srt = R.int_key_sort(key)
    if srt is None:
        pytest.skip("n < 2")
    keys, outs = R.group_reduce_sorted(srt, specs, -(1 << 63))
    uk, inv = torch.unique(key, sorted=True, return_inverse=True)
    assert torch.equal(keys, uk)
    g = uk.shape[0]
    ref = [torch.bincount(inv, minlength=g),
           torch.zeros(g, dtype=torch.int64, device="cuda").index_add_(0, inv, a),
           torch.full((g,), float("inf"), dtype=torch.float64, device="cuda").scatter_reduce(0, inv, f, "amin"),
           torch.full((g,), float("-inf"), dtype=torch.float64, device="cuda").scatter_reduce(0, inv, f, "amax"),
           torch.full((g,), 2**63 - 1, dtype=torch.int64, device="cuda").scatter_reduce(0, inv, a, "amin")]
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
