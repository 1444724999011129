"""Radix aggregation kernels (csrc/kernels/grace.hip "Radix aggregation", ops/radixagg.py) against
a plain PyTorch reference of the same GroupBy: torch.unique + index_add / scatter_reduce."""
import pytest
import torch

pytestmark = pytest.mark.gpu

I64 = torch.int64


def _ref(key, specs):
    uniq, inv = torch.unique(key.to(I64), return_inverse=True)
    g = uniq.shape[0]
    outs = []
    for op, v, dt in specs:
        if op == "count":
            outs.append(torch.bincount(inv, minlength=g).to(I64))
            continue
        v = v.to(dt)
        if op == "sum":
            outs.append(torch.zeros(g, dtype=dt, device=v.device).index_add_(0, inv, v))
        else:
            init = (float("inf") if op == "min" else float("-inf")) if dt == torch.float64 else \
                (torch.iinfo(I64).max if op == "min" else torch.iinfo(I64).min)
            outs.append(torch.full((g,), init, dtype=dt, device=v.device).scatter_reduce_(
                0, inv, v, "amin" if op == "min" else "amax", include_self=True))
    return uniq, outs


def _check(key, specs, got, float_tol=None):
    assert got is not None
    keys, outs = got
    rk, routs = _ref(key, specs)
    order = torch.argsort(keys)
    assert torch.equal(keys[order], rk)
    for (op, _, dt), o, r in zip(specs, outs, routs):
        o = o[order]
        if dt == torch.float64 and op == "sum":
            torch.testing.assert_close(o, r, rtol=1e-12, atol=1e-9)
        else:
            assert torch.equal(o, r), op


@pytest.mark.parametrize("n,keys", [(3_000_000, 1 << 30), (3_000_000, 5000), (1_000_000, 300_000)])
def test_radix_aggregate_int(n, keys):
    from dryad_amd.ops import radixagg as RA
    g = torch.Generator(device="cuda").manual_seed(n ^ keys)
    k = torch.randint(0, keys, (n,), device="cuda", generator=g)
    v1 = torch.randint(-2**40, 2**40, (n,), device="cuda", generator=g)
    v2 = torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g)
    v3 = torch.randint(-1000, 1000, (n,), device="cuda", generator=g)
    specs = [("count", None, I64), ("sum", v1, I64), ("min", v2, I64), ("max", v3, I64)]
    _check(k, specs, RA.radix_aggregate(k, specs, force=True))


def test_radix_aggregate_one_value_16_byte_rows_and_narrow_key():
    from dryad_amd.ops import radixagg as RA
    g = torch.Generator(device="cuda").manual_seed(7)
    k = torch.randint(-2**31, 2**31 - 1, (2_000_000,), device="cuda", generator=g, dtype=torch.int32)
    v = torch.randint(-2**50, 2**50, (2_000_000,), device="cuda", generator=g)
    specs = [("sum", v, I64), ("max", v, I64), ("count", None, I64)]
    _check(k, specs, RA.radix_aggregate(k, specs, force=True))


def test_radix_aggregate_few_keys_many_empty_partitions():
    """~10 distinct keys: almost every radix partition, the trailing ones included, is empty
    (ra_agg_kernel's prefetch of an empty partition must stay inside the row buffer)."""
    from dryad_amd.ops import radixagg as RA
    g = torch.Generator(device="cuda").manual_seed(5)
    k = torch.randint(0, 10, (1_000_000,), device="cuda", generator=g) * (1 << 40)
    v = torch.randint(-2**40, 2**40, (1_000_000,), device="cuda", generator=g)
    specs = [("count", None, I64), ("sum", v, I64), ("max", v, I64)]
    _check(k, specs, RA.radix_aggregate(k, specs, force=True))
    _check(k[:1000], [(o, None if x is None else x[:1000], d) for o, x, d in specs],
           RA.radix_aggregate(k[:1000], [(o, None if x is None else x[:1000], d) for o, x, d in specs],
                              force=True))


def test_radix_aggregate_float():
    from dryad_amd.ops import radixagg as RA
    g = torch.Generator(device="cuda").manual_seed(11)
    k = torch.randint(0, 1 << 22, (2_000_000,), device="cuda", generator=g)
    x = torch.randn(2_000_000, device="cuda", dtype=torch.float64, generator=g)
    specs = [("sum", x, torch.float64), ("min", x, torch.float64), ("max", x, torch.float64)]
    _check(k, specs, RA.radix_aggregate(k, specs, force=True))


def test_radix_aggregate_sentinel_key_skew_and_overflow():
    from dryad_amd.ops import radixagg as RA
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 4_000_000
    k = torch.randint(-2**63, 2**63 - 1, (n,), device="cuda", generator=g)
    k[::7] = -2**63                    # the LDS table's empty-slot key: fallback partition
    k[1::3] = 42                       # one heavy key (a third of the rows)
    v = torch.randint(-2**40, 2**40, (n,), device="cuda", generator=g)
    specs = [("count", None, I64), ("sum", v, I64), ("min", v, I64)]
    _check(k, specs, RA.radix_aggregate(k, specs, force=True))
    # far too few partitions for ~2.4M distinct keys: every partition's table fills
    _check(k, specs, RA.radix_aggregate(k, specs, nd_est=1, force=True))


@pytest.mark.parametrize("parts", [1, 2])
def test_group_by_query_uses_radix_path(monkeypatch, parts):
    import dryad_amd as D
    from dryad_amd.ops import radixagg as RA
    monkeypatch.setattr(RA, "MIN_ROWS", 1 << 12)
    calls = []
    orig = RA.radix_aggregate
    monkeypatch.setattr(RA, "radix_aggregate", lambda *a, **kw: calls.append(1) or orig(*a, **kw))
    # keys spread past 2^32 (the "auto" route) in one case, narrow in the other
    data = [((i * 7919 % 50_000) << (33 if parts == 2 else 0), i % 13, -i, i * 3) for i in range(200_000)]

    def q(ctx):
        return ctx.FromEnumerable(data).GroupBy(
            lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                          g.Max(lambda r: r[3])))
    gpu = D.DryadLinqContext(platform="gpu")
    gpu.PartitionCount = parts
    gpu.GroupByAggregation = "radix"              # every large integer key (ops/tuning.py)
    local = D.DryadLinqContext(1)
    local.LocalDebug = True
    assert sorted(q(gpu)) == sorted(q(local))
    assert calls
    assert not gpu._get_executor().last_result["fallbacks"]


def test_auto_route_takes_only_wide_keys(monkeypatch):
    from dryad_amd.ops import radixagg as RA
    from dryad_amd.ops import tuning
    monkeypatch.setattr(RA, "MIN_ROWS", 16)
    narrow = torch.arange(100_000, device="cuda")
    with tuning.scope(groupby_aggregation="auto"):
        assert not RA.wanted(narrow) and RA.wanted(narrow << 40) and RA.wanted(-(narrow << 20))
    with tuning.scope(groupby_aggregation="radix"):
        assert RA.wanted(narrow)
    with tuning.scope(groupby_aggregation="sort"):
        assert not RA.wanted(narrow << 40)
