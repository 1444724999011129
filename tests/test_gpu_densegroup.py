"""Dense-key GroupBy aggregation (csrc/kernels/densegroup.hip) vs a plain torch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(key, specs):
    uk, inv = torch.unique(key.to(torch.int64), return_inverse=True)
    g = uk.shape[0]
    out = {}
    for i, (op, v, _dt) in enumerate(specs):
        if op == "count":
            out[i] = torch.bincount(inv, minlength=g)
        elif op == "sum":
            out[i] = torch.zeros(g, dtype=torch.int64, device=key.device).index_add_(0, inv, v.to(torch.int64))
        else:
            init = torch.full((g,), (1 << 63) - 1 if op == "min" else -(1 << 63), dtype=torch.int64, device=key.device)
            out[i] = init.scatter_reduce_(0, inv, v.to(torch.int64), "amin" if op == "min" else "amax")
    return uk, out


def _check(key, specs):
    from dryad_amd.ops import densegroup as DG
    got = DG.dense_aggregate(key, specs, force=True)
    assert got is not None
    keys, outs = got
    order = torch.argsort(keys.to(torch.int64))
    uk, ref = _reference(key, specs)
    assert torch.equal(keys.to(torch.int64)[order], uk)
    for i in range(len(specs)):
        assert torch.equal(outs[i][order], ref[i]), specs[i][0]


@pytest.mark.parametrize("span_bits,n", [(14, 100_000), (21, 2_000_000), (25, 3_000_000), (32, 1_500_000)])
def test_dense_groupby_matches_torch(span_bits, n):
    g = torch.Generator(device="cuda").manual_seed(span_bits)
    kmin = -(1 << (span_bits - 2)) + 12345
    key = torch.randint(0, 1 << span_bits, (n,), generator=g, device="cuda") + kmin
    a = torch.randint(-1000, 1000, (n,), generator=g, device="cuda")
    b = torch.randint(-(1 << 40), 1 << 40, (n,), generator=g, device="cuda")
    c = torch.randint(0, 7, (n,), generator=g, device="cuda", dtype=torch.int32)
    _check(key, [("count", None, torch.int64), ("sum", a, torch.int64), ("min", b, torch.int64),
                 ("max", c, torch.int32)])
    _check(key, [("sum", b, torch.int64), ("count", None, torch.int64), ("max", b, torch.int64)])


def test_dense_groupby_skewed_and_int32_key():
    """Half the rows on one key (one run gets a huge share), an int32 key column."""
    g = torch.Generator(device="cuda").manual_seed(9)
    n = 2_000_000
    key = torch.randint(0, 1 << 22, (n,), generator=g, device="cuda", dtype=torch.int32)
    key[::2] = 777
    v = torch.randint(0, 1 << 31, (n,), generator=g, device="cuda")
    _check(key, [("sum", v, torch.int64), ("count", None, torch.int64), ("max", v, torch.int64)])


def test_dense_groupby_declines_what_it_cannot_pack():
    from dryad_amd.ops import densegroup as DG
    n = 1 << 16
    small = torch.randint(0, 1000, (n,), device="cuda")              # span below one LDS table
    assert DG.dense_aggregate(small, [("count", None, torch.int64)], force=True) is None
    wide = torch.randint(0, 1 << 40, (n,), device="cuda")            # span past two passes
    assert DG.dense_aggregate(wide, [("count", None, torch.int64)], force=True) is None
    key = torch.randint(0, 1 << 20, (n,), device="cuda")
    f = torch.rand(n, device="cuda", dtype=torch.float64)
    assert DG.dense_aggregate(key, [("sum", f, torch.float64)], force=True) is None
    big = [torch.randint(-(1 << 62), 1 << 62, (n,), device="cuda") for _ in range(2)]
    assert DG.dense_aggregate(key, [("min", big[0], torch.int64), ("max", big[1], torch.int64)], force=True) is None


def test_groupby_query_takes_dense_path():
    """GroupBy over gen://records64 through the GPU executor: generator bounds -> dense path."""
    import dryad_amd as D
    from dryad_amd.ops import densegroup as DG
    calls = []
    orig = DG.dense_aggregate

    def spy(*a, **k):
        r = orig(*a, **k)
        calls.append(r is not None)
        return r

    DG.dense_aggregate = spy
    try:
        n = 3_000_000
        src = f"gen://records64?count={n}&partitions=1&keys={1 << 22}&seed=5"
        c = D.DryadLinqContext(platform="gpu")
        c.PartitionCount = 1
        res = list(c.FromStore(src).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]))))
    finally:
        DG.dense_aggregate = orig
    assert calls and calls[0]
    from dryad_amd.models.records_cpu import gen_columns
    cols = gen_columns(0, n, 1 << 22, 5, ncols=2)
    import numpy as np
    uk, inv = np.unique(cols[0], return_inverse=True)
    cnt = np.bincount(inv)
    s1 = np.bincount(inv, weights=cols[1].astype(np.float64))
    got = sorted(res)
    assert len(got) == len(uk)
    assert [k for k, _, _ in got] == uk.tolist()
    assert [c for _, c, _ in got] == cnt.tolist()
    assert np.array_equal(np.array([s for _, _, s in got], dtype=np.float64), s1)


def test_dense_state_update_matches_torch_scatter():
    """ops/densegroup.dense_state_update (one pass of atomics per row) == the library scatter
    reductions it replaces: occupancy, count, int64 sum of int32 values, min / max of int64 values,
    float64 sum; keys repeat within the batch."""
    from dryad_amd.ops import densegroup as DG
    g = torch.Generator(device="cuda").manual_seed(3)
    n, lo, R = 2_000_003, -5000, 300_000
    key = torch.randint(lo, lo + R, (n,), device="cuda", generator=g)
    v32 = torch.randint(-2**31, 2**31 - 1, (n,), device="cuda", generator=g, dtype=torch.int32)
    v64 = torch.randint(-2**62, 2**62, (n,), device="cuda", generator=g)
    vf = torch.randn(n, device="cuda", generator=g, dtype=torch.float64)
    mk = lambda fill, dt=torch.int64: torch.full((R,), fill, dtype=dt, device="cuda")  # noqa: E731
    cnt, sm, mn, mx, fs = mk(0), mk(0), mk(2**63 - 1), mk(-2**63), mk(0.0, torch.float64)
    seen = torch.zeros(R, dtype=torch.int8, device="cuda")
    specs = [(cnt, "count", None), (sm, "sum", v32), (mn, "min", v64), (mx, "max", v64), (fs, "sum", vf)]
    assert DG.dense_state_ok(specs, key)
    DG.dense_state_update(key, lo, seen, specs)
    idx = key - lo
    assert torch.equal(seen, torch.zeros_like(seen).index_fill_(0, idx, 1))
    assert torch.equal(cnt, mk(0).index_add_(0, idx, torch.ones_like(idx)))
    assert torch.equal(sm, mk(0).index_add_(0, idx, v32.to(torch.int64)))
    assert torch.equal(mn, mk(2**63 - 1).scatter_reduce_(0, idx, v64, "amin"))
    assert torch.equal(mx, mk(-2**63).scatter_reduce_(0, idx, v64, "amax"))
    assert torch.allclose(fs, mk(0.0, torch.float64).index_add_(0, idx, vf), rtol=1e-9, atol=1e-9)
    with pytest.raises(RuntimeError):
        DG.dense_state_update(key[:10] + R, lo, seen, specs)
    # the same accumulators as the columns of one [R, 5] matrix (a key's slots side by side), no
    # occupancy bytes
    mat = torch.zeros((R, 5), dtype=torch.int64, device="cuda")
    mat[:, 2] = 2**63 - 1
    mat[:, 3] = -2**63
    cols = [mat[:, 0], mat[:, 1], mat[:, 2], mat[:, 3], mat.view(torch.float64)[:, 4]]
    aos = [(c, op, v) for c, (_, op, v) in zip(cols, specs)]
    assert DG.dense_state_ok(aos, key, stride=5) and not DG.dense_state_ok(aos, key)
    DG.dense_state_update(key, lo, None, aos, rng=R, stride=5)
    for c, (ref, _, _) in zip(cols, specs):
        assert torch.allclose(c, ref, rtol=1e-9, atol=1e-9) if c.dtype == torch.float64 else torch.equal(c, ref)
