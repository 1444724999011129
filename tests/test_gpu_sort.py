"""Numerics of the sort/partition/gather HIP kernels vs plain PyTorch/numpy references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _u64(a):
    return a.cpu().numpy().view(np.uint64)


def _ref_order(e, lo_mask=0xFFFFFFFFFFFFFFFF):
    """numpy stable lexsort on (hi, lo & mask): reference permutation."""
    a = _u64(e)
    lo = a[:, 0] & np.uint64(lo_mask)
    hi = a[:, 1]
    return np.lexsort((lo, hi), axis=0)


@pytest.mark.parametrize("n", [1, 7, 2048, 2049, 100_003, 1_000_000])
def test_sort_entries_full_128(n):
    from dryad_amd.ops import sort as S
    g = torch.Generator(device="cuda").manual_seed(n)
    e = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda", generator=g)
    ref = e.cpu().numpy()[_ref_order(e)]
    out = S.sort_entries(e.clone(), 0, 128)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_sort_entries_is_stable_on_key_bits():
    from dryad_amd.ops import sort as S
    n = 300_000
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, 50, (n,), device="cuda")           # few distinct hi keys
    e[:, 0] = torch.arange(n, device="cuda")                        # row index = original order
    out = S.sort_entries(e.clone(), 64, 128).cpu().numpy()
    ref = e.cpu().numpy()[np.argsort(e[:, 1].cpu().numpy(), kind="stable")]
    np.testing.assert_array_equal(out, ref)


def test_partition_pass_starts():
    from dryad_amd.ops import sort as S
    n = 123_457
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, 8, (n,), device="cuda")
    e[:, 0] = torch.arange(n, device="cuda")
    out, starts = S.partition_pass(e, 64)
    h = np.bincount(e[:, 1].cpu().numpy(), minlength=256)
    exp = np.concatenate([[0], np.cumsum(h)])
    np.testing.assert_array_equal(starts.cpu().numpy(), exp)
    ref = e.cpu().numpy()[np.argsort(e[:, 1].cpu().numpy(), kind="stable")]
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("stride,off,klen", [(100, 0, 10), (16, 4, 8), (13, 1, 12), (24, 8, 3)])
def test_extract_keys(stride, off, klen):
    from dryad_amd.ops import sort as S
    n = 5000
    rows = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device="cuda")
    e = S.extract_keys(rows, off, klen, 0).cpu().numpy().view(np.uint64)
    r = rows.cpu().numpy()
    for i in [0, 1, 17, n - 1]:
        key = bytes(r[i, off:off + klen]) + bytes(12 - klen)
        hi = int.from_bytes(key[:8], "big")
        lo = (int.from_bytes(key[8:12], "big") << 32) | i
        assert int(e[i, 1]) == hi and int(e[i, 0]) == lo


def test_gather_rows_entries_and_index():
    from dryad_amd.ops import sort as S
    n, stride = 10_000, 100
    rows = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device="cuda")
    perm = torch.randperm(n, device="cuda")
    ent = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    ent[:, 0] = perm
    out = S.gather_rows(rows, entries=ent)
    assert torch.equal(out, rows[perm])
    rows2 = torch.randint(0, 256, (n, 36), dtype=torch.uint8, device="cuda")
    out2 = S.gather_rows(rows2, index=perm.to(torch.int64))
    assert torch.equal(out2, rows2[perm])


def test_range_dest_matches_searchsorted():
    from dryad_amd.ops import sort as S
    n = 50_000
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, 1000, (n,), device="cuda")
    e[:, 0] = torch.arange(n, device="cuda")
    seps = torch.zeros((7, 2), dtype=torch.int64, device="cuda")
    sv = torch.tensor([100, 200, 200, 450, 600, 800, 999], device="cuda")
    seps[:, 1] = sv
    out = S.range_dest(e.clone(), seps, 0)
    ref = torch.searchsorted(sv, e[:, 1], right=False)   # count of seps strictly below key
    assert torch.equal(out[:, 1], ref)
    assert torch.equal(out[:, 0], e[:, 0])


def test_range_dest_sub_major_numbering():
    from dryad_amd.ops import sort as S
    n = 40_000
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, 800, (n,), device="cuda")
    e[:, 0] = torch.arange(n, device="cuda")
    sv = torch.tensor([100, 200, 300, 400, 500, 600, 700], device="cuda")   # 8 ranges = 2 ranks x 4 subs
    seps = torch.zeros((7, 2), dtype=torch.int64, device="cuda")
    seps[:, 1] = sv
    out = S.range_dest(e.clone(), seps, 0, subs=4, ranks=2)
    g = torch.searchsorted(sv, e[:, 1], right=False)                  # range r * 4 + b
    assert torch.equal(out[:, 1], (g % 4) * 2 + g // 4)
    assert torch.equal(out[:, 0], e[:, 0])


@pytest.mark.parametrize("n,stride,nb", [(1, 100, 8), (5000, 100, 3), (300_001, 100, 128), (3_000_003, 100, 256),
                                         (70_000, 16, 256),
                                         (4097, 36, 17), (100_000, 128, 64), (20_000, 132, 5)])
def test_bucket_scatter_rows_is_a_stable_partition(n, stride, nb):
    from dryad_amd.ops import sort as S
    g = torch.Generator(device="cuda").manual_seed(n + stride)
    rows = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device="cuda", generator=g)
    e = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = torch.randint(0, nb, (n,), device="cuda", generator=g)
    e[:, 0] = torch.arange(n, device="cuda")
    out = torch.empty_like(rows)
    st = S.bucket_scatter_rows(e, rows, out)
    d = e[:, 1].cpu().numpy()
    order = np.argsort(d, kind="stable")
    np.testing.assert_array_equal(out.cpu().numpy(), rows.cpu().numpy()[order])
    h = np.bincount(d, minlength=256)
    np.testing.assert_array_equal(np.array(st), np.concatenate([[0], np.cumsum(h)]))


def test_terasort_generate_and_check():
    from dryad_amd.ops import terasort as TS
    n = 100_000
    a = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    b = torch.empty((2 * n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(a, n, 42)
    TS.generate(b, 0, 42)
    assert torch.equal(a, b[n:])                      # counter-based: slices agree
    r = a[5].cpu().numpy().tobytes()
    assert r[10:12] == b"\x00\x11" and r[96:] == bytes([0xCC, 0xDD, 0xEE, 0xFF])
    assert r[12:44].decode() == format(n + 5, "032X")
    acc = TS.check(a)
    perm = torch.randperm(n, device="cuda")
    acc2 = TS.check(a[perm].contiguous())
    assert acc[0].item() == acc2[0].item()            # order-independent checksum


def test_local_sort_rows_matches_python_sorted():
    from dryad_amd.ops import recordsort as RS, terasort as TS
    n = 200_000
    bufs = RS.SortBuffers.allocate(n, 100, "cuda")
    TS.generate(bufs.rows_in[:n], 0, 7)
    src = bufs.rows_in[:n].cpu().numpy()
    out = RS.distributed_sort_rows(bufs, n, 0, 10).cpu().numpy()
    keys = [bytes(r[:10]) + i.to_bytes(4, "big") for i, r in enumerate(src)]
    order = sorted(range(n), key=lambda i: keys[i])
    np.testing.assert_array_equal(out, src[order])
    acc = TS.check(torch.from_numpy(out).cuda())
    assert acc[1].item() == 0


def test_local_sort_descending():
    from dryad_amd.ops import recordsort as RS
    n = 20_000
    rows = torch.randint(0, 256, (n, 12), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(rows)
    ea = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    eb = torch.empty_like(ea)
    got = RS.local_sort_rows(rows, out, ea, eb, 2, 9, descending=True).cpu().numpy()
    src = rows.cpu().numpy()
    order = sorted(range(n), key=lambda i: (bytes(255 - x for x in src[i, 2:11]), i))
    np.testing.assert_array_equal(got, src[order])


@pytest.mark.parametrize("dup", [False, True])
def test_prefix_sort_with_tie_fixup_matches_full_sort(dup):
    from dryad_amd.ops import sort as S
    n = 400_000
    e = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda")
    if dup:   # long runs of equal 64-bit prefixes force the fallback path
        e[:, 1] = torch.randint(0, 3, (n,), device="cuda")
    else:     # a few short ties
        e[: n // 100, 1] = e[n // 100: 2 * (n // 100), 1]
    e[:, 0] = (e[:, 0] & ~0xFFFFFFFF) | torch.arange(n, device="cuda")
    full = S.sort_entries(e.clone(), 32, 128).cpu().numpy()
    pre = S.sort_entries_prefix(e.clone(), 32).cpu().numpy()
    np.testing.assert_array_equal(pre, full)


def test_gather_rows_matches_index_select():
    from dryad_amd.ops import sort as S
    n = 300_001
    for stride in (100, 64):              # 16-byte vector gather (100) and the dword gather
        rows = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device="cuda")
        perm = torch.randperm(n, device="cuda")
        assert torch.equal(S.gather_rows(rows, index=perm), rows[perm])


def test_sort_entries_matches_reference():
    from dryad_amd.ops import sort as S
    n = 250_003
    e = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda")
    a = S.sort_entries(e.clone(), 0, 128).cpu().numpy()
    np.testing.assert_array_equal(a, e.cpu().numpy()[_ref_order(e)])


@pytest.mark.parametrize("kind", ["uniform", "prefix", "narrow", "dups", "allsame", "small"])
def test_hybrid_sort_matches_full_sort(kind):
    from dryad_amd.ops import sort as S
    n = 3000 if kind == "small" else 600_000
    e = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda")
    if kind == "prefix":      # constant top 20 bits (range-partitioned rank)
        e[:, 1] = (e[:, 1] & ((1 << 44) - 1)) | (0x5A5A5 << 44)
    elif kind == "narrow":    # only 20 varying bits in hi
        e[:, 1] = e[:, 1] & ((1 << 20) - 1)
    elif kind == "dups":      # runs far longer than the LDS window -> fallback path
        e[:, 1] = torch.randint(0, 5, (n,), device="cuda") << 40
    elif kind == "allsame":
        e[:, 1] = 77
    e[:, 0] = (e[:, 0] & ~0xFFFFFFFF) | torch.arange(n, device="cuda")
    for begin in (0, 48, 64, 96):
        full = S.sort_entries(e.clone(), begin, 128).cpu().numpy()
        st = {}
        got = S.sort_entries_hybrid(e.clone(), begin, 128, stats=st).cpu().numpy()
        np.testing.assert_array_equal(got, full, err_msg=f"{kind} begin={begin} {st}")


def test_hybrid_sort_masks_bits_below_begin():
    """Bits below begin_bit are payload: order among equal keys must be input order."""
    from dryad_amd.ops import sort as S
    n = 400_000
    e = torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device="cuda")
    e[:, 1] = e[:, 1] & ((1 << 62) - 1)
    e[: n // 2, 1] = e[n // 2:, 1]          # every key appears twice
    full = S.sort_entries(e.clone(), 64, 128).cpu().numpy()
    got = S.sort_entries_hybrid(e.clone(), 64, 128).cpu().numpy()
    np.testing.assert_array_equal(got, full)


def test_terasort_generate_with_keys_matches_extract():
    from dryad_amd.ops import sort as S, terasort as TS
    n = 100_003
    a = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    keys = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    rng = torch.tensor([-1, 0], dtype=torch.int64, device="cuda")
    TS.generate_with_keys(a, 77, 5, keys, rng)
    TS.generate(b, 77, 5)
    assert torch.equal(a, b)
    ref = S.extract_keys(b, 0, 10, 0)
    assert torch.equal(keys, ref)
    mn, mx = S.hi_range(ref)
    assert [int(x) & (2**64 - 1) for x in rng.cpu().tolist()] == [mn, mx]


@pytest.mark.parametrize("nkeys", [1, 7, 1000, 300_000])
def test_seg_reduce_multi_matches_torch(nkeys):
    from dryad_amd.ops import relational as R, sort as S
    n = 500_003
    k = torch.randint(0, nkeys, (n,), device="cuda", dtype=torch.int64)
    vi = torch.randint(-10**6, 10**6, (n,), device="cuda", dtype=torch.int64)
    vf = torch.randn(n, device="cuda", dtype=torch.float64)
    e, b0, lo_mask = R.build_keys([k])
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    cnt, si, mn, mx, sf, mnf, mxf = R.seg_reduce_multi(srt, seg, nseg, [
        ("count", None, torch.int64), ("sum", vi, torch.int64), ("min", vi, torch.int64), ("max", vi, torch.int64),
        ("sum", vf, torch.float64), ("min", vf, torch.float64), ("max", vf, torch.float64)])
    keys = k.index_select(0, (srt[:, 0] & 0xFFFFFFFF).index_select(0, starts))
    uk, inv = torch.unique(k, return_inverse=True)
    assert torch.equal(keys, uk)
    assert torch.equal(cnt, torch.bincount(inv, minlength=uk.numel()))
    assert torch.equal(si, torch.zeros_like(uk).index_add_(0, inv, vi))
    ref_min = torch.full_like(uk, 2**62).scatter_reduce(0, inv, vi, "amin")
    ref_max = torch.full_like(uk, -2**62).scatter_reduce(0, inv, vi, "amax")
    assert torch.equal(mn, ref_min) and torch.equal(mx, ref_max)
    torch.testing.assert_close(sf, torch.zeros(uk.numel(), dtype=torch.float64, device="cuda").index_add_(0, inv, vf))
    assert torch.equal(mnf, torch.full((uk.numel(),), 1e300, dtype=torch.float64, device="cuda").scatter_reduce(0, inv, vf, "amin"))
    assert torch.equal(mxf, torch.full((uk.numel(),), -1e300, dtype=torch.float64, device="cuda").scatter_reduce(0, inv, vf, "amax"))


def test_seg_reduce_multi_matches_torch():
    from dryad_amd.ops import relational as R
    torch.manual_seed(1)
    for n, nk in ((1, 1), (511, 3), (513, 600), (4097, 2), (1_000_003, 50), (2_000_000, 1_500_000)):
        k = torch.sort(torch.randint(0, nk, (n,), device="cuda"))[0]
        flags = torch.ones(n, dtype=torch.int64, device="cuda")
        flags[1:] = (k[1:] != k[:-1]).long()
        seg = torch.cumsum(flags, 0) - 1
        nseg = int(seg[-1]) + 1
        vi = torch.randint(-10**6, 10**6, (n,), device="cuda")
        vf = torch.randn(n, device="cuda", dtype=torch.float64)
        c, sm, mn, mxf = R.seg_reduce_multi(None, seg, nseg, [("count", None, torch.int64), ("sum", vi, torch.int64),
                                                              ("min", vi, torch.int64), ("max", vf, torch.float64)])
        assert torch.equal(c, torch.bincount(seg, minlength=nseg))
        assert torch.equal(sm, torch.zeros(nseg, dtype=torch.int64, device="cuda").index_add_(0, seg, vi))
        assert torch.equal(mn, torch.full((nseg,), 2**62, device="cuda").scatter_reduce(0, seg, vi, "amin"))
        assert torch.equal(mxf, torch.full((nseg,), -1e300, dtype=torch.float64, device="cuda").scatter_reduce(
            0, seg, vf, "amax"))


@pytest.mark.parametrize("n,split", [(1, True), (5000, False), (300_001, True), (2_000_003, True)])
def test_gen_samples_match_stored_entries(n, split):
    """The sampler over gen://terasort from the generator alone (keys generated at the sampled
    positions) == sampling the stored records' entries."""
    from dryad_amd.ops import recordsort as RS
    from dryad_amd.ops import terasort as TS
    first, seed, rank = 12345, 99, 1
    M64 = (1 << 64) - 1
    mask = M64 if split else TS.LO_KEY_MASK_10
    lo_or = (rank << 32) if split else 0
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    ent = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    TS.generate_with_keys(rows, first, seed, ent)
    ent[:, 0].bitwise_or_(lo_or)
    m, stride = RS.sample_count(n, 1 << 20)
    off = RS.sample_offset(314159, rank, stride)
    ref_s = ent[off: off + stride * m: stride][:m].clone()
    ref_s[:, 0] &= RS._as_i64(mask)
    samp = RS.gen_samples((first, seed), n, rank, lo_or, mask, 1 << 20, 314159, rows.device)
    assert torch.equal(samp, ref_s)


@pytest.mark.parametrize("n,start", [(1, 0), (255, 3), (70_001, 1), (1_300_000, 5)])
def test_extract_keys64_tile_matches_row_extract(n, start):
    """Entries read through LDS tiles (any 4-byte alignment of the first row) == extract_keys64,
    and the fused histograms == the digit counts of the windows."""
    from dryad_amd.ops import sort as S
    from dryad_amd.ops import terasort as TS
    buf = torch.empty((n + start, 100), dtype=torch.uint8, device="cuda")
    TS.generate(buf, 777, 5)
    rows = buf[start:]
    for P in (0, 7, 40):
        ref = S.extract_keys64(rows, 0, 10, P, torch.empty(n, dtype=torch.int64, device="cuda"))
        got, hist = S.extract_keys64_tile(rows, 0, 10, P, torch.empty(n, dtype=torch.int64, device="cuda"), hist=True)
        assert torch.equal(got, ref)
        if hist is not None:
            h = hist.view(-1, 4, 256).sum(0).cpu()
            win = ((ref >> 32) & 0xFFFFFFFF).cpu()
            for p in range(4):
                assert torch.equal(h[p].long(), torch.bincount((win >> (8 * p)) & 0xFF, minlength=256))
    ref = S.extract_keys64(rows, 3, 7, 0, torch.empty(n, dtype=torch.int64, device="cuda"))    # unaligned key
    got, _ = S.extract_keys64_tile(rows, 3, 7, 0, torch.empty(n, dtype=torch.int64, device="cuda"))
    assert torch.equal(got, ref)
