"""Fine-bucket exchange of the multi-rank TeraSort (csrc/kernels/tsmerge.hip, ops/recordsort.py
pack_gen_fine / merge_received_rounds) against numpy references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from dryad_amd.ops import recordsort as RS  # noqa: E402
from dryad_amd.ops import sort as S  # noqa: E402
from dryad_amd.ops import terasort as TS  # noqa: E402


def test_gen_entries64_match_generated_rows():
    n, first, seed = 300_000, 12345, 77
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(rows, first, seed)
    e = torch.empty(n, dtype=torch.int64, device="cuda")
    TS.gen_entries64(e, first, seed, hist=False)
    r = rows[:, :4].cpu().numpy().astype(np.uint64)
    win = (r[:, 0] << 24) | (r[:, 1] << 16) | (r[:, 2] << 8) | r[:, 3]
    got = e.cpu().numpy().view(np.uint64)
    assert np.array_equal(got >> np.uint64(32), win)
    assert np.array_equal(got & np.uint64(0xFFFFFFFF), np.arange(n, dtype=np.uint64))


@pytest.mark.parametrize("fb", [16, 24])
@pytest.mark.parametrize("n,skew", [(200_000, 0), (200_003, 0), (1, 0), (7, 1), (100_001, 1)])
def test_fine_starts(fb, n, skew):
    """Bucket starts of window-sorted entries; four entries per lane with 16-byte loads, or 8-byte
    loads when the entries are not 16-byte aligned (``skew``: a slice one entry in)."""
    g = np.random.default_rng(fb + n)
    win = np.sort(g.integers(0, 1 << 32, size=n, dtype=np.uint64))
    win[:min(n, 5000)] = win[min(n - 1, 5000)]   # a long run of one bucket
    full = torch.from_numpy(((win << np.uint64(32)) | np.arange(n, dtype=np.uint64)).view(np.int64)).cuda()
    e = full
    if skew:
        e = torch.cat([full[:1], full]).contiguous()[1:]
    starts = TS.fine_starts(e, fb).cpu().numpy().astype(np.int64)
    b = (win >> np.uint64(32 - fb)).astype(np.int64)
    exp = np.searchsorted(b, np.arange((1 << fb) + 1), side="left")
    assert np.array_equal(starts, exp)


def test_gen_gather64_in_entry_order():
    n, first, seed = 50_000, 999, 5
    perm = torch.randperm(n, device="cuda").to(torch.int64)
    ent = (perm << 32) | perm            # any window; the low word is the record offset
    out = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    TS.gen_gather64(out, ent, first, seed)
    ref = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(ref, first, seed)
    assert torch.equal(out, ref[perm])


def test_tile_merge_orders_buckets_and_flags_overflow():
    g = np.random.default_rng(3)
    W, K, fb = 3, 40, 24
    cnt = g.integers(0, 120, size=(W, K)).astype(np.int32)
    cnt[1, 7] = 1100                              # a bucket past one workgroup's capacity
    cnt[:, 11] = [300, 300, 300]                  # past the LDS stage: the register-path kernel
    cnt[:, 13] = [300, 300, 136]                  # exactly the LDS stage (736 rows)
    cnt[:, 17] = [0, 1024, 0]                     # exactly the capacity, one source
    total = int(cnt.sum())
    rows = g.integers(0, 256, size=(total, 100), dtype=np.uint8)
    # rows of bucket k share their top fb key bits: bucket id in the first 24 bits, random below
    src_bucket = np.concatenate([np.repeat(np.arange(K), cnt[s]) for s in range(W)])
    hi = (src_bucket.astype(np.uint64) + np.uint64(1000)) << np.uint64(64 - fb)
    hi |= g.integers(0, 1 << (64 - fb), size=total, dtype=np.uint64) & np.uint64((1 << (64 - fb)) - 1)
    hi[::7] &= ~np.uint64(0xFFFF)                  # some equal prefixes: ties resolved by bytes 8..9
    rows[:, :8] = hi.astype(">u8").view(np.uint8).reshape(total, 8)
    rows[::11, 8:10] = 0                           # and some equal full keys: stable by (source, slot)
    pre = np.zeros((W, K), dtype=np.int64)
    acc = 0
    for s in range(W):
        for k in range(K):
            pre[s, k] = acc
            acc += cnt[s, k]
    col = cnt.sum(0).astype(np.int64)
    outoff = np.cumsum(col) - col
    rows_t = torch.from_numpy(rows).cuda()
    out = torch.zeros_like(rows_t)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    TS.tile_merge(rows_t, out, torch.from_numpy(pre).cuda(), torch.from_numpy(cnt).cuda(),
                  torch.from_numpy(outoff).cuda(), fb, flag)
    assert int(flag.item()) == 1
    got = out.cpu().numpy()
    for k in range(K):
        idx = np.concatenate([np.arange(pre[s, k], pre[s, k] + cnt[s, k]) for s in range(W)])
        order = sorted(range(len(idx)), key=lambda i: (bytes(rows[idx[i], :10]), i))
        exp = rows[idx[order]]
        seg = got[outoff[k]: outoff[k] + col[k]]
        if k == 7:
            assert not seg.any()                  # left out for the caller's fallback
        else:
            assert np.array_equal(seg, exp), k


def test_fine_bits_keep_buckets_small():
    assert RS.fine_bits(10_000_000_000) == 24          # 8 ranks x 1.25e9: ~600 rows per bucket
    assert RS.fine_bits(1000) == 16
    for total in (2_500_000_000, 5_000_000_000, 10_000_000_000):
        assert total / (1 << RS.fine_bits(total)) <= 1.01 * RS.FINE_ROWS
    assert TS.tile_cap() >= 1.5 * RS.FINE_ROWS


@pytest.mark.parametrize("W,rank", [(4, 1), (2, 0)])
def test_loopback_rank_output_is_exact(W, rank):
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortLoopbackJob
    n = 400_000
    job = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=n), W, rank)
    job.step()
    v = job.validate()
    assert v["ok"], v
    # reference: every record of the job whose key lies in this rank's fine range, stable by
    # (key, source rank, record number)
    allrows = torch.empty((W * n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(allrows, 0, job.cfg.seed)
    a = allrows.cpu().numpy()
    hi = a[:, :8].copy().view(">u8").reshape(-1).astype(np.uint64)
    lo, top = job.bounds
    sel = np.nonzero((hi >= np.uint64(lo)) & (hi <= np.uint64(top)))[0]
    order = np.lexsort([sel, a[sel, 9], a[sel, 8], hi[sel]])     # last key = primary
    exp = a[sel[order]]
    got = job.out.cpu().numpy()
    assert got.shape == exp.shape
    assert np.array_equal(got, exp)


def test_merge_received_rounds_falls_back_on_a_skewed_bucket():
    """A fine bucket past one workgroup's capacity (heavy key skew) flags its round, which is then
    sorted by the stored-row radix sort: the output is still the exact stable order."""
    g = np.random.default_rng(11)
    W, B, fb = 2, 2, 16
    n_src = [30_000, 25_000]
    L = [0, 1 << 15, 1 << 16]                     # range 0 = buckets [0, 2^15), range 1 = the rest
    pieces, fine_rows = [], []
    for s in range(W):
        n = n_src[s]
        hi = g.integers(0, 1 << 64, size=n, dtype=np.uint64)
        hot = g.random(n) < 0.05                   # ~2750 rows of the job in bucket 777 (range 0)
        hi[hot] = (np.uint64(777) << np.uint64(48)) | (hi[hot] & np.uint64((1 << 48) - 1))
        rows = g.integers(0, 256, size=(n, 100), dtype=np.uint8)
        rows[:, :8] = hi.astype(">u8").view(np.uint8).reshape(n, 8)
        rows[::13, 8:10] = 7
        b = (hi >> np.uint64(64 - fb)).astype(np.int64)
        order = np.argsort(b, kind="stable")      # the send side's bucket order
        rows, b = rows[order], b[order]
        pieces.append((rows, b))
    # receive layout: round r = range r, source-major pieces
    blocks, off, fine = [], [0], np.zeros((W, 1 << fb), dtype=np.int32)
    for r in range(B):
        for s in range(W):
            rows, b = pieces[s]
            sel = (b >= L[r]) & (b < L[r + 1])
            blocks.append(rows[sel])
        off.append(off[-1] + sum(len(x) for x in blocks[-W:]))
    for s in range(W):
        fine[s] = np.bincount(pieces[s][1], minlength=1 << fb)
    recv = np.concatenate(blocks)
    N = recv.shape[0]
    bufs = RS.SortBuffers.allocate(N, 100, "cuda")
    bufs.rows_in[:N] = torch.from_numpy(recv).cuda()
    out = RS.merge_received_rounds(bufs, off, torch.from_numpy(fine).cuda(), L, fb, B, 0, [N] * B, 0)
    got = out.cpu().numpy()
    exp = []
    for r in range(B):
        blk = recv[off[r]: off[r + 1]]
        key = [bytes(x[:10]) for x in blk]
        exp.append(blk[sorted(range(len(blk)), key=lambda i: (key[i], i))])
    assert np.array_equal(got, np.concatenate(exp))


@pytest.mark.parametrize("rec,key_off,key_len,desc", [
    (100, 0, 10, False), (64, 8, 8, False), (64, 8, 8, True), (68, 3, 5, True), (128, 120, 8, False),
    (12, 0, 2, False), (16, 6, 10, True), (40, 0, 10, True)])
def test_tile_merge_any_width_and_key(rec, key_off, key_len, desc):
    """ts_tile_merge over rows of other widths, a key of <= 10 bytes anywhere in the row, ascending
    or descending: every bucket in the stable order (key, source, slot) of a numpy reference; a hot
    bucket takes the register-path kernel."""
    g = np.random.default_rng(rec * 31 + key_off)
    W, fb, n = 3, 16, 60_000
    rows = g.integers(0, 256, size=(n, rec), dtype=np.uint8)
    rows[: 900, key_off: key_off + 2] = 0x5A            # one hot bucket (~900 rows > the LDS stage)
    rows[1000::200, key_off: key_off + key_len] = rows[950, key_off: key_off + key_len]    # equal keys
    key = np.zeros((n, 10), dtype=np.uint8)
    key[:, :key_len] = rows[:, key_off: key_off + key_len]
    if desc:
        key[:, :key_len] ^= 0xFF
    bucket = ((key[:, 0].astype(np.int64) << 8) | key[:, 1]) >> (16 - fb)
    src = g.integers(0, W, size=n)
    pieces = []
    cnt = np.zeros((W, 1 << fb), dtype=np.int32)
    for s in range(W):
        sel = np.nonzero(src == s)[0]
        sel = sel[np.argsort(bucket[sel], kind="stable")]       # the send side's bucket order
        pieces.append(sel)
        cnt[s] = np.bincount(bucket[sel], minlength=1 << fb)
    order_in = np.concatenate(pieces)
    recv = rows[order_in]
    pre = np.zeros_like(cnt, dtype=np.int64)
    base = 0
    for s in range(W):
        pre[s] = base + np.cumsum(cnt[s]) - cnt[s]
        base += int(cnt[s].sum())
    col = cnt.sum(0).astype(np.int64)
    outoff = np.cumsum(col) - col
    out = torch.zeros((n, rec), dtype=torch.uint8, device="cuda")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    TS.tile_merge(torch.from_numpy(recv).cuda(), out, torch.from_numpy(pre).cuda(), torch.from_numpy(cnt).cuda(),
                  torch.from_numpy(outoff).cuda(), fb, flag, key_off=key_off, key_len=key_len, descending=desc)
    assert int(flag.item()) == 0
    k = key[order_in]
    exp = recv[np.lexsort([np.arange(n)] + [k[:, j] for j in range(9, -1, -1)])]
    assert np.array_equal(out.cpu().numpy(), exp)


def test_bucket_copy_orders_one_key_buckets_of_any_size():
    """Fine buckets that each hold one key (2-byte keys, fb = 16): the merge is the W slices in
    source order, including buckets far past the LDS merge's 1024 rows."""
    g = np.random.default_rng(5)
    W, fb, n, rec = 3, 16, 90_000, 20
    rows = g.integers(0, 256, size=(n, rec), dtype=np.uint8)
    rows[:, :2] = g.integers(0, 40, size=(n, 2), dtype=np.uint8)       # 1600 keys, ~56 rows each
    rows[:5000, :2] = 7                                               # one key of 5000+ rows
    bucket = (rows[:, 0].astype(np.int64) << 8) | rows[:, 1]
    src = g.integers(0, W, size=n)
    pieces = [np.nonzero(src == s)[0] for s in range(W)]
    pieces = [p[np.argsort(bucket[p], kind="stable")] for p in pieces]
    cnt = np.stack([np.bincount(bucket[p], minlength=1 << fb) for p in pieces]).astype(np.int32)
    order_in = np.concatenate(pieces)
    recv = rows[order_in]
    pre = np.zeros_like(cnt, dtype=np.int64)
    base = 0
    for s in range(W):
        pre[s] = base + np.cumsum(cnt[s]) - cnt[s]
        base += int(cnt[s].sum())
    col = cnt.sum(0).astype(np.int64)
    outoff = np.cumsum(col) - col
    out = torch.zeros((n, rec), dtype=torch.uint8, device="cuda")
    TS.bucket_copy(torch.from_numpy(recv).cuda(), out, torch.from_numpy(pre).cuda(), torch.from_numpy(cnt).cuda(),
                   torch.from_numpy(outoff).cuda())
    exp = recv[np.lexsort([np.arange(n), bucket[order_in]])]
    assert np.array_equal(out.cpu().numpy(), exp)
