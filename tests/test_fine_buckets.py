"""CPU checks of the fine-bucket exchange's host-side geometry (ops/recordsort.py): bucket bits,
range bounds cut to bucket edges, hi-word bounds of a range."""
from dryad_amd.ops import recordsort as RS


def test_fine_bits_targets_bucket_rows():
    assert RS.fine_bits(10_000_000_000) == 24
    assert RS.fine_bits(2_500_000_000) == 22
    assert RS.fine_bits(0) == RS.FINE_MIN_BITS
    assert RS.fine_bits(10 ** 15) == RS.FINE_MAX_BITS
    for total in (10 ** 7, 3 * 10 ** 8, 10 ** 9, 10 ** 10):
        fb = RS.fine_bits(total)
        assert RS.FINE_MIN_BITS <= fb <= RS.FINE_MAX_BITS
        assert fb == RS.FINE_MIN_BITS or total > RS.FINE_ROWS * (1 << (fb - 1))


def test_fine_bounds_cut_separators_to_bucket_edges():
    fb = 20
    seps = [(1 << 63) + 12345, (3 << 62) + (1 << 44) + 7]
    L = RS.fine_bounds(seps, fb)
    assert L == [0, (1 << 19), (3 << 18) + 1, 1 << 20]
    assert all(a <= b for a, b in zip(L, L[1:]))
    lo, hi = RS.fine_hi_bounds(L, fb, 1)
    assert lo == 1 << 63 and hi == ((3 << 18) + 1 << 44) - 1
    assert RS.fine_hi_bounds(L, fb, 2)[1] == (1 << 64) - 1


def test_overlap_schedule_merges_once_the_rows_under_the_output_are_sent():
    """overlap_schedule: round j's merge waits for its own arrival and for the payload round that
    sends the last send rows under out[off[j]:off[j+1]]; a round that would hold its receive slot
    longer than the slots allow makes the exchange fall back (None)."""
    W, B = 2, 4
    # send-row starts st[b * W + r]: 100 rows per round
    st = [0, 50, 100, 150, 200, 250, 300, 350, 400]
    # balanced receive: every merge waits only for its own round
    assert RS.overlap_schedule(st, [0, 100, 200, 300, 400], B, W, 400, 3) == [0, 1, 2, 3]
    # round 0 receives 130 rows: its output reaches into round 1's send rows
    assert RS.overlap_schedule(st, [0, 130, 200, 300, 400], B, W, 400, 3) == [1, 1, 2, 3]
    # rows past the sent ones never held data (n_sent), and with separate output buffers
    # (n_sent = 0) nothing overlays the send rows
    assert RS.overlap_schedule(st, [0, 130, 200, 300, 420], B, W, 400, 3) == [1, 1, 2, 3]
    assert RS.overlap_schedule(st, [0, 330, 340, 350, 360], B, W, 0, 3) == [0, 1, 2, 3]
    # round 0's output reaches round 3's rows: 3 rounds of lag do not fit 3 slots
    assert RS.overlap_schedule(st, [0, 330, 340, 350, 400], B, W, 400, 3) is None
    assert RS.overlap_schedule(st, [0, 330, 340, 350, 400], B, W, 400, 4) == [3, 3, 3, 3]


def test_fine_subs_targets_one_gib_rounds():
    assert RS.fine_subs(125 * 10**9, 8) == 128
    assert RS.fine_subs(125 * 10**9, 1) == 128
    assert RS.fine_subs(10**6, 2) == 4
    assert RS.fine_subs(10**15, 8) == 256           # world * rounds <= 2048


def test_fine_merge_arguments_match_the_per_round_formula():
    """FineMerge computes every round's (slice starts, counts, output offsets) up front, round-major;
    each round's slices equal the per-round prefix-sum formula."""
    import torch
    torch.manual_seed(0)
    W, B, base, K, rank = 4, 5, 37, 200, 1
    kb0 = sorted(torch.randint(0, K, (B - 1,)).tolist())
    L = [0] * (rank * B) + [base] + [base + x for x in kb0] + [base + K] + [base + K] * (B * 2 - rank * B - B)
    fine = torch.randint(0, 5, (W, K), dtype=torch.int32)
    m = RS.FineMerge(fine, L, 16, B, rank, torch.empty((10, 100), dtype=torch.uint8))
    ex = torch.cumsum(fine.view(-1).long(), 0).view(W, K) - fine
    ex = ex - ex[:, :1]
    col = fine.sum(0, dtype=torch.int64)
    cex = torch.cumsum(col, 0) - col
    for b in range(B):
        k0, k1 = L[rank * B + b] - base, L[rank * B + b + 1] - base
        rps = (ex[:, k1:k1 + 1] if k1 < K else (ex[:, -1:] + fine[:, -1:])) - ex[:, k0:k0 + 1]
        pre = ex[:, k0:k1] - ex[:, k0:k0 + 1] + (torch.cumsum(rps, 0) - rps)
        assert torch.equal(m.pre[W * k0: W * k1].view(W, k1 - k0), pre), b
        assert torch.equal(m.cnt[W * k0: W * k1].view(W, k1 - k0), fine[:, k0:k1]), b
        assert torch.equal(m.outoff[k0:k1], cex[k0:k1] - cex[k0]), b


def test_fine_merge_of_a_rank_without_buckets():
    """A rank whose key ranges hold no fine bucket (all keys equal, kept together on another rank):
    no merge arguments, nothing indexed."""
    import torch
    L = [0, 0, 0, 0, 0, 65536, 65536, 65536, 65536]        # W = 2, B = 4: rank 0 owns nothing
    m = RS.FineMerge(torch.zeros((2, 0), dtype=torch.int32), L, 16, 4, 0, torch.empty((4, 100), dtype=torch.uint8))
    assert m.kb == [0] * 5 and m.pre.numel() == 0
    m.merge(0, torch.empty((0, 100), dtype=torch.uint8), 0, 0, 0)


def test_fine_rows_ok_any_width_and_key():
    from dryad_amd.ops import recordsort as RS
    ok = lambda rec, pitch, ko, kl: RS.fine_rows_ok(rec, pitch, ko, kl, 8, 1000)  # noqa: E731
    assert ok(100, 100, 0, 10) and ok(100, 128, 0, 10)            # TeraSort rows
    assert ok(64, 64, 8, 8) and ok(12, 12, 0, 2) and ok(128, 128, 118, 10) and ok(64, 128, 0, 4)
    assert not ok(64, 64, 8, 12)          # keys past 10 bytes: the E128 path
    assert not ok(66, 66, 0, 8)           # rows not a multiple of 4 bytes
    assert not ok(8, 8, 0, 4) and not ok(132, 132, 0, 10)
    assert not ok(64, 64, 60, 8)          # key past the row
    assert not ok(64, 80, 0, 8)           # other pitches
    assert not RS.fine_rows_ok(64, 64, 8, 8, 1, 1000) and RS.fine_rows_ok(64, 64, 8, 8, 1, 1000, one_rank=True)
    assert not RS.fine_rows_ok(64, 64, 8, 8, 65, 1000)
