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
