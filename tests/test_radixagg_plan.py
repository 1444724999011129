"""CPU checks of the radix-aggregation planning (digit widths, distinct estimate) and of the
output hole closing (ops/radixagg.py); the kernels themselves: tests/test_gpu_radixagg.py."""
import torch

from dryad_amd.ops import radixagg as RA


def test_plan_bits_targets_lds_table():
    assert RA.plan_bits(738_000_000) == [8, 7, 7]
    assert sum(RA.plan_bits(10)) == RA.MIN_BITS
    assert all(w <= 8 for w in RA.plan_bits(1 << 40)) and sum(RA.plan_bits(1 << 40)) == RA.MAX_BITS


def test_distinct_estimate_bounds():
    n = 1_000_000_000
    assert RA.distinct_upper_estimate(65_500, 65_536, n) == n          # all distinct: upper bound
    est = RA.distinct_upper_estimate(30_000, 65_536, n)
    assert 30_000 <= est <= 100_000
    assert RA.distinct_upper_estimate(100, 65_536, n) >= 100


def _holey(total_groups, chunk, tails_cut, seed=0):
    """Simulate chunk reservation: groups 0..G-1 laid out with holes at each worker's last chunk."""
    g = torch.Generator().manual_seed(seed)
    workers = len(tails_cut)
    arr = torch.full((total_groups + (workers + 1) * chunk,), -1, dtype=torch.int64)
    head, val, tails = 0, 0, []
    for w, keep in enumerate(tails_cut):
        nchunks = int(torch.randint(0, 3, (1,), generator=g))
        for c in range(nchunks):
            used = chunk if c < nchunks - 1 else keep
            arr[head:head + used] = torch.arange(val, val + used)
            val += used
            if c == nchunks - 1:
                tails.append((head + used, head + chunk))
            head += chunk
        if nchunks == 0:
            tails.append((0, 0))
    return arr, head, tails, val


def test_close_holes_compacts_every_group():
    for seed in range(5):
        arr, head, tails, groups = _holey(0, 16, [3, 0, 16, 7, 1, 9], seed)
        other = arr.clone() * 10
        total = RA._close_holes(head, tails, [arr, other])
        assert total == groups
        assert sorted(arr[:total].tolist()) == list(range(groups))
        assert torch.equal(other[:total], arr[:total] * 10)
