"""utils/validate.py: order-independent group fingerprints for the benchmarks' validation."""
import torch

from dryad_amd.utils import validate as V


def _rows(n=20000, keys=3000, seed=1):
    g = torch.Generator().manual_seed(seed)
    k = torch.randint(0, keys, (n,), generator=g)
    vals = [torch.randint(-1000, 1000, (n,), generator=g) for _ in range(3)]
    return k, vals


def test_reference_groupby_and_fingerprint_are_order_independent():
    k, vals = _rows()
    ops = ["count", "sum", "min", "max"]
    groups = V.groups_of(k, vals, ops)
    d = {}
    for i in range(k.numel()):
        kk = int(k[i])
        c, s, mn, mx = d.get(kk, (0, 0, None, None))
        v1, v2, v3 = int(vals[0][i]), int(vals[1][i]), int(vals[2][i])
        d[kk] = (c + 1, s + v1, v2 if mn is None else min(mn, v2), v3 if mx is None else max(mx, v3))
    assert groups[0].tolist() == sorted(d)
    assert [tuple(int(c[i]) for c in groups[1:]) for i in range(groups[0].numel())] == [d[x] for x in sorted(d)]
    fp = V.group_fingerprint(groups)
    perm = torch.randperm(groups[0].numel(), generator=torch.Generator().manual_seed(3))
    assert V.group_fingerprint([c[perm] for c in groups]) == fp
    # split over "ranks" and combined
    half = groups[0].numel() // 2
    assert V.combine([V.group_fingerprint([c[:half] for c in groups]),
                      V.group_fingerprint([c[half:] for c in groups])]) == fp
    # the chunked, key-range expected path gives the same value
    chunks = lambda: ([k[a:a + 4096]] + [v[a:a + 4096] for v in vals] for a in range(0, k.numel(), 4096))  # noqa
    assert V.expected_fingerprint(chunks, ops, V.key_ranges(0, 2999, 5)) == fp


def test_a_corrupted_group_changes_the_fingerprint():
    k, vals = _rows()
    groups = V.groups_of(k, vals, ["count", "sum", "min", "max"])
    fp = V.group_fingerprint(groups)
    for col in range(5):
        bad = [c.clone() for c in groups]
        bad[col][17] += 1                   # one group's key / count / sum / min / max off by one
        assert V.group_fingerprint(bad) != fp, col
    # two groups merged with their totals preserved (what a totals-only check would accept)
    bad = [c.clone() for c in groups]
    bad[1][0] += bad[1][1]
    bad[2][0] += bad[2][1]
    bad = [torch.cat([c[:1], c[2:]]) for c in bad]
    assert int(bad[1].sum()) == int(groups[1].sum()) and int(bad[2].sum()) == int(groups[2].sum())
    assert V.group_fingerprint(bad) != fp
