"""Row layouts of columnar tables for the fine-bucket sort (ops/rowpack.py): key parts cut to the
job's value range, the ordered-value mapping, integer key columns recovered from the key bytes."""
import numpy as np
import torch

from dryad_amd.gpu.table import DeviceTable, Shape
from dryad_amd.ops import rowpack as RP


def _table(**cols):
    n = next(iter(cols.values())).shape[0]
    return DeviceTable(n, Shape("tuple", list(cols)), dict(cols))


def test_ordered_values_keep_the_order():
    for dt, vals in ((torch.int64, [-(1 << 63), -5, -1, 0, 1, 7, (1 << 63) - 1]),
                     (torch.int32, [-(1 << 31), -2, 0, 3, (1 << 31) - 1]),
                     (torch.int8, [-128, -1, 0, 127]),
                     (torch.float32, [-np.inf, -2.5, -1e-30, 0.0, 1e-30, 3.0, np.inf]),
                     (torch.float64, [-1e300, -1.0, 0.0, 2.0, 1e300])):
        o = [RP.ordered(v, dt) for v in vals]
        assert o == sorted(o) and len(set(o)) == len(o), (dt, o)
    assert RP.ordered(-0.0, torch.float32) == RP.ordered(0.0, torch.float32)


def test_plan_cuts_key_parts_to_the_value_range():
    n = 100
    t = _table(Key=torch.arange(n, dtype=torch.int64), V1=torch.arange(n, dtype=torch.int64) * 1000,
               F=torch.rand(n, dtype=torch.float32), B=torch.zeros(n, dtype=torch.uint8))
    keys = [t.cols["V1"]]
    b = RP.merge_bounds([RP.key_bounds(keys, n) + [0, 0], RP.key_bounds(keys, 0) + [0, 0]], 1)
    assert b == [((1 << 63), (1 << 63) + 99_000)]
    lay = RP.plan(t, keys, b)
    # 99000 needs 17 bits: a 3-byte key part shifted to the top; V1 is recovered from it
    assert lay.key_len == 3 and lay.fields[0][:2] == ("V1", torch.int64) and lay.fields[0][5]
    assert lay.fields[0][7] == 64 - 17 and lay.fields[0][8] == 3
    offs = {f[0]: f[2] for f in lay.fields[1:]}
    assert offs == {"Key": 8, "F": 16, "B": 20} and lay.rec == 24
    assert [f[0] for f in lay.fields].count("V1") == 1


def test_plan_refuses_what_does_not_fit():
    n = 10
    t = _table(A=torch.arange(n, dtype=torch.int64), B=torch.arange(n, dtype=torch.int64))
    full = [(0, (1 << 64) - 1)] * 2
    assert RP.plan(t, [t.cols["A"], t.cols["B"]], full) is None          # 16 key bytes
    assert RP.plan(t, [t.cols["A"], t.cols["B"]], [(0, 1000), (0, 1000)]).key_len == 4
    wide = _table(**{f"c{i}": torch.zeros(n, dtype=torch.int64) for i in range(17)})
    assert RP.plan(wide, [wide.cols["c0"]], [(0, 1)]) is None           # rows past 128 bytes
    f = _table(F=torch.rand(n, dtype=torch.float64))
    lay = RP.plan(f, [f.cols["F"]], RP.merge_bounds([RP.key_bounds([f.cols["F"]], n)], 1))
    assert lay.fields[0][0] is None and ("F", torch.float64) in [x[:2] for x in lay.fields]   # floats stay raw


def test_equal_keys_take_one_byte():
    n = 5
    t = _table(K=torch.full((n,), 42, dtype=torch.int32), V=torch.arange(n, dtype=torch.int64))
    lay = RP.plan(t, [t.cols["K"]], RP.merge_bounds([RP.key_bounds([t.cols["K"]], n)], 1))
    assert lay.key_len == 1 and lay.fields[0][7] == 63
