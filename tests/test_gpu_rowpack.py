"""Columns <-> byte-keyed rows on the device (csrc/kernels/rowpack.hip) against numpy: the packed
key bytes order the rows like the key values (ints, floats, tuples, descending by inversion), and
unpacking restores every column bit for bit."""
import numpy as np
import pytest
import torch

from dryad_amd.gpu.table import DeviceTable, Shape
from dryad_amd.ops import rowpack as RP

pytestmark = pytest.mark.gpu


def _table(cols):
    n = next(iter(cols.values())).shape[0]
    return DeviceTable(n, Shape("tuple", list(cols)), dict(cols))


def _layout(t, keys):
    return RP.plan(t, keys, RP.merge_bounds([RP.key_bounds(keys, t.n)], len(keys)))


@pytest.mark.parametrize("case", ["int64", "int32_small", "float32", "float64_neg", "tuple", "int8_bool"])
def test_pack_orders_like_the_key_and_unpack_restores(case):
    g = torch.Generator(device="cpu").manual_seed(hash(case) % 1000)
    n = 100_003
    dev = "cuda"
    cols = {"Key": torch.randint(-(1 << 62), 1 << 62, (n,), generator=g),
            "V1": torch.randint(0, 1 << 31, (n,), generator=g),
            "F": torch.randn(n, generator=g, dtype=torch.float32),
            "D": torch.randn(n, generator=g, dtype=torch.float64) * 1e6,
            "S": torch.randint(-50, 50, (n,), generator=g, dtype=torch.int32),
            "b": torch.randint(0, 2, (n,), generator=g).to(torch.bool),
            "c": torch.randint(-128, 128, (n,), generator=g, dtype=torch.int8)}
    cols["F"][::97] = -0.0
    cols = {k: v.to(dev) for k, v in cols.items()}
    t = _table(cols)
    keys = {"int64": ["Key"], "int32_small": ["S"], "float32": ["F"], "float64_neg": ["D"], "tuple": ["S", "V1"],
            "int8_bool": ["c", "b"]}[case]
    kt = [cols[k] for k in keys]
    lay = _layout(t, kt)
    assert lay is not None
    rows = torch.empty((n, lay.rec), dtype=torch.uint8, device=dev)
    RP.pack(t, kt, lay, rows)
    # the key bytes order the rows like the key values (stable ties)
    kb = rows[:, : lay.key_len].cpu().numpy()
    order_bytes = np.lexsort([np.arange(n)] + [kb[:, j] for j in range(lay.key_len - 1, -1, -1)])
    vals = [cols[k].cpu().numpy() for k in keys]
    vals = [np.where(v == 0, 0, v) if v.dtype.kind == "f" else v.astype(np.int64) for v in vals]   # -0.0 == 0.0
    order_vals = np.lexsort([np.arange(n)] + vals[::-1])
    assert np.array_equal(order_bytes, order_vals)
    # unpacked columns are the originals, bit for bit (into caller memory and allocated)
    mem = torch.empty(n * lay.rec + 4096, dtype=torch.uint8, device=dev)
    for m in (mem, None):
        back = RP.unpack(rows, lay, m)
        assert list(back) == list(cols)
        for k in cols:
            assert torch.equal(back[k].view(torch.uint8), cols[k].view(torch.uint8)), (case, k)
