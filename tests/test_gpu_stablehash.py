"""Device partitioner hash (csrc/kernels/stablehash.hip) == host stable_hash for every key kind,
so a keyed shuffle sends a key to the same consumer whether its producer ran on the device or
fell back to the host, and whatever column width a partition inferred (int32 vs int64)."""
import pytest
import torch

import dryad_amd as D
from dryad_amd.gpu import ops as G
from dryad_amd.gpu.table import DeviceTable, Shape
from dryad_amd.ops import relational as R
from dryad_amd.runtime.vertex_ops import _h as stable_hash, hash_port

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _dev_hash(keys, tuple_form=False):
    n = keys[0].t.shape[0] if keys[0].kind != R.H_STR else keys[0].off.shape[0]
    _, h = R.stable_hash_dest(keys, n, 0, tuple_form, DEV, want_hash=True)
    return [x & ((1 << 64) - 1) for x in h.tolist()]


@pytest.mark.parametrize("dtype", [torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8, torch.bool])
def test_integer_columns(dtype):
    if dtype == torch.bool:
        vals = [True, False, True]
    elif dtype == torch.uint8:
        vals = [0, 1, 200, 255]
    else:
        info = torch.iinfo(dtype)
        vals = [0, 1, -1, 7, info.min, info.max, 12345 % (info.max + 1)]
    c = torch.tensor(vals, dtype=dtype, device=DEV)
    got = _dev_hash([R.HashKey.column(c)])
    assert got == [stable_hash(v) for v in vals]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_float_columns(dtype):
    vals = [0.0, -0.0, 1.0, -3.0, 2.5, -1e-3, float("inf"), float("-inf"), float("nan"), 1e30, 2.0 ** 63, -2.0 ** 63]
    c = torch.tensor(vals, dtype=dtype, device=DEV)
    host = [float(x) for x in c.cpu().tolist()]        # the value the host sees after the dtype cast
    got = _dev_hash([R.HashKey.column(c)])
    assert got == [stable_hash(v) for v in host]


def test_int32_and_int64_agree():
    a = torch.arange(-5000, 5000, dtype=torch.int32, device=DEV)
    assert _dev_hash([R.HashKey.column(a)]) == _dev_hash([R.HashKey.column(a.to(torch.int64))])
    assert _dev_hash([R.HashKey.column(a)]) == _dev_hash([R.HashKey.column(a.to(torch.float64))])


def test_tuple_bytes_and_strings():
    a = torch.tensor([1, 2, 3], dtype=torch.int64, device=DEV)
    b = torch.tensor([0.5, -2.0, 7.0], dtype=torch.float64, device=DEV)
    got = _dev_hash([R.HashKey.column(a), R.HashKey.column(b)], tuple_form=True)
    assert got == [stable_hash((1, 0.5)), stable_hash((2, -2.0)), stable_hash((3, 7.0))]
    rows = torch.randint(0, 256, (50, 12), dtype=torch.uint8, device=DEV)
    got = _dev_hash([R.HashKey.bytes_field(rows, 2, 7)])
    host = rows.cpu().numpy()
    assert got == [stable_hash(bytes(host[i, 2:9])) for i in range(50)]
    words = ["", "a", "héllo", "dryad", "x" * 300]
    blob = "".join(words).encode("utf-8")
    off, o = [], 0
    for w in words:
        off.append(o)
        o += len(w.encode("utf-8"))
    heap = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(DEV)
    ot = torch.tensor(off, dtype=torch.int64, device=DEV)
    lt = torch.tensor([len(w.encode("utf-8")) for w in words], dtype=torch.int64, device=DEV)
    assert _dev_hash([R.HashKey.string(heap, ot, lt)]) == [stable_hash(w) for w in words]


@pytest.mark.parametrize("nparts", [3, 8, 300, 5000])
def test_hash_partition_matches_host(nparts):
    vals = torch.randint(-10 ** 12, 10 ** 12, (20000,), dtype=torch.int64, device=DEV)
    t = DeviceTable(vals.shape[0], Shape("scalar", ["v"]), {"v": vals})
    perm, st = G.hash_partition_perm(t, lambda x: x, nparts)
    assert len(st) == nparts + 1 and st[0] == 0 and st[-1] == vals.shape[0]
    host = vals.cpu().tolist()
    p = perm.cpu().tolist()
    for d in range(nparts):
        for i in p[st[d]:st[d + 1]]:
            assert hash_port(host[i], nparts) == d
    assert p == sorted(p, key=lambda i: (hash_port(host[i], nparts), i))   # stable inside a port


def test_mixed_width_partitions_colocate():
    """gen://range infers int32 for a partition whose values fit and int64 for one that does
    not; a keyed shuffle of x % 100 must still put equal keys together."""
    src = "gen://range?start=2147482000&count=4000&partitions=2"
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 2
    got = c.FromStore(src).Select(lambda x: x % 100).HashPartition(lambda x: x, 4).Distinct().Count()
    assert got == 100
