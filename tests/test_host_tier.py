"""Pinned-host tier (host://, HostRows), raw-rows partfile parts and the out-of-core sort planning
(CPU: no GPU needed; the sort itself is covered by tests/test_gpu_extsort.py)."""
import os

import numpy as np
import pytest
import torch

import dryad_amd as D
from dryad_amd.io.hosttable import HostRows, is_registered
from dryad_amd.io.providers import provider_for


def test_host_rows_roundtrip_and_view():
    a = torch.arange(60, dtype=torch.uint8).reshape(6, 10)
    h = HostRows.from_tensor(a, key_off=2, key_len=3, pinned=False)
    assert h.n == 6 and h.stride == 10 and h.nbytes == 60 and not h.pinned
    assert h.to_objects()[1] == bytes(range(10, 20))
    v = h.view(4)
    assert v.n == 4 and v.to_objects() == h.to_objects()[:4] and v.key_off == 2
    assert not is_registered(h.rows)
    h.release()
    assert h.n == 0


def test_host_provider_object_roundtrip():
    ctx = D.DryadLinqContext(1)
    ctx.LocalDebug = True
    uri = "host://tier_test"
    ctx.FromEnumerable(list(range(20))).Where(lambda x: x % 3 == 0).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    prov = provider_for(uri)
    assert prov.exists(uri)
    assert sorted(ctx.FromStore(uri)) == [0, 3, 6, 9, 12, 15, 18]
    assert prov.local_rows(uri, 0) is None               # object partitions, not HostRows
    prov.delete(uri)
    assert not prov.exists(uri)


def test_host_provider_holds_rows_tables():
    uri = "host://rows_test"
    prov = provider_for(uri)
    h = HostRows.from_tensor(torch.full((3, 8), 7, dtype=torch.uint8), pinned=False)
    prov.put(uri, {"dtype": None, "partitions": 1, "local": {0: h}})
    assert prov.stream_info(uri) == (1, 24)
    assert prov.local_rows(uri, 0) is h
    assert prov.read_partition(uri, 0, None) == [bytes([7] * 8)] * 3
    prov.delete(uri)


def test_partfile_raw_rows_parts(tmp_path):
    from dryad_amd.io import partfile as PF
    from dryad_amd.runtime.jobmanager import write_schema
    meta = str(tmp_path / "rows_table")
    base = PF.default_base(meta)
    os.makedirs(os.path.dirname(base), exist_ok=True)
    rows = np.arange(5 * 12, dtype=np.uint8).reshape(5, 12)
    tmp = PF.tmp_part_path(base, 0, 0, 0, 0)
    rows.tofile(tmp)
    PF.commit_parts(meta, base, [tmp])
    write_schema(meta, None, "rows", stride=12, key_off=0, key_len=4)
    uri = "partfile://" + meta
    prov = provider_for(uri)
    assert prov.read_partition(uri, 0, None) == [bytes(r) for r in rows]
    mm, ko, kl = prov.rows_part(uri, 0)
    assert mm.shape == (5, 12) and (ko, kl) == (0, 4) and np.array_equal(np.asarray(mm), rows)


def test_external_sort_geometry_fits_budget():
    from dryad_amd.ops.extsort import plan_geometry
    budget = 48 * 10**9
    chunk, cap, P = plan_geometry(10**9, 10**9, 100, 1, budget)
    assert chunk * (4 * 100 + 16) <= budget and cap * (4 * 100 + 32) <= budget
    assert P * cap * 0.7 >= 10**9 and P <= 256
    chunk8, _, P8 = plan_geometry(125_000_000, 10**9, 100, 8, budget)
    assert chunk8 * (7 * 100 + 16) <= budget and P8 * 8 <= 256
    with pytest.raises(RuntimeError):
        plan_geometry(10**12, 10**12, 100, 1, 10**9)    # would need > 256 range buckets


def test_mapped_host_rows_are_a_file(tmp_path):
    """The disk tier: a memory-mapped HostRows writes through to its file and survives release."""
    import numpy as np
    from dryad_amd.io.hosttable import HostRows
    path = str(tmp_path / "rows.bin")
    h = HostRows.mapped(path, 1000, 16, 0, 8)
    src = torch.randint(0, 256, (1000, 16), dtype=torch.uint8)
    h.rows.copy_(src)
    v = h.view(600)
    assert v.path == path and torch.equal(v.rows, src[:600])
    h.release()
    got = np.fromfile(path, dtype=np.uint8).reshape(1000, 16)
    assert np.array_equal(got, src.numpy())
    e = HostRows.mapped(str(tmp_path / "empty.bin"), 0, 16)
    assert e.n == 0 and (tmp_path / "empty.bin").exists()
