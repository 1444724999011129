"""Out-of-core sort (ops/extsort.py): HBM budget far below the data, buckets spilled to pinned host
memory.  Checked against the in-HBM sort of the same rows and a numpy stable sort."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _gen_rows(n, first=0, seed=11):
    from dryad_amd.ops import terasort as TS
    rows = torch.empty((n, 100), dtype=torch.uint8, device="cuda")
    TS.generate(rows, first, seed)
    return rows


def _in_hbm_sorted(rows):
    from dryad_amd.ops import recordsort as RS
    n = rows.shape[0]
    out = torch.empty_like(rows)
    ea = torch.empty((n + 16, 2), dtype=torch.int64, device="cuda")
    eb = torch.empty_like(ea)
    return RS.local_sort_rows(rows, out, ea, eb, 0, 10).cpu()


def _np_stable_sort(rows: np.ndarray, key_off, key_len):
    keys = np.ascontiguousarray(rows[:, key_off:key_off + key_len]).view(f"S{key_len}").ravel()
    return rows[np.argsort(keys, kind="stable")]


@pytest.mark.parametrize("n,budget", [(3_000_000, 64 << 20), (700_001, 24 << 20)])
def test_extsort_generator_matches_in_hbm_sort(n, budget):
    from dryad_amd.ops import extsort as EX
    st = EX.ExtSortStats()
    out = EX.external_sort(EX.GenTeraSortSource(0, n, 11), 0, 10, budget=budget, stats=st)
    assert st.chunks > 1 and st.buckets > 1, st
    assert out.n == n and st.max_bucket <= st.bucket_cap
    ref = _in_hbm_sorted(_gen_rows(n))
    assert torch.equal(out.rows, ref)
    h, bad, _, _ = EX.check_terasort_host(out, chunk_rows=250_000)
    assert bad == 0


@pytest.mark.parametrize("n,budget", [(3_000_000, 160 << 20), (900_001, 64 << 20)])
def test_extsort_hybrid_keeps_buckets_resident(n, budget):
    """Hybrid mode: the buckets that fit next to the working arena stay sorted in HBM; the tiered
    result equals the in-HBM sort and only the other buckets crossed PCIe."""
    from dryad_amd.io.hosttable import TieredRows
    from dryad_amd.ops import extsort as EX
    st = EX.ExtSortStats()
    out = EX.external_sort(EX.GenTeraSortSource(0, n, 11), 0, 10, budget=budget, stats=st, resident=True)
    assert isinstance(out, TieredRows) and st.resident_buckets >= 1 and 0 < st.resident_rows < n
    assert out.n == n and out.device_rows == st.resident_rows
    assert [s.is_cuda for s in out.segments] == [False, True]
    got = torch.cat([s.cpu() for s in out.segments])
    assert torch.equal(got, _in_hbm_sorted(_gen_rows(n)))
    host = n - st.resident_rows
    assert st.bytes_d2h == 2 * host * 100 and st.bytes_h2d == host * 100
    h, bad, _, _ = EX.check_terasort_host(out, chunk_rows=250_000)
    assert bad == 0


def test_extsort_hybrid_host_source_is_stable():
    from dryad_amd.io.hosttable import HostRows
    from dryad_amd.ops import extsort as EX
    n, stride = 400_000, 32
    g = np.random.default_rng(6)
    a = g.integers(0, 256, size=(n, stride), dtype=np.uint8)
    a[:, 4:14] = g.integers(0, 9, size=(n, 1), dtype=np.uint8)
    a[:, 20:28] = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)
    src = HostRows.from_tensor(torch.from_numpy(a), key_off=4, key_len=10)
    st = EX.ExtSortStats()
    out = EX.external_sort(EX.HostRowsSource(src), 4, 10, budget=12 << 20, stats=st, resident=True)
    got = np.concatenate([s.cpu().numpy() for s in out.segments]) if hasattr(out, "segments") else out.rows.numpy()
    assert st.resident_rows > 0
    np.testing.assert_array_equal(got, _np_stable_sort(a, 4, 10))


def test_extsort_host_source_duplicate_keys_is_stable():
    """Few distinct keys: runs of equal keys larger than a bucket are split by the tie tag and
    the result is the stable order."""
    from dryad_amd.io.hosttable import HostRows
    from dryad_amd.ops import extsort as EX
    n, stride = 400_000, 32
    g = np.random.default_rng(5)
    a = g.integers(0, 256, size=(n, stride), dtype=np.uint8)
    a[:, 4:14] = g.integers(0, 7, size=(n, 1), dtype=np.uint8)       # 7 distinct 10-byte keys
    a[:, 20:28] = np.arange(n, dtype=np.uint64).view(np.uint8).reshape(n, 8)   # original position
    src = HostRows.from_tensor(torch.from_numpy(a), key_off=4, key_len=10)
    st = EX.ExtSortStats()
    out = EX.external_sort(EX.HostRowsSource(src), 4, 10, budget=6 << 20, stats=st)
    assert st.buckets > 7 and st.bytes_h2d >= 3 * n * stride
    np.testing.assert_array_equal(out.rows.numpy(), _np_stable_sort(a, 4, 10))


def test_extsort_host_source_short_keys():
    from dryad_amd.io.hosttable import HostRows
    from dryad_amd.ops import extsort as EX
    n, stride = 250_000, 16
    g = np.random.default_rng(9)
    a = g.integers(0, 256, size=(n, stride), dtype=np.uint8)
    src = HostRows.from_tensor(torch.from_numpy(a), key_off=0, key_len=3)
    out = EX.external_sort(EX.HostRowsSource(src), 0, 3, budget=2 << 20)
    np.testing.assert_array_equal(out.rows.numpy(), _np_stable_sort(a, 0, 3))


def test_query_out_of_core_orderby_to_host_table():
    """FromStore(gen) -> OrderBy -> ToStore(host://) with a small HBM budget runs the external
    sort through the GPU executor; reading host:// back into HBM sorts in place."""
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    n = 1_000_000
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.HbmBudgetBytes = 48 << 20
    src = f"gen://terasort?records={n}&partitions=1&seed=11"
    ctx.FromStore(src).OrderBy(lambda r: r[0:10]).ToStore("host://ooc_sorted", delete_if_exists=True).SubmitAndWait()
    res = ctx._get_executor().last_result
    assert res["external_sort"] is not None and res["external_sort"].buckets > 1
    assert not res["fallbacks"]
    h = provider_for("host://ooc_sorted").local_rows("host://ooc_sorted", 0)
    assert torch.equal(h.rows, _in_hbm_sorted(_gen_rows(n)))
    # host:// -> HBM -> Where -> back: the pinned tier is readable by later jobs
    cnt = ctx.FromStore("host://ooc_sorted").Where(lambda r: r[0] < 128).Count()
    assert cnt == int((h.rows[:, 0] < 128).sum())
    provider_for("host://ooc_sorted").delete("host://ooc_sorted")


def test_query_out_of_core_orderby_to_disk_partfile(tmp_path):
    """FromStore(gen) -> OrderBy -> ToStore(partfile://) with the disk tier forced: the sorted rows
    are written through a memory-mapped file that becomes the part file (no host-DRAM copy of the
    output), and read back equal to the in-HBM sort."""
    import os
    import numpy as np
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    n = 600_000
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.HbmBudgetBytes = 40 << 20
    ctx.ExternalSort = True
    ctx.ExternalSortToDisk = True
    out = f"partfile://{tmp_path}/sorted"
    src = f"gen://terasort?records={n}&partitions=1&seed=5"
    ctx.FromStore(src).OrderBy(lambda r: r[0:10]).ToStore(out, delete_if_exists=True).SubmitAndWait()
    res = ctx._get_executor().last_result
    assert res["external_sort"] is not None and res["external_sort"].buckets > 1
    assert res["external_sort"].tier == "disk"
    mm, off, ln = provider_for(out).rows_part(out, 0)
    assert (off, ln) == (0, 10)
    assert np.array_equal(np.asarray(mm), _in_hbm_sorted(_gen_rows(n, 0, 5)).numpy())
    assert not [f for f in os.listdir(tmp_path) if ".extsort." in f]


@pytest.mark.parametrize("resident", [False, True])
def test_extsort_descending_is_a_stable_reverse_order(resident):
    """OrderByDescending out of core: inverted key bits for the sample, the range destinations and
    every bucket sort; equal keys keep the source order (stable) -- against numpy."""
    from dryad_amd.io.hosttable import HostRows
    from dryad_amd.ops import extsort as EX
    n, stride = 400_003, 24
    g = np.random.default_rng(5)
    a = g.integers(0, 256, size=(n, stride), dtype=np.uint8)
    a[:, 2] = 7                                    # many equal 3-byte keys (ties)
    src = HostRows.from_tensor(torch.from_numpy(a), key_off=0, key_len=3)
    out = EX.external_sort(EX.HostRowsSource(src), 0, 3, budget=4 << 20, resident=resident, descending=True)
    got = out.rows.numpy() if hasattr(out, "rows") else np.concatenate([x.cpu().numpy() for x in out.segments])
    k_int = a[:, 0].astype(np.int64) << 16 | a[:, 1].astype(np.int64) << 8 | a[:, 2].astype(np.int64)
    np.testing.assert_array_equal(got, a[np.argsort(-k_int, kind="stable")])


def test_query_out_of_core_orderby_descending_to_host_table():
    import dryad_amd as D
    from dryad_amd.io.providers import provider_for
    n = 800_000
    ctx = D.DryadLinqContext(platform="gpu")
    ctx.HbmBudgetBytes = 48 << 20
    src = f"gen://terasort?records={n}&partitions=1&seed=11"
    ctx.FromStore(src).OrderByDescending(lambda r: r[0:10]).ToStore("host://ooc_desc", delete_if_exists=True) \
        .SubmitAndWait()
    res = ctx._get_executor().last_result
    assert res["external_sort"] is not None and res["external_sort"].buckets > 1 and not res["fallbacks"]
    h = provider_for("host://ooc_desc").local_rows("host://ooc_desc", 0)
    ref = _in_hbm_sorted(_gen_rows(n))
    assert torch.equal(h.rows, ref.flip(0))        # distinct TeraSort keys: exactly the reverse
    provider_for("host://ooc_desc").delete("host://ooc_desc")
