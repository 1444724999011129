"""Fine-bucket exchange over a materialised table (ops/recordsort.send_fine_rows, the ts_pack_rows
kernel): the send-side pack against a torch gather, its error handling, and the per-rank program
of a multi-rank TeraSort (loopback) with the table generated in HBM, read from a partfile, or the
GenFusedShuffle variant.  The multi-rank runs over gloo ranks sharing the GPU are in
tests/test_gpu_multirank.py (tests/dist/gpu_fine_rows_ranks.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _entries(idx: torch.Tensor, window: torch.Tensor) -> torch.Tensor:
    return (window.to(torch.int64) << 32) | idx.to(torch.int64)


@pytest.mark.parametrize("pitch", [100, 128])
def test_pack_rows_matches_gather(pitch):
    from dryad_amd.ops import terasort as TS
    dev = torch.device("cuda")
    n = 300_001
    g = torch.Generator(device="cpu").manual_seed(pitch)
    store = torch.randint(0, 256, (n, pitch), dtype=torch.uint8, generator=g).to(dev)
    rows = store[:, :100]
    perm = torch.randperm(n, generator=g).to(dev)
    ent = _entries(perm, torch.randint(0, 1 << 31, (n,), generator=g).to(dev))
    out = torch.full((n, 100), 0xAB, dtype=torch.uint8, device=dev)
    bad = TS.pack_rows(out, rows, ent, n)
    assert int(bad.item()) == 0
    assert torch.equal(out, rows.index_select(0, perm))
    # segments: out rows [0, 1000) <- entries [5000, 6000), [1000, n - 5000) <- [6000, ...), the
    # rest <- entries [0, 5000): a round-major send buffer over window-sorted entries
    seg = torch.tensor([[0, 5000], [1000, 6000], [n - 5000, 0]], dtype=torch.int64, device=dev)
    q = torch.cat([torch.arange(5000, 6000), torch.arange(6000, n), torch.arange(0, 5000)]).to(dev)
    out.fill_(0)
    TS.pack_rows(out, rows, ent, n, seg=seg)
    assert torch.equal(out, rows.index_select(0, perm.index_select(0, q)))


def test_pack_rows_error_word_and_bad_index():
    from dryad_amd.ops import terasort as TS
    dev = torch.device("cuda")
    n = 70_000
    rows = torch.randint(0, 256, (n, 100), dtype=torch.uint8, device=dev)
    ent = _entries(torch.arange(n, device=dev), torch.zeros(n, dtype=torch.int64, device=dev))
    out = torch.full((n, 100), 7, dtype=torch.uint8, device=dev)
    err = torch.ones(1, dtype=torch.int32, device=dev)           # a failed look-back sort: nothing read
    TS.pack_rows(out, rows, ent, n, err=err)
    assert bool((out == 7).all())
    ent[123] = (ent[123] & ~0xFFFFFFFF) | (n + 5)                   # a row past the table: zero-filled
    bad = TS.pack_rows(out, rows, ent, n)
    assert int(bad.item()) == 1
    assert bool((out[123] == 0).all())
    keep = torch.ones(n, dtype=torch.bool, device=dev)
    keep[123] = False
    assert torch.equal(out[keep], rows[keep])


@pytest.mark.parametrize("mode", ["table", "gen-fused"])
def test_loopback_rank_program(mode):
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortLoopbackJob
    job = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=3_000_000), 4, 2, mode=mode)
    for _ in range(2):
        job.step()
        v = job.validate()
        assert v["ok"], v
        assert 0.8 * job.n < v["records"] < 1.2 * job.n
    assert set(job.phases) == {"input_ms", "sample_ms", "separators_entry_sort_ms", "pack_ms", "receive_sort_ms"}
    assert len(job.rounds["merge_ms"]) == job.B
    if mode == "table":
        # the modelled node step: the overlapped exchange puts round 0 on the wire after one
        # round's pack, the bulk order after all of them
        m = job.model(300.0)
        assert m["modelled"] and m["first_round_queued_ms"] < m["bulk_first_round_queued_ms"], m
        assert m["overlapped_step_ms"] > 0 and m["wire_ms"] > 0, m


def test_loopback_rank_program_from_partfile(tmp_path):
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortLoopbackJob
    uri = f"partfile://{tmp_path}/lb_in"
    job = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=2_000_000), 2, 1, input_uri=uri)
    assert os.path.getsize(job.input) == 2_000_000 * 100
    job.step()
    v = job.validate()
    assert v["ok"], v
    # the same rank program from the generator gives the same output bytes
    ref = TeraSortLoopbackJob(TeraSortConfig(records_per_rank=2_000_000), 2, 1)
    ref.step()
    assert torch.equal(job.out, ref.out)


def test_gather_fixup_reads_nothing_after_a_failed_lookback_sort():
    """Histograms that do not count the entries make the look-back sort give up (err != 0) and
    leave stale entries; the row gather then must not read through them (it used to gather
    first and check the flag afterwards, reading rows far past the table)."""
    from dryad_amd.ops import _lib
    from dryad_amd.ops import sort as S
    dev = torch.device("cuda")
    n = max(S.ONESWEEP_MIN, 1 << 20) + 123
    rows = torch.randint(0, 256, (n, 100), dtype=torch.uint8, device=dev)
    e = S.extract_keys64(rows, 0, 10, 0, torch.empty(n, dtype=torch.int64, device=dev))
    parts = int(_lib.lib().dr_extract_keys64_tile_parts(_lib.c_u64(n)))
    zero_hist = torch.zeros(parts * 1024, dtype=torch.int32, device=dev)
    err = S.lookback_error()
    tmp = torch.full((n,), -1, dtype=torch.int64, device=dev)       # stale entries naming no row
    srt = S.sort_entries64(e, tmp, 32, gen_hist=zero_hist, err=err)
    assert int(err.item()) != 0
    out = torch.full((n, 100), 7, dtype=torch.uint8, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    S.gather_fixup(rows, srt, out, 0, 10, 32, flag, err=err)
    torch.cuda.synchronize()
    assert bool((out == 7).all())
    # the compact row sort over the same rows still ends sorted (its fallback passes)
    got = S.sort_rows_compact(rows, torch.empty_like(rows), torch.empty(n, dtype=torch.int64, device=dev),
                              torch.empty(n, dtype=torch.int64, device=dev), 0, 10)
    keys = got[:, :10].cpu().numpy()
    assert all(bytes(keys[i]) <= bytes(keys[i + 1]) for i in range(0, n - 1, 997))


@pytest.mark.parametrize("key,desc", [("V1", False), ("Key", True)])
def test_records64_loopback_rank_program(key, desc):
    """The per-rank program of a columnar OrderBy (models/records_sort.py) at a small size: packed
    rows through the fine-bucket send side and LDS merge, unpacked, validated (order, fingerprint
    of the received rows, range)."""
    from dryad_amd.models.records_sort import Records64LoopbackJob
    job = Records64LoopbackJob(4, 2, 300_000, key=key, descending=desc, nkeys=50_000, slack=0.2)   # ~300 samples a rank
    job.step()
    v = job.validate()
    assert v["ok"], v
    assert job.rec == 64 and set(job.phases) >= {"pack_columns_ms", "receive_merge_ms", "unpack_ms"}
    m = job.model(300.0)
    assert m["overlapped_step_ms"] > 0 and m["modelled"]
