"""Stored-data TeraSort (models/terasort.TeraSortStoredJob, bench.py --input): a partfile of raw
100-byte rows written from the generator by the device writer, read back through the native
chunked reader at a 128-byte pitch, sorted by the compact pitch-128 sort from entries extracted
right after the read, and written as a partfile: valsort-validated, with the read / write byte
counts of the job reported."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_read_rows_pitched_matches_contiguous(tmp_path):
    from dryad_amd.io import reader as RD
    n, w = 700_001, 100
    data = torch.randint(0, 256, (n, w), dtype=torch.uint8)
    p = tmp_path / "rows.bin"
    p.write_bytes(b"\0" * 37 + data.numpy().tobytes())
    big = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
    view = big[:, :w]
    old = RD.CHUNK
    try:
        RD.CHUNK = 1 << 20                       # many chunks, rows straddling the 64 MB default
        RD.read_rows_to_device(str(p), "cuda", 37, n, w, view)
    finally:
        RD.CHUNK = old
    assert torch.equal(view.cpu(), data)
    assert int(big[:, w:].sum().item()) == 0


def test_reads_after_a_chunk_change_stay_inside_the_ring(tmp_path):
    """The pinned ring is created once, at the CHUNK of its first use; a later, larger CHUNK must
    not make the native reader write past its buffers (it did: a segfault in the next job)."""
    from dryad_amd.io import reader as RD
    old, old_ring = RD.CHUNK, RD._RING
    try:
        RD._RING = None
        RD.CHUNK = 1 << 20
        RD._ring()                               # the ring at 1 MB buffers
        RD.CHUNK = old
        n, w = 40_000, 100                       # 4 MB: several 1 MB chunks
        data = torch.randint(0, 256, (n, w), dtype=torch.uint8)
        p = tmp_path / "rows.bin"
        p.write_bytes(data.numpy().tobytes())
        flat = RD.read_to_device(str(p), "cuda")
        assert torch.equal(flat.cpu(), data.view(-1))
        big = torch.zeros((n, 128), dtype=torch.uint8, device="cuda")
        RD.read_rows_to_device(str(p), "cuda", 0, n, w, big[:, :w])
        assert torch.equal(big[:, :w].cpu(), data)
    finally:
        RD.CHUNK = old
        RD._RING = old_ring


def test_stored_terasort_end_to_end(tmp_path):
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortStoredJob
    from dryad_amd.parallel.comm import init_world
    w = init_world(device="cuda")
    cfg = TeraSortConfig(records_per_rank=3_000_000)
    job = TeraSortStoredJob(cfg, w, f"partfile://{tmp_path}/in", f"partfile://{tmp_path}/out")
    prep = job.prepare()
    assert prep["reused"] is False
    assert job.prepare()["reused"] is True       # a table of this size is reused
    expect = job.input_checksum()
    job.step()
    val = job.validate(*expect)
    assert val["ok"], val
    rep = job.report()
    assert rep["read_GB"] == pytest.approx(3e6 * 100 / 1e9, rel=1e-6)
    assert rep["write_GB"] == pytest.approx(3e6 * 100 / 1e9, rel=1e-6)
    assert rep["sort_path"] and "pitch128" in rep["sort_path"], rep
    assert not rep["fallbacks"], rep
    assert os.path.exists(f"{tmp_path}/out")
    torch.cuda.synchronize()
