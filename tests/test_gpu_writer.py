"""HBM -> part file through the native writer (io/writer.py): byte-exact from device tensors of
several chunks, and the executor's partfile commit going through it."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_write_device_chunks(tmp_path, monkeypatch):
    from dryad_amd.io import writer as WR
    monkeypatch.setattr(WR, "CHUNK", 1 << 20)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(0, 256, (5 * (1 << 20) + 12345,), dtype=torch.uint8, device="cuda", generator=g)
    p = str(tmp_path / "d.bin")
    st = WR.WriteStats()
    assert WR.write_device(p, x, st) == x.numel()
    assert np.array_equal(np.fromfile(p, dtype=np.uint8), x.cpu().numpy())
    assert st.bytes == x.numel() and st.seconds > 0


def test_partfile_output_written_natively(tmp_path):
    import dryad_amd as D
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 2
    uri = "partfile://" + str(tmp_path / "o.pt")
    src = "gen://records64?count=300000&partitions=2&keys=1000&seed=3"
    c.FromStore(src).Where(lambda r: r[1] % 3 == 0).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    res = c._get_executor().last_result
    assert res["write"]["bytes"] > 0
    got = sorted(c.FromStore(uri))
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    exp = sorted(loc.FromStore(src).Where(lambda r: r[1] % 3 == 0))
    assert got == exp


def test_write_device_pieces_to_several_files(tmp_path, monkeypatch):
    from dryad_amd.io import writer as WR
    monkeypatch.setattr(WR, "CHUNK", 1 << 20)
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randint(0, 256, (7 * (1 << 20) + 4321,), dtype=torch.uint8, device="cuda", generator=g)
    bounds = [0, 3 * (1 << 20) + 100, 3 * (1 << 20) + 100, 6 * (1 << 20), x.numel()]   # one empty file
    paths = [str(tmp_path / f"p{j}") for j in range(4)]
    st = WR.WriteStats()
    sizes = WR.write_device_pieces(paths, x, bounds, st)
    assert sizes == [bounds[j + 1] - bounds[j] for j in range(4)]
    h = x.cpu().numpy()
    for j in range(4):
        assert np.array_equal(np.fromfile(paths[j], dtype=np.uint8), h[bounds[j]: bounds[j + 1]])
    assert st.bytes == x.numel()


def test_partfile_output_split_into_part_files(tmp_path):
    """PartFileSplitBytes: each partition written as several part files at once, in order."""
    import dryad_amd as D
    from dryad_amd.io import partfile as PF
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 2
    c.PartFileSplitBytes = 1 << 20
    uri = "partfile://" + str(tmp_path / "s.pt")
    src = "gen://records64?count=300000&partitions=2&keys=100000&seed=4"
    c.FromStore(src).OrderBy(lambda r: r[0]).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    meta = PF.read_meta(str(tmp_path / "s.pt"))
    assert meta.count > 2
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    got = list(loc.FromStore(uri))                # part order = the sorted order
    exp = list(loc.FromStore(src).OrderBy(lambda r: r[0]))
    assert [r[0] for r in got] == [r[0] for r in exp]
    assert sorted(got) == sorted(exp)


def test_stored_terasort_split_output(tmp_path):
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortStoredJob
    from dryad_amd.parallel.comm import init_world
    w = init_world(device="cuda")
    job = TeraSortStoredJob(TeraSortConfig(records_per_rank=1_000_000), w, f"partfile://{tmp_path}/in",
                            f"partfile://{tmp_path}/out")
    job.ctx.PartFileSplitBytes = 16 << 20          # 100 MB of rows -> 5 part files
    job.prepare()
    expect = job.input_checksum()
    job.step()
    val = job.validate(*expect)
    assert val["ok"] and val["parts"] == 5, val         # 1e8 bytes // 16 MiB
