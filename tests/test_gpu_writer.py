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
