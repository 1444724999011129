"""Native part writer (csrc/runtime/partwriter.cpp + io/writer.py) from host data (CPU; the
device path is covered by tests/test_gpu_writer.py)."""
import os

import numpy as np
import pytest
import torch

from dryad_amd.io import writer as WR


@pytest.mark.parametrize("mapped", [False, True])
def test_part_writer_host_chunks(tmp_path, monkeypatch, mapped):
    monkeypatch.setattr(WR, "CHUNK", 1 << 16)           # many chunks through a small ring
    monkeypatch.setattr(WR, "MAPPED", mapped)           # pwrite() and shared-mapping writers
    p = str(tmp_path / "part.bin")
    rng = np.random.default_rng(2)
    pieces = [rng.integers(0, 256, size=n, dtype=np.uint8) for n in (0, 1, 65535, 65536, 300_001, 7)]
    st = WR.WriteStats()
    with WR.PartWriter(p, None, st) as w:
        for x in pieces:
            w.write(torch.from_numpy(x))
        w.write(b"tail")
    exp = b"".join(x.tobytes() for x in pieces) + b"tail"
    assert os.path.getsize(p) == len(exp) and open(p, "rb").read() == exp
    assert st.bytes == len(exp)


def test_part_writer_abort_releases_ring(tmp_path):
    p = str(tmp_path / "a.bin")
    try:
        with WR.PartWriter(p) as w:
            w.write(b"x" * 100)
            raise KeyError("boom")
    except KeyError:
        pass
    WR.write_device(str(tmp_path / "b.bin"), torch.arange(10, dtype=torch.uint8))   # the ring is free again
    assert open(str(tmp_path / "b.bin"), "rb").read() == bytes(range(10))
