"""Replaced partfile tables recycle their part files (io/partfile.py RECYCLE_DIR): the parts of a
table deleted in the background move to the recycle directory, new part files claim them by
rename, and the native writer overwrites them in place (reuse=True) and cuts them to size."""
import os
import time

import torch

from dryad_amd.io import partfile as PF
from dryad_amd.io import writer as WR


def _table(tmp_path, name, sizes):
    meta = str(tmp_path / name)
    base = PF.default_base(meta)
    os.makedirs(os.path.dirname(base), exist_ok=True)
    chosen = []
    for i, n in enumerate(sizes):
        p = f"{base}.{i:08X}.tmp"
        with open(p, "wb") as f:
            f.write(bytes([i + 1]) * n)
        chosen.append(p)
    PF.commit_parts(meta, base, chosen)
    return meta, base


def test_background_delete_recycles_parts_and_writer_reuses_them(tmp_path):
    meta, base = _table(tmp_path, "t", [3000, 5000, 4000])
    PF.delete(meta, background=True)
    assert not os.path.exists(meta)
    rdir = os.path.join(os.path.dirname(base), PF.RECYCLE_DIR)
    assert sorted(os.path.getsize(os.path.join(rdir, f)) for f in os.listdir(rdir)) == [3000, 4000, 5000]
    new = [f"{base}.new.{j}" for j in range(2)]
    assert PF.claim_recycled(new) == 2
    assert sorted(os.path.getsize(p) for p in new) == [4000, 5000]         # the largest first
    assert len(os.listdir(rdir)) == 1
    data = torch.arange(1000, dtype=torch.int32).view(torch.uint8)       # 4000 bytes
    sizes = WR.write_device_pieces(new, data, [0, 1500, 4000], reuse=True)
    assert sizes == [1500, 2500]
    got = open(new[0], "rb").read() + open(new[1], "rb").read()
    assert got == bytes(data.numpy())


def test_claim_skips_existing_paths_and_empty_pool(tmp_path):
    meta, base = _table(tmp_path, "u", [100])
    PF.delete(meta, background=True)
    existing = f"{base}.x.0"
    with open(existing, "wb") as f:
        f.write(b"keep")
    assert PF.claim_recycled([existing, f"{base}.x.1", f"{base}.x.2"]) == 1
    assert open(existing, "rb").read() == b"keep"
    assert os.path.getsize(f"{base}.x.1") == 100
    assert not os.path.exists(f"{base}.x.2")
    assert PF.claim_recycled([f"{base}.y.0"]) == 0


def test_sweep_removes_stale_recycled_files(tmp_path):
    d = tmp_path / PF.RECYCLE_DIR
    d.mkdir()
    old = d / f"r-{int((time.time() - 1000) * 1e3)}-abc-0"
    fresh = d / f"r-{int(time.time() * 1e3)}-def-0"
    old.write_bytes(b"x")
    fresh.write_bytes(b"y")
    PF._sweep(str(d), 600)
    assert not old.exists() and fresh.exists()


def test_drop_recycled_unlinks_unclaimed(tmp_path):
    meta, base = _table(tmp_path, "v", [100, 200])
    PF.delete(meta, background=True)
    rdir = os.path.join(os.path.dirname(base), PF.RECYCLE_DIR)
    assert len(os.listdir(rdir)) == 2
    PF.drop_recycled(base)
    for _ in range(100):
        if not os.listdir(rdir):
            break
        time.sleep(0.02)
    assert os.listdir(rdir) == []
