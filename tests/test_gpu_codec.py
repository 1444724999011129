"""Device DryadLinqBinary codec (fixed-width records) vs the host encoder, and partfile
round trips through the GPU executor (parallel part writes + device decode on read)."""
import pytest
import torch

import dryad_amd as D
from dryad_amd import types as T

pytestmark = pytest.mark.gpu


def test_encode_decode_match_host_codec():
    from dryad_amd.io import binary as B
    from dryad_amd.ops import codec as CD
    from dryad_amd.gpu.table import from_objects
    dt = T.RecordT([("a", T.Int32), ("b", T.Int64), ("c", T.Float64), ("d", T.Byte), ("e", T.Int16)], tuple)
    recs = [(i, i * 1_000_003 - 7, i / 3.0, i % 256, -i % 1000) for i in range(5000)]
    host = B.encode_records(dt, recs)
    t = from_objects(recs, dt, "cuda")
    dev = CD.encode(t, dt)
    assert dev.cpu().numpy().tobytes() == host
    back = CD.decode(torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda(), dt)
    assert back.to_objects() == recs


def test_partfile_roundtrip_on_gpu_executor(tmp_path):
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = 3
    uri = f"partfile://{tmp_path}/t.pt"
    data = [(i, float(i) * 0.5) for i in range(30_000)]
    g.FromEnumerable(data).Select(lambda t: (t[0] * 2, t[1] + 1.0)).ToStore(uri).SubmitAndWait()
    back = sorted(g.FromStore(uri).Where(lambda t: t[0] % 4 == 0))
    exp = sorted((a * 2, b + 1.0) for a, b in data if (a * 2) % 4 == 0)
    assert back == exp
    fb = {op for _, op, _ in g._get_executor().last_result["fallbacks"]}
    assert "read" not in fb and "where" not in fb
    # the files are ordinary DryadLinqBinary partfiles: the CPU executor reads them too
    c = D.DryadLinqContext(2)
    assert sorted(c.FromStore(uri)) == sorted((a * 2, b + 1.0) for a, b in data)


@pytest.mark.parametrize("n,start,wide", [(1, 0, False), (255, 3, False), (70_001, 5, False), (3000, 1, True)])
def test_tiled_codec_any_alignment_and_width(n, start, wide):
    """LDS-tiled decode / encode (records of <= 128 bytes; wider ones take the per-field kernel)
    of a part starting at any byte offset, against the host codec."""
    import numpy as np
    from dryad_amd.io import binary as B
    from dryad_amd.ops import codec as CD
    fields = [("a", T.Int16), ("b", T.Int64), ("c", T.Byte), ("d", T.Float64), ("e", T.Int32)]
    if wide:
        fields += [(f"w{i}", T.Int64) for i in range(16)]
    dt = T.RecordT(fields, tuple)
    rng = np.random.default_rng(n)
    recs = [tuple(int(rng.integers(-3000, 3000)) if ft in (T.Int16, T.Int32, T.Int64) else
                  int(rng.integers(0, 256)) if ft is T.Byte else float(rng.standard_normal())
                  for _, ft in fields) for _ in range(n)]
    host = B.encode_records(dt, recs)
    buf = torch.zeros(len(host) + start + 16, dtype=torch.uint8, device="cuda")
    buf[start:start + len(host)] = torch.frombuffer(bytearray(host), dtype=torch.uint8).cuda()
    t = CD.decode(buf[start:start + len(host)], dt)
    assert t.to_objects() == recs
    enc = CD.encode(t, dt)
    assert enc.cpu().numpy().tobytes() == host
