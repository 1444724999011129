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
