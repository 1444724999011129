"""Device record-boundary discovery for variable-length parts without an index sidecar
(csrc/kernels/varscan.hip via ops/codec.block_index_device): the offsets of every B-th record
must equal the host scan (codec.cpp scan_record_blocks) for strings, multi-field records and
text lines, at chunk sizes that force multi-chunk walks, strings longer than many chunks, and
streams the speculative parse must decline (then block_index falls back to the host)."""
import random

import numpy as np
import pytest
import torch

from dryad_amd import types as T
from dryad_amd.io import binary as B
from dryad_amd.ops import codec as CD

pytestmark = pytest.mark.gpu

REC = T.RecordT([("a", T.String), ("b", T.Int32), ("c", T.Float64), ("d", T.String), ("e", T.Bool)])


def _rstr(rng, long_frac=0.05):
    n = rng.randint(0, 40) if rng.random() > long_frac else rng.randint(100, 9000)
    return "".join(rng.choice("abcdefghij é€\U0001d11exyz") for _ in range(n))


def _data(kind, seed=1, count=4000):
    rng = random.Random(seed)
    if kind == "strings":
        return T.String, [_rstr(rng) for _ in range(count)]
    if kind == "records":
        return REC, [(_rstr(rng), rng.randint(-5, 10 ** 6), rng.random(), _rstr(rng), rng.random() < .5)
                     for _ in range(count)]
    if kind == "lines":
        return T.LineRecordT, [T.LineRecord("line %d %s" % (i, "x" * (i % 50))) for i in range(count)]
    if kind == "regular":
        return REC, [(str(i), i, 0.5, "y" * (i % 7), True) for i in range(count)]
    raise KeyError(kind)


def _check(dt, recs, chunk, block=64):
    data = B.encode_records(dt, recs)
    n, offs = CD.block_index_host(np.frombuffer(data, dtype=np.uint8), dt, block)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    got = CD.block_index_device(buf, dt, block, chunk)
    assert got is not None, "device scan declined a well-formed stream"
    assert got[0] == n == len(recs)
    assert torch.equal(got[1].cpu(), torch.from_numpy(offs))
    return buf, n, got[1]


@pytest.mark.parametrize("kind", ["strings", "records", "lines", "regular"])
@pytest.mark.parametrize("chunk", [32, 256, 4096])
def test_device_boundaries_equal_host_scan(kind, chunk):
    dt, recs = _data(kind)
    _check(dt, recs, chunk)


def test_decode_with_device_index_round_trips():
    dt, recs = _data("records", seed=7)
    buf, n, offs = _check(dt, recs, 4096, CD.BLOCK)
    t = CD.decode_var(buf, dt, n, offs)
    enc, _ = CD.encode_var(t, dt)
    assert torch.equal(enc, buf)


def test_edge_sizes():
    for recs in ([], ["a"], [""], ["z" * 50000], ["q" * 5000, "", "r" * 70000, "s"]):
        data = B.encode_records(T.String, recs)
        buf = torch.frombuffer(bytearray(data) or bytearray(1), dtype=torch.uint8).cuda()[: len(data)]
        got = CD.block_index_device(buf, T.String, 2, 64)
        assert got is not None and got[0] == len(recs)
        n, offs = CD.block_index_host(np.frombuffer(data, dtype=np.uint8), T.String, 2)
        assert torch.equal(got[1].cpu(), torch.from_numpy(offs))


def test_irregular_stream_falls_back_to_host():
    # a byte count the writer would never pair with its unit count (bytes < units): the device
    # parse declines, block_index still returns the host scan's index
    data = bytes([5, 2]) + b"ab" + B.encode_records(T.String, ["hello", "world"])
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    assert CD.block_index_device(buf, T.String, 1, 32) is None
    n, offs, _ = CD.block_index(buf, T.String, 1)
    assert n == 3 and offs.cpu().tolist() == [0, 4, 11]
