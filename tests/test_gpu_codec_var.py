"""Device codec for variable-length records (csrc/kernels/codec.hip) and the chunked pinned
reader (csrc/runtime/partreader.cpp + io/reader.py): byte-identical round trips against the host
DryadLinqBinary codec (io/binary.py), partfile tables with strings read on the device."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _records(n, seed=3):
    rng = np.random.default_rng(seed)
    alpha = list("abcdefghij") + ["é", "ß", "中", "文", "😀", "\U0001F680", " "]
    out = []
    for i in range(n):
        k = int(rng.integers(0, 4))
        ln = [0, 3, 60, 300][k]                         # 300 chars: 4-byte compact lengths
        s = "".join(alpha[j] for j in rng.integers(0, len(alpha), size=ln))
        t = "".join(alpha[j] for j in rng.integers(0, len(alpha), size=int(rng.integers(0, 8))))
        out.append((s, int(rng.integers(-2**31, 2**31)), float(rng.standard_normal()), t, bool(i % 3)))
    return out


def _dtype():
    from dryad_amd import types as T
    return T.RecordT([("a", T.String), ("b", T.Int32), ("c", T.Float64), ("d", T.String), ("e", T.Bool)])


def test_var_codec_round_trip_bytes_identical():
    from dryad_amd.io import binary as B
    from dryad_amd.ops import codec as CD
    dt = _dtype()
    recs = _records(5000)
    data = B.encode_records(dt, recs)
    n, offs = CD.block_index_host(np.frombuffer(data, dtype=np.uint8), dt)
    assert n == len(recs)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    t = CD.decode_var(buf, dt, n, torch.from_numpy(offs).cuda())
    assert t.to_objects() == recs
    enc, boffs = CD.encode_var(t, dt)
    assert bytes(enc.cpu().numpy()) == data
    assert np.array_equal(boffs.cpu().numpy(), offs)


def test_var_codec_line_records_and_index_mismatch():
    from dryad_amd import types as T
    from dryad_amd.io import binary as B
    from dryad_amd.ops import codec as CD
    lines = [T.LineRecord(x) for x in ["", "a b", "x" * 200, "中文 text", "😀 ok"] * 300]
    data = B.encode_records(T.LineRecordT, lines)
    n, offs = CD.block_index_host(np.frombuffer(data, dtype=np.uint8), T.LineRecordT)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    t = CD.decode_var(buf, T.LineRecordT, n, torch.from_numpy(offs).cuda())
    assert [r.Line for r in t.to_objects()] == [r.Line for r in lines]
    enc, _ = CD.encode_var(t, T.LineRecordT)
    assert bytes(enc.cpu().numpy()) == data
    bad = torch.from_numpy(offs + 1).cuda()            # a wrong index is detected, not trusted
    with pytest.raises(CD.DecodeError):
        CD.decode_var(buf, T.LineRecordT, n, bad)


def test_chunked_reader_to_device(tmp_path):
    from dryad_amd.io import reader as RD
    p = str(tmp_path / "blob.bin")
    data = np.random.default_rng(1).integers(0, 256, size=3 * RD.CHUNK + 12345, dtype=np.uint8)
    data.tofile(p)
    st = RD.ReadStats()
    out = RD.read_to_device(p, "cuda", stats=st)
    assert st.chunks == 4 and torch.equal(out.cpu(), torch.from_numpy(data))
    part = RD.read_to_device(p, "cuda", offset=RD.CHUNK - 7, length=RD.CHUNK + 11)
    assert torch.equal(part.cpu(), torch.from_numpy(data[RD.CHUNK - 7:2 * RD.CHUNK + 4]))


def test_partfile_strings_read_on_device(tmp_path):
    """A partfile table with string fields (written with its block index) is decoded on the
    device with no host fallback; without the index the host scan supplies it."""
    import dryad_amd as D
    from dryad_amd.io import partfile as PF
    from dryad_amd.io.providers import provider_for
    dt = _dtype()
    recs = _records(20000, seed=9)
    uri = "partfile://" + str(tmp_path / "tbl.pt")
    provider_for(uri).write_table(uri, [recs[:7000], recs[7000:]], dt)
    meta = PF.read_meta(str(tmp_path / "tbl.pt"))
    assert PF.read_index(meta.part_path(0)) is not None
    for drop_index in (False, True):
        if drop_index:
            os.remove(meta.part_path(1) + PF.INDEX_SUFFIX)
        c = D.DryadLinqContext(platform="gpu")
        c.PartitionCount = 2
        got = list(c.FromStore(uri, dtype=dt).Where(lambda r: r[1] > 0).Select(lambda r: (r[0], r[3], r[1])))
        exp = [(r[0], r[3], r[1]) for r in recs if r[1] > 0]
        assert sorted(got) == sorted(exp)
        assert not c._get_executor().last_result["fallbacks"], c._get_executor().last_result["fallbacks"]


def test_wordcount_on_partfile_line_records(tmp_path):
    import dryad_amd as D
    from collections import Counter
    from dryad_amd import types as T
    from dryad_amd.io.providers import provider_for
    from dryad_amd.models.wordcount import synthetic_corpus, word_count_query
    txt = str(tmp_path / "c.txt")
    synthetic_corpus(txt, 20000)
    with open(txt) as f:
        lines = f.read().split("\n")[:-1]
    uri = "partfile://" + str(tmp_path / "wc.pt")
    provider_for(uri).write_table(uri, [[T.LineRecord(x) for x in lines[i::3]] for i in range(3)], T.LineRecordT)
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 3
    res = dict(word_count_query(c, uri))
    assert res == dict(Counter(" ".join(lines).split()))
    assert not c._get_executor().last_result["fallbacks"]


def test_tampered_index_sidecar_is_rebuilt(tmp_path):
    """A sidecar whose offsets are in bounds but wrong (one block start moved by a byte) decodes
    to a DecodeError, which the read turns into a rebuilt index: the query result is exact."""
    import dryad_amd as D
    from dryad_amd.io import partfile as PF
    from dryad_amd.io.providers import provider_for
    dt = _dtype()
    recs = _records(9000, seed=4)
    uri = "partfile://" + str(tmp_path / "tam.pt")
    provider_for(uri).write_table(uri, [recs], dt)
    part = PF.read_meta(str(tmp_path / "tam.pt")).part_path(0)
    n, nb, blk, offs = PF.read_index(part)
    assert offs.shape[0] >= 3
    offs = offs.copy()
    offs[1] += 1
    PF.write_index(part, n, nb, offs, blk)
    assert PF.read_index(part) is not None          # plausible on its face
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 1
    got = list(c.FromStore(uri, dtype=dt).Select(lambda r: (r[0], r[1])))
    assert got == [(r[0], r[1]) for r in recs]
