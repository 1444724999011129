"""Byte-format tests: DryadLinqBinary record encoding (golden bytes derived from the reference
writer's rules, DryadLinqBinaryWriter.cs), the native C++ codec against the Python codec, the
partfile format (DrPartitionFile.cpp / DataProvider.cs) and Rabin fingerprints."""
import datetime
import decimal
import uuid

import numpy as np
import pytest

import dryad_amd as D
from dryad_amd import types as T
from dryad_amd.io import binary as B
from dryad_amd.io import partfile as PF
from dryad_amd.native import runtime


def enc(dtype, v):
    return B.encode_records(dtype, [v])


def test_primitives_little_endian():
    assert enc(T.Int32, 1) == b"\x01\x00\x00\x00"
    assert enc(T.Int32, -2) == b"\xfe\xff\xff\xff"
    assert enc(T.Int64, 2**40) == (2**40).to_bytes(8, "little")
    assert enc(T.Int16, -1) == b"\xff\xff"
    assert enc(T.Bool, True) == b"\x01"
    assert enc(T.Float64, 1.5) == np.float64(1.5).tobytes()
    assert enc(T.Float32, -0.25) == np.float32(-0.25).tobytes()
    assert enc(T.Byte, 255) == b"\xff" and enc(T.SByte, -1) == b"\xff"


def test_compact_int():
    w = B.BinaryWriter()
    for v in (0, 1, 0x7F, 0x80, 0x1234, 2**30):
        w.write_compact(v)
    b = w.getvalue()
    assert b[:3] == b"\x00\x01\x7f"
    assert b[3:7] == b"\x80\x00\x00\x80"
    assert b[7:11] == b"\x80\x00\x12\x34"
    r = B.BinaryReader(b)
    assert [r.read_compact() for _ in range(6)] == [0, 1, 0x7F, 0x80, 0x1234, 2**30]


def test_string_encoding_width_rule():
    # short string: char count 1 byte, byte count 1 byte ((len+1)*3 < 0x80)
    assert enc(T.String, "ab") == b"\x02\x02ab"
    # 41 chars -> max bytes 126 < 128 -> 1-byte count; 42 chars -> 129 -> 4-byte count
    s41, s42 = "x" * 41, "y" * 42
    assert enc(T.String, s41)[:2] == b"\x29\x29"
    e = enc(T.String, s42)
    assert e[:1] == b"\x2a" and e[1:5] == b"\x80\x00\x00\x2a" and e[5:] == s42.encode()
    # non-ASCII: UTF-16 unit count vs UTF-8 byte count; astral chars count 2 units
    e = enc(T.String, "é😀")
    assert e[0] == 3 and e[1] == len("é😀".encode())
    for s in ["", "a", "hello world", "é😀" * 30, "z" * 1000]:
        assert B.decode_records(T.String, enc(T.String, s)) == [s]


def test_datetime_decimal_guid():
    d = datetime.datetime(2001, 2, 3, 4, 5, 6, 789000)
    b = enc(T.DateTime, d)
    ticks = int.from_bytes(b, "little")
    assert ticks == ((d - datetime.datetime(1, 1, 1)).days * 86400 + 4 * 3600 + 5 * 60 + 6) * 10**7 + 7890000
    assert B.decode_records(T.DateTime, b) == [d]
    g = uuid.UUID("12345678-1234-5678-1234-567812345678")
    assert enc(T.Guid, g) == g.bytes_le
    for v in ["0", "1.5", "-123456789.000001", "79228162514264337593543950335"]:
        x = decimal.Decimal(v)
        assert B.decode_records(T.Decimal, enc(T.Decimal, x)) == [x]
    assert len(enc(T.Decimal, decimal.Decimal("1.5"))) == 16


def test_record_types_and_nullable_bitvector():
    import dataclasses
    import typing

    @dataclasses.dataclass
    class R:
        a: int
        s: typing.Optional[str]
        f: float

    dt = T.record_type(R)
    assert dt.nullable_fields == {"s"}
    b = B.encode_records(dt, [R(1, None, 2.0), R(2, "x", 3.0)])
    # first record: bitvector len 1, bit 1 set (field s null) ; then a (int64) and f
    assert b[:2] == b"\x01\x02"
    out = B.decode_records(dt, b)
    assert out == [R(1, None, 2.0), R(2, "x", 3.0)]
    tup = T.infer_type((1, "a", 2.5))
    assert B.decode_records(tup, B.encode_records(tup, [(1, "a", 2.5)])) == [(1, "a", 2.5)]


def test_native_codec_matches_python_codec():
    R = runtime()
    rng = np.random.default_rng(0)
    strs = ["", "a", "héllo", "x" * 50, "😀" * 3] * 20
    ints = rng.integers(-2**31, 2**31, len(strs)).astype(np.int32)
    flts = rng.random(len(strs))
    recs = list(zip(ints.tolist(), strs, flts.tolist()))
    dt = T.RecordT([("i", T.Int32), ("s", T.String), ("f", T.Float64)], tuple)
    py = B.encode_records(dt, recs)
    off = np.zeros(len(strs) + 1, dtype=np.int64)
    data = b"".join(s.encode() for s in strs)
    off[1:] = np.cumsum([len(s.encode()) for s in strs])
    nat = R.encode_records(len(recs), [5, 14, 10], [ints, (off, np.frombuffer(data, np.uint8)), flts])
    assert nat == py
    n, cols = R.decode_records(py, [5, 14, 10])
    assert n == len(recs)
    assert np.array_equal(cols[0].view(np.int32), ints)
    assert bytes(cols[1][1]) == data and np.array_equal(cols[1][0], off)
    assert np.array_equal(cols[2].view(np.float64), flts)


def test_native_lines_to_records():
    R = runtime()
    text = b"alpha\nbeta\r\ngamma\rdelta"
    b = R.lines_to_records(text)
    assert B.decode_records(T.String, b) == ["alpha", "beta", "gamma", "delta"]
    st, en = R.split_lines(b"a\n\nb")
    assert list(st) == [0, 2, 3] and list(en) == [1, 2, 4]


def test_partfile_roundtrip(tmp_path):
    meta = str(tmp_path / "tbl")
    base = PF.default_base(meta)
    import os
    os.makedirs(os.path.dirname(base), exist_ok=True)
    tmps = []
    for i, recs in enumerate([[1, 2], [3], []]):
        p = PF.tmp_part_path(base, i, 7, 0, 1)
        B.write_records(p, T.Int32, recs)
        tmps.append(p)
    m = PF.commit_parts(meta, base, tmps)
    text = open(meta).read().splitlines()
    assert text[0] == base and text[1] == "3" and text[2] == "0,8" and text[3] == "1,4" and text[4] == "2,0"
    m2 = PF.read_meta(meta)
    assert m2.paths() == [f"{base}.00000000", f"{base}.00000001", f"{base}.00000002"]
    assert [B.read_records(p, T.Int32) for p in m2.paths()] == [[1, 2], [3], []]
    # machine:override column
    PF.write_meta(meta, PF.PartFileMeta(base, [PF.PartEntry(0, 8, "host1", "/abs/override")]))
    assert PF.read_meta(meta).part_path(0) == "/abs/override"


def _py_rabin_table(poly):
    tab = [0] * 256
    f = poly
    i = 0x80
    while i:
        tab[i] = f
        f = (f >> 1) ^ (poly if f & 1 else 0)
        i >>= 1
    i = 1
    while i < 256:
        for k in range(1, i):
            tab[i + k] = tab[i] ^ tab[k]
        i <<= 1
    return tab


def test_rabin_fingerprint_matches_definition():
    R = runtime()
    r = R.Rabin64()
    poly = r.empty()
    tab = _py_rabin_table(poly)
    assert list(r.table(0).astype(object)) == tab
    data = b"The quick brown fox"
    fp = poly
    for x in data:
        fp = (fp >> 8) ^ tab[(fp & 0xFF) ^ x]
    assert r.extend(poly, data) == fp
    # word-wise extension equals byte-wise extension of the little-endian bytes
    v = 0x0123456789ABCDEF
    assert r.extend_u64(poly, v) == r.extend(poly, v.to_bytes(8, "little"))
    assert r.extend_u32(poly, 0xDEADBEEF) == r.extend(poly, (0xDEADBEEF).to_bytes(4, "little"))


def test_output_gzip_compression_roundtrip(tmp_path):
    import gzip
    import dryad_amd as D
    from dryad_amd.context import CompressionScheme
    from dryad_amd.io import partfile as PF
    c = D.DryadLinqContext(2)
    c.OutputDataCompressionScheme = CompressionScheme.GZIP
    uri = f"partfile://{tmp_path}/z.pt"
    data = [(i, i * 0.25) for i in range(5000)]
    c.FromEnumerable(data).ToStore(uri).SubmitAndWait()
    part = PF.read_meta(str(tmp_path / "z.pt")).part_path(0)
    raw = open(part, "rb").read()
    assert raw[:2] == b"\x1f\x8b" and len(gzip.decompress(raw)) > len(raw)
    assert sorted(D.DryadLinqContext(2).FromStore(uri)) == data
