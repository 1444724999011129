"""Byte-compatible ``DryadLinqBinaryWriter`` / ``DryadLinqBinaryReader`` (record wire format).

Format (reference LinqToDryad/DryadLinqBinaryWriter.cs:256-649, DryadLinqBinaryReader.cs:341-700):
  * byte/sbyte/bool: 1 byte; short/ushort 2; int/uint 4; long/ulong 8 — little endian
  * float/double: IEEE bits as uint32/uint64
  * char: UTF-8 encoding of the single UTF-16 code unit
  * decimal: the 16 raw bytes of System.Decimal (flags, hi, lo, mid as int32 LE)
  * DateTime: ticks | kind << 62 as uint64; SqlDateTime: DayTicks, TimeTicks as int32
  * Guid: 16 raw bytes (= uuid.bytes_le)
  * compact int: 1 byte if val < 0x80 else 4 bytes big-endian with the top bit set
  * string: compact(#UTF-16 code units) + compact(#UTF-8 bytes) whose width (1 or 4 bytes) is
    chosen from the *maximum* byte count (len+1)*3, then the UTF-8 bytes
Streams are concatenations of records; 256 KiB blocks are an I/O artefact only.

The pure-Python codec is the reference implementation (and the LocalDebug / object-executor path);
the C++ runtime (``_dryad_native.Codec``) and the GPU decode kernels must produce identical bytes.
"""
from __future__ import annotations

import datetime as _dt
import decimal as _decimal
import io
import struct
import uuid as _uuid

from ..errors import DryadLinqException, ErrorCode
from ..types import SqlDateTime

DEFAULT_BLOCK_SIZE = 256 * 1024
_EPOCH = _dt.datetime(1, 1, 1)
_KIND_SHIFT = 62

_S = {k: struct.Struct("<" + k) for k in "bBhHiIqQfd"}


def compact_size(val: int) -> int:
    return 1 if val < 0x80 else 4


def utf16_len(s: str) -> int:
    n = len(s)
    for ch in s:
        if ord(ch) > 0xFFFF:
            n += 1
    return n


def max_utf8_bytes(nchars: int) -> int:
    """System.Text.UTF8Encoding.GetMaxByteCount."""
    return (nchars + 1) * 3


def datetime_to_ticks(v: _dt.datetime) -> int:
    kind = 0
    if v.tzinfo is not None:
        kind = 1 if v.utcoffset() == _dt.timedelta(0) else 2
        v = v.replace(tzinfo=None)
    d = v - _EPOCH
    ticks = (d.days * 86400 + d.seconds) * 10_000_000 + d.microseconds * 10
    return ticks | (kind << _KIND_SHIFT)


def ticks_to_datetime(u: int) -> _dt.datetime:
    kind = (u >> _KIND_SHIFT) & 3
    ticks = u & ((1 << _KIND_SHIFT) - 1)
    v = _EPOCH + _dt.timedelta(microseconds=ticks // 10)
    if kind == 1:
        v = v.replace(tzinfo=_dt.timezone.utc)
    return v


def decimal_to_bytes(v: _decimal.Decimal) -> bytes:
    sign, digits, exp = v.as_tuple()
    if not isinstance(exp, int):
        raise DryadLinqException(ErrorCode.TypeNotSerializable, "non-finite decimal")
    mant = int("".join(map(str, digits)) or "0")
    scale = -exp if exp < 0 else 0
    if exp > 0:
        mant *= 10 ** exp
    while mant >= (1 << 96) and scale > 0:
        mant //= 10
        scale -= 1
    if scale > 28:
        mant //= 10 ** (scale - 28)
        scale = 28
    flags = (scale << 16) | (0x80000000 if sign else 0)
    lo, mid, hi = mant & 0xFFFFFFFF, (mant >> 32) & 0xFFFFFFFF, (mant >> 64) & 0xFFFFFFFF
    return struct.pack("<IIII", flags, hi, lo, mid)


def bytes_to_decimal(b: bytes) -> _decimal.Decimal:
    flags, hi, lo, mid = struct.unpack("<IIII", b)
    mant = (hi << 64) | (mid << 32) | lo
    scale = (flags >> 16) & 0xFF
    sign = 1 if flags & 0x80000000 else 0
    return _decimal.Decimal((sign, tuple(int(c) for c in str(mant)), -scale))


class BinaryWriter:
    """Writes records into an in-memory buffer, flushing whole blocks to ``stream`` if given."""

    def __init__(self, stream=None, block_size: int = DEFAULT_BLOCK_SIZE):
        self._buf = bytearray()
        self._stream = stream
        self._block = block_size
        self.bytes_written = 0

    # -- primitives
    def _p(self, fmt, v):
        self._buf += _S[fmt].pack(v)

    def write_byte(self, v): self._buf.append(v & 0xFF)
    def write_sbyte(self, v): self._p("b", v)
    def write_bool(self, v): self._buf.append(1 if v else 0)
    def write_int16(self, v): self._p("h", v)
    def write_uint16(self, v): self._p("H", v)
    def write_int32(self, v): self._p("i", v)
    def write_uint32(self, v): self._p("I", v)
    def write_int64(self, v): self._p("q", v)
    def write_uint64(self, v): self._p("Q", v & 0xFFFFFFFFFFFFFFFF)
    def write_float(self, v): self._p("f", v)
    def write_double(self, v): self._p("d", v)

    def write_char(self, ch: str):
        self._buf += ch.encode("utf-8", "surrogatepass")

    def write_decimal(self, v):
        self._buf += decimal_to_bytes(_decimal.Decimal(v))

    def write_datetime(self, v: _dt.datetime):
        self.write_uint64(datetime_to_ticks(v))

    def write_sqldatetime(self, v: SqlDateTime):
        self.write_int32(v.DayTicks)
        self.write_int32(v.TimeTicks)

    def write_guid(self, v: _uuid.UUID):
        self._buf += v.bytes_le

    def write_compact(self, v: int):
        if v < 0x80:
            self._buf.append(v & 0xFF)
        else:
            self._buf += bytes(((v >> 24) & 0xFF | 0x80, (v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF))

    def _write_compact_width(self, v: int, width: int):
        if width == 1:
            self._buf.append(v & 0xFF)
        else:
            self._buf += bytes(((v >> 24) & 0xFF | 0x80, (v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF))

    def write_string(self, s: str):
        n = utf16_len(s)
        data = s.encode("utf-8", "surrogatepass")
        self.write_compact(n)
        self._write_compact_width(len(data), compact_size(max_utf8_bytes(n)))
        self._buf += data

    def write_raw(self, b: bytes):
        self._buf += b

    # -- records / blocks
    def end_record(self):
        if self._stream is not None and len(self._buf) >= self._block:
            self.flush()

    def flush(self):
        if self._stream is not None and self._buf:
            self._stream.write(self._buf)
            self.bytes_written += len(self._buf)
            self._buf = bytearray()

    def getvalue(self) -> bytes:
        return bytes(self._buf)

    def close(self):
        self.flush()


class BinaryReader:
    """Reads a record stream from bytes / a file-like object."""

    def __init__(self, data=None, stream=None, uri: str = ""):
        if stream is not None:
            data = stream.read()
        self._mv = memoryview(bytes(data) if not isinstance(data, (bytes, bytearray, memoryview)) else data)
        self._pos = 0
        self.uri = uri

    def eof(self) -> bool:
        return self._pos >= len(self._mv)

    @property
    def position(self) -> int:
        return self._pos

    def _take(self, n):
        p = self._pos
        if p + n > len(self._mv):
            raise DryadLinqException(ErrorCode.EndOfStreamEncountered, f"end of stream in {self.uri or 'buffer'}")
        self._pos = p + n
        return self._mv[p:p + n]

    def _u(self, fmt):
        s = _S[fmt]
        return s.unpack(self._take(s.size))[0]

    def read_byte(self): return self._take(1)[0]
    def read_sbyte(self): return self._u("b")
    def read_bool(self): return self._take(1)[0] != 0
    def read_int16(self): return self._u("h")
    def read_uint16(self): return self._u("H")
    def read_int32(self): return self._u("i")
    def read_uint32(self): return self._u("I")
    def read_int64(self): return self._u("q")
    def read_uint64(self): return self._u("Q")
    def read_float(self): return self._u("f")
    def read_double(self): return self._u("d")

    def read_char(self) -> str:
        b0 = self.read_byte()
        n = 1 if b0 < 0x80 else 2 if b0 < 0xE0 else 3 if b0 < 0xF0 else 4
        rest = bytes(self._take(n - 1)) if n > 1 else b""
        return (bytes([b0]) + rest).decode("utf-8", "surrogatepass")

    def read_decimal(self): return bytes_to_decimal(bytes(self._take(16)))
    def read_datetime(self): return ticks_to_datetime(self.read_uint64())
    def read_sqldatetime(self): return SqlDateTime(self.read_int32(), self.read_int32())
    def read_guid(self): return _uuid.UUID(bytes_le=bytes(self._take(16)))

    def read_compact(self) -> int:
        b1 = self.read_byte()
        if b1 < 0x80:
            return b1
        b = self._take(3)
        return ((b1 & 0x7F) << 24) | (b[0] << 16) | (b[1] << 8) | b[2]

    def read_string(self) -> str:
        self.read_compact()
        nbytes = self.read_compact()
        return bytes(self._take(nbytes)).decode("utf-8", "surrogatepass")

    def read_raw(self, n: int) -> bytes:
        return bytes(self._take(n))


def encode_records(dtype, records) -> bytes:
    w = BinaryWriter()
    for r in records:
        dtype.encode(w, r)
    return w.getvalue()


def decode_records(dtype, data) -> list:
    r = BinaryReader(data)
    out = []
    while not r.eof():
        out.append(dtype.decode(r))
    return out


INDEX_BLOCK = 64     # records per block of the part index sidecar (io/partfile.write_index)


def write_records(path, dtype, records, index: bool = True) -> int:
    """Write a part file; with ``index`` also its record block index sidecar (every
    INDEX_BLOCK-th record's offset) when the records are not fixed-width."""
    offs = [] if index and dtype is not None and dtype.fixed_width is None else None
    n = 0
    with open(path, "wb") as f:
        w = BinaryWriter(f)
        for r in records:
            if offs is not None and n % INDEX_BLOCK == 0:
                offs.append(w.bytes_written + len(w._buf))
            dtype.encode(w, r)
            w.end_record()
            n += 1
        w.close()
        nbytes = w.bytes_written
    if offs is not None:
        from . import partfile as PF
        PF.write_index(path, n, nbytes, offs, INDEX_BLOCK)
    return nbytes


def read_records(path, dtype) -> list:
    with open(path, "rb") as f:
        return decode_records(dtype, f.read())


def iter_records(path, dtype):
    with open(path, "rb") as f:
        r = BinaryReader(stream=f, uri=str(path))
    while not r.eof():
        yield dtype.decode(r)
