"""Storage schemes (DataProvider registry).

Reference: LinqToDryad/DataProvider.cs:62-682 (per-scheme GetStreamInfo / Ingress / Egress /
CheckExistence / GetTemporaryStreamUri), DataPath.cs:39-58 (schemes partfile, hdfs, wasb,
azureblob).  Schemes here:

  * ``partfile:///abs/meta``  host partitioned files (byte-compatible, see io/partfile.py)
  * ``hbm://name``            device-resident tables kept in HBM by the GPU executor of this process
                              (one entry per local partition); the MI355X replacement for temp
                              partfiles between jobs
  * ``mem://name``            host-memory tables of this process (object executor / tests)
  * ``gen://kind?args``       synthetic generator stores (terasort, range, uniform), partition i is
                              a pure function of (args, i): idempotent under vertex re-execution

hdfs/wasb/azureblob are not available on a single MI355X node without network; asking for them
raises ``DryadLinqException(UnrecognizedDataSource)``.
"""
from __future__ import annotations

import os
import threading
import urllib.parse
import uuid

from ..errors import DryadLinqException, ErrorCode
from . import binary as B
from . import partfile as PF


def T_Pickle():
    from ..types import Pickle
    return Pickle


def parse_uri(uri: str):
    if "://" not in uri:
        # plain path => partfile
        return "partfile", os.path.abspath(uri), {}
    scheme, rest = uri.split("://", 1)
    scheme = scheme.lower()
    query = {}
    if "?" in rest:
        rest, q = rest.split("?", 1)
        query = {k: v[-1] for k, v in urllib.parse.parse_qs(q).items()}
    if scheme in ("partfile", "file"):
        path = rest
        if path.startswith("/") and len(path) > 2 and path[2] == ":":   # partfile:///C:/x
            path = path[1:]
        return scheme, path, query
    return scheme, rest, query


class DataProvider:
    scheme = ""

    def stream_info(self, uri) -> tuple[int, int]:
        raise NotImplementedError

    def exists(self, uri) -> bool:
        raise NotImplementedError

    def check_existence(self, uri, delete_if_exists: bool):
        if self.exists(uri):
            if not delete_if_exists:
                raise DryadLinqException(ErrorCode.StreamAlreadyExists, f"can't output to existing table {uri}")
            self.delete(uri)

    def delete(self, uri):
        raise NotImplementedError

    def read_partition(self, uri, i: int, dtype):
        raise NotImplementedError

    def write_table(self, uri, partitions: list, dtype, delete_if_exists=True):
        raise NotImplementedError

    def temp_uri(self, name: str) -> str:
        raise NotImplementedError

    def read_all(self, uri, dtype):
        n, _ = self.stream_info(uri)
        for i in range(n):
            yield from self.read_partition(uri, i, dtype)


class PartfileProvider(DataProvider):
    scheme = "partfile"

    def _path(self, uri):
        return parse_uri(uri)[1]

    def stream_info(self, uri):
        m = PF.read_meta(self._path(uri))
        return m.count, m.total_size

    def exists(self, uri):
        return os.path.exists(self._path(uri))

    def delete(self, uri, background: bool = False):
        path = self._path(uri)
        PF.delete(path, background=background)
        if os.path.exists(path + ".dryadtype"):
            os.remove(path + ".dryadtype")

    def part_paths(self, uri):
        return PF.read_meta(self._path(uri)).paths()

    def schema(self, uri):
        from ..runtime.jobmanager import read_schema
        return read_schema(self._path(uri))

    def read_partition(self, uri, i, dtype):
        path = PF.read_meta(self._path(uri)).part_path(i)
        with open(path, "rb") as f:
            data = f.read()
        sch = self.schema(uri)
        if sch is not None and sch.get("format") == "rows":
            st = int(sch["stride"])
            return [data[i:i + st] for i in range(0, len(data), st)]
        if sch is not None and sch.get("format") == "pickle":
            import gzip
            import pickle
            from ..runtime.jobmanager import pickled_table_trusted
            if not pickled_table_trusted(self._path(uri)):
                raise DryadLinqException(
                    ErrorCode.FailedToDeserialize,
                    f"{uri} holds pickled records written by another process; loading them would run "
                    "code from the file (set DRYAD_TRUST_PICKLED_TABLES=1 to allow it)")
            if data[:2] == b"\x1f\x8b":
                data = gzip.decompress(data)
            return pickle.loads(data) if data else []
        if dtype is None or dtype == T_Pickle():
            dtype = sch["dtype"] if sch is not None else None
        if dtype is None:
            from ..types import LineRecordT
            dtype = LineRecordT
        if data[:2] == b"\x1f\x8b":       # gzip-compressed record stream (OutputDataCompressionScheme)
            import gzip
            data = gzip.decompress(data)
        return B.decode_records(dtype, data)

    def part_file(self, uri, i):
        """Path of part i when its bytes are the record stream itself (not gzip-compressed), so a
        reader can move them straight to HBM (io/reader.py); None otherwise."""
        path = PF.read_meta(self._path(uri)).part_path(i)
        with open(path, "rb") as f:
            if f.read(2) == b"\x1f\x8b":
                return None
        return path

    def read_partition_bytes(self, uri, i) -> bytes:
        """The decoded record-stream bytes of part i (gzip-compressed parts are inflated)."""
        path = PF.read_meta(self._path(uri)).part_path(i)
        with open(path, "rb") as f:
            data = f.read()
        if data[:2] == b"\x1f\x8b":
            import gzip
            data = gzip.decompress(data)
        return data

    def write_table(self, uri, partitions, dtype, delete_if_exists=True):
        """Ingress: one part file per partition (records in DryadLinqBinary)."""
        meta_path = self._path(uri)
        if delete_if_exists:
            PF.delete(meta_path)
        os.makedirs(os.path.dirname(os.path.abspath(meta_path)) or ".", exist_ok=True)
        base = PF.default_base(meta_path)
        os.makedirs(os.path.dirname(base), exist_ok=True)
        tmps = []
        for pos, recs in enumerate(partitions):
            tmp = PF.tmp_part_path(base, pos, 0, pos, 0)
            if isinstance(recs, (bytes, bytearray)):
                with open(tmp, "wb") as f:
                    f.write(recs)
            else:
                B.write_records(tmp, dtype, recs)
            tmps.append(tmp)
        meta = PF.commit_parts(meta_path, base, tmps)
        if dtype is not None:
            from ..runtime.jobmanager import write_schema
            write_schema(meta_path, dtype, "binary")
        return meta

    def temp_uri(self, name):
        root = os.environ.get("DRYAD_TEMP_DIR") or os.path.join(os.environ.get("TMPDIR", "/tmp"), "DryadLinqTemp")
        os.makedirs(root, exist_ok=True)
        return "partfile://" + os.path.join(root, name)

    def rows_part(self, uri, i):
        """(memory map [n, stride] uint8, key_off, key_len) of part i of a raw-rows table, or None."""
        import numpy as np
        sch = self.schema(uri)
        if sch is None or sch.get("format") != "rows":
            return None
        path = PF.read_meta(self._path(uri)).part_path(i)
        st = int(sch["stride"])
        size = os.path.getsize(path)
        mm = np.memmap(path, dtype=np.uint8, mode="r", shape=(size // st, st)) if size else \
            np.zeros((0, st), dtype=np.uint8)
        return mm, int(sch.get("key_off", 0)), int(sch.get("key_len", st))


class _MemoryTables:
    def __init__(self):
        self.tables = {}
        self.lock = threading.Lock()


_MEM = _MemoryTables()


class MemProvider(DataProvider):
    """Host-memory tables: ``{name: (dtype, [partition lists])}``."""
    scheme = "mem"

    def _name(self, uri):
        return parse_uri(uri)[1]

    def stream_info(self, uri):
        t = _MEM.tables.get(self._name(uri))
        if t is None:
            raise DryadLinqException(ErrorCode.StreamDoesNotExist, f"no such table {uri}")
        return len(t[1]), sum(len(p) for p in t[1])

    def exists(self, uri):
        return self._name(uri) in _MEM.tables

    def delete(self, uri):
        _MEM.tables.pop(self._name(uri), None)

    def read_partition(self, uri, i, dtype):
        return list(_MEM.tables[self._name(uri)][1][i])

    def write_table(self, uri, partitions, dtype, delete_if_exists=True):
        with _MEM.lock:
            _MEM.tables[self._name(uri)] = (dtype, [list(p) for p in partitions])

    def temp_uri(self, name):
        return "mem://" + name


class HbmProvider(DataProvider):
    """Device-resident tables of this process: ``{name: (dtype, [local partition batches])}``.
    On a GPU rank each entry holds the rank's partitions as columnar batches in HBM."""
    scheme = "hbm"
    tables: dict = {}

    def _name(self, uri):
        return parse_uri(uri)[1]

    def stream_info(self, uri):
        t = self.tables.get(self._name(uri))
        if t is None:
            raise DryadLinqException(ErrorCode.StreamDoesNotExist, f"no such HBM table {uri}")
        return t["partitions"], t.get("bytes", 0)

    def exists(self, uri):
        return self._name(uri) in self.tables

    def delete(self, uri):
        ent = self.tables.pop(self._name(uri), None)
        if ent is not None and ent.get("pool") is not None:
            for b in ent.get("pins", []):
                ent["pool"].unpin(b)

    def put(self, uri, entry: dict):
        if self._name(uri) in self.tables:
            self.delete(uri)
        self.tables[self._name(uri)] = entry

    def get(self, uri) -> dict:
        t = self.tables.get(self._name(uri))
        if t is None:
            raise DryadLinqException(ErrorCode.StreamDoesNotExist, f"no such HBM table {uri}")
        return t

    def read_partition(self, uri, i, dtype):
        t = self.get(uri)
        b = t["local"].get(i)
        if b is None:
            raise DryadLinqException(ErrorCode.FailedToGetReadPathsForStream, f"partition {i} of {uri} is not resident on this rank")
        return b.to_objects() if hasattr(b, "to_objects") else list(b)

    def write_table(self, uri, partitions, dtype, delete_if_exists=True):
        self.put(uri, {"dtype": dtype, "partitions": len(partitions), "local": dict(enumerate(partitions))})

    def temp_uri(self, name):
        return "hbm://" + name


class HostProvider(DataProvider):
    """Pinned-host tables (the tier between HBM and disk, io/hosttable.py): ``{name: entry}`` with
    ``entry["local"][p]`` = a ``HostRows`` row table or a record list for each partition this
    process holds.  Out-of-core sorts (ops/extsort.py) write their output here; on the object
    executors ``host://`` behaves like ``mem://``."""
    scheme = "host"
    tables: dict = {}

    def _name(self, uri):
        return parse_uri(uri)[1]

    def stream_info(self, uri):
        t = self.get(uri)
        return t["partitions"], sum(getattr(v, "nbytes", 0) for v in t["local"].values())

    def exists(self, uri):
        return self._name(uri) in self.tables

    def delete(self, uri):
        ent = self.tables.pop(self._name(uri), None)
        if ent is not None:
            for v in ent["local"].values():
                if hasattr(v, "release"):
                    v.release()

    def put(self, uri, entry: dict):
        if self._name(uri) in self.tables:
            self.delete(uri)
        self.tables[self._name(uri)] = entry

    def get(self, uri) -> dict:
        t = self.tables.get(self._name(uri))
        if t is None:
            raise DryadLinqException(ErrorCode.StreamDoesNotExist, f"no such host table {uri}")
        return t

    def local_rows(self, uri, i):
        """The ``HostRows`` of partition i (None if it is held as records)."""
        from .hosttable import HostRows
        v = self.get(uri)["local"].get(i)
        return v if isinstance(v, HostRows) else None

    def read_partition(self, uri, i, dtype):
        b = self.get(uri)["local"].get(i)
        if b is None:
            raise DryadLinqException(ErrorCode.FailedToGetReadPathsForStream, f"partition {i} of {uri} is not resident in this process")
        return b.to_objects() if hasattr(b, "to_objects") else list(b)

    def write_table(self, uri, partitions, dtype, delete_if_exists=True):
        self.put(uri, {"dtype": dtype, "partitions": len(partitions),
                       "local": {i: list(p) for i, p in enumerate(partitions)}})

    def temp_uri(self, name):
        return "host://" + name


class GenProvider(DataProvider):
    """Synthetic generator stores.  ``gen://range?count=N&partitions=P[&start=S]`` yields ints;
    ``gen://terasort?records=N&partitions=P&seed=S`` yields 100-byte TeraSort records (as bytes on
    the object path, generated directly in HBM by the GPU executor);
    ``gen://points?count=N&partitions=P&blobs=B&seed=S`` yields 128-dim float32 blob points
    (tuples on the object path, one [n, 128] HBM tensor on the GPU executor);
    ``gen://records64?count=N&partitions=P&keys=K&seed=S[&cols=C]`` yields 64-byte records of 8
    int64 fields (Key uniform in [0, K), V1..V7 31-bit values), columnar in HBM; ``&mode=dim``
    makes it a dimension table (keys a bijection of [0, K), payload a function of the key);
    ``gen://names?count=N&partitions=P&keys=K&seed=S[&mode=dim]`` yields (Name, V1, V2) records with
    a string key "u<decimal>" (models/names.py)."""
    scheme = "gen"

    def _args(self, uri):
        _, kind, q = parse_uri(uri)
        return kind.strip("/"), q

    def stream_info(self, uri):
        kind, q = self._args(uri)
        p = int(q.get("partitions", 1))
        if kind == "terasort":
            return p, int(q.get("records", 0)) * 100
        if kind == "points":
            return p, int(q.get("count", 0)) * 4 * 128
        if kind == "records64":
            return p, int(q.get("count", 0)) * 8 * int(q.get("cols", 8))
        if kind == "names":
            from ..models import names as NM
            return p, int(q.get("count", 0)) * (16 + max(16, NM.namelen(q)))
        return p, int(q.get("count", 0)) * 4

    def exists(self, uri):
        return True

    def schema(self, uri):
        from .. import types as T
        kind, _ = self._args(uri)
        dt = {"range": T.Int32, "terasort": T.Pickle, "points": T.Vector(T.Float32, 128)}.get(kind)
        if kind == "records64":
            from ..models.records_cpu import FIELDS
            ncols = int(self._args(uri)[1].get("cols", 8))
            dt = T.RecordT([(f, T.Int64) for f in FIELDS[:ncols]], tuple)
        if kind == "names":
            from ..models import names as NM
            dt = NM.dtype()
        return {"dtype": dt}

    def delete(self, uri):
        raise DryadLinqException(ErrorCode.AttemptToReadFromAWriteStream, "generator stores are read-only")

    def bounds(self, uri, i):
        kind, q = self._args(uri)
        p = int(q.get("partitions", 1))
        n = int(q.get("records", q.get("count", 0)))
        return (n * i) // p, (n * (i + 1)) // p

    def read_partition(self, uri, i, dtype):
        kind, q = self._args(uri)
        lo, hi = self.bounds(uri, i)
        if kind == "range":
            start = int(q.get("start", 0))
            return list(range(start + lo, start + hi))
        if kind == "terasort":
            from ..models.terasort_cpu import gen_records
            return gen_records(lo, hi - lo, int(q.get("seed", 0)))
        if kind == "points":
            from ..models.kmeans_cpu import gen_point_records
            return gen_point_records(lo, hi - lo, int(q.get("blobs", 64)), int(q.get("seed", 0)))
        if kind == "records64":
            from ..models.records_cpu import gen_records
            from ..models.records_cpu import dim_multiplier
            nk = int(q.get("keys", 1 << 20))
            return gen_records(lo, hi - lo, nk, int(q.get("seed", 0)), int(q.get("cols", 8)),
                               dim_multiplier(nk) if q.get("mode") == "dim" else 0)
        if kind == "names":
            from ..models import names as NM
            from ..models.records_cpu import dim_multiplier
            nk = int(q.get("keys", 1 << 20))
            return NM.host_records(lo, hi - lo, nk, int(q.get("seed", 0)),
                                   dim_multiplier(nk) if q.get("mode") == "dim" else 0, NM.namelen(q))
        raise DryadLinqException(ErrorCode.UnrecognizedDataSource, f"unknown generator {kind}")

    def temp_uri(self, name):
        raise DryadLinqException(ErrorCode.AttemptToReadFromAWriteStream, "generator stores are read-only")


class TextProvider(DataProvider):
    """Plain text files as LineRecord tables (reference A-8: LineRecord text I/O).

    ``text:///path/to/file.txt?partitions=P`` splits one file into P byte ranges cut at line
    boundaries; ``text:///path/to/dir`` (or a glob ``text:///path/part-*``) is one partition per
    file.  Lines end at '\\n', '\\r\\n' or a lone '\\r' (Appendix C).  Written tables are a directory of
    part files ``part-%08X.txt``."""
    scheme = "text"

    def _spec(self, uri):
        _, path, q = parse_uri(uri)
        return path, q

    def _files(self, uri):
        import glob as _glob
        path, _ = self._spec(uri)
        if os.path.isdir(path):
            return sorted(os.path.join(path, f) for f in os.listdir(path) if not f.startswith("."))
        if any(ch in path for ch in "*?["):
            return sorted(_glob.glob(path))
        return [path]

    def ranges(self, uri):
        """[(file, start, end)] per partition, cut after a '\n'."""
        files = self._files(uri)
        _, q = self._spec(uri)
        p = int(q.get("partitions", 0) or 0)
        if len(files) != 1 or p <= 1:
            return [(f, 0, os.path.getsize(f)) for f in files]
        f = files[0]
        size = os.path.getsize(f)
        cuts = [0]
        with open(f, "rb") as fh:
            for k in range(1, p):
                pos = max(cuts[-1], (size * k) // p)
                fh.seek(pos)
                if pos > 0:
                    fh.seek(pos - 1)
                    if fh.read(1) != b"\n":
                        fh.readline()
                cuts.append(min(size, fh.tell()))
        cuts.append(size)
        return [(f, cuts[i], cuts[i + 1]) for i in range(p)]

    def stream_info(self, uri):
        r = self.ranges(uri)
        return len(r), sum(b - a for _, a, b in r)

    def exists(self, uri):
        return bool(self._files(uri)) and all(os.path.exists(f) for f in self._files(uri))

    def delete(self, uri):
        import shutil
        path, _ = self._spec(uri)
        if os.path.isdir(path):
            shutil.rmtree(path)
        elif os.path.exists(path):
            os.remove(path)

    def schema(self, uri):
        from ..types import LineRecordT
        return {"dtype": LineRecordT}

    def read_partition_bytes(self, uri, i) -> bytes:
        f, a, b = self.ranges(uri)[i]
        with open(f, "rb") as fh:
            fh.seek(a)
            return fh.read(b - a)

    def read_partition(self, uri, i, dtype):
        from ..types import LineRecord
        data = self.read_partition_bytes(uri, i)
        if not data:
            return []
        import re
        lines = re.split(rb"\r\n|\r|\n", data)
        if lines and lines[-1] == b"":
            lines.pop()
        return [LineRecord(x.decode("utf-8", "replace")) for x in lines]

    def write_table(self, uri, partitions, dtype, delete_if_exists=True):
        path, _ = self._spec(uri)
        if delete_if_exists:
            self.delete(uri)
        os.makedirs(path, exist_ok=True)
        for i, recs in enumerate(partitions):
            tmp = os.path.join(path, f".part-{i:08X}.tmp")
            with open(tmp, "wb") as fh:
                for r in recs:
                    fh.write((r.Line if hasattr(r, "Line") else str(r)).encode("utf-8") + b"\n")
            os.replace(tmp, os.path.join(path, f"part-{i:08X}.txt"))

    def temp_uri(self, name):
        root = os.environ.get("DRYAD_TEMP_DIR") or os.path.join(os.environ.get("TMPDIR", "/tmp"), "DryadLinqTemp")
        return "text://" + os.path.join(root, name)


_PROVIDERS = {p.scheme: p for p in (PartfileProvider(), MemProvider(), HbmProvider(), HostProvider(), GenProvider(),
                                    TextProvider())}
_PROVIDERS["file"] = _PROVIDERS["partfile"]


def provider_for(uri: str) -> DataProvider:
    scheme = parse_uri(uri)[0]
    p = _PROVIDERS.get(scheme)
    if p is None:
        raise DryadLinqException(ErrorCode.UnrecognizedDataSource,
                                 f"unsupported storage scheme '{scheme}' (available: {sorted(_PROVIDERS)})")
    return p


def register_provider(p: DataProvider):
    _PROVIDERS[p.scheme] = p


def unique_name(prefix="tmp") -> str:
    return f"{prefix}-{uuid.uuid4().hex[:12]}"
