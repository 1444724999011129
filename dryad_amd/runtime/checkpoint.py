"""Persisted stage outputs: what lets a relaunched gang resume a job after a lost rank process.

The reference survives the loss of a vertex process because every vertex output is a file that
outlives it: a failed vertex is re-executed from its persisted inputs (DrActiveVertex::
ReactToFailedVertex, GraphManager/vertex/DrVertex.cpp:1042-1171; DrGraph::ReportFailure,
DrGraph.cpp:392-456), and a partition becomes visible only through commit-by-rename
(DrPartitionFile.cpp:496-600).  Here channels live in HBM, inside the rank processes; when one of
them dies the launcher (csrc/launcher/dryad_launch.cpp) stops the gang and starts a fresh one,
and the job's stages whose outputs were persisted here are not run again.

Layout: ``<root>/<job key>/s<stage>/p<partition>.{json,pkl,d0..d7}`` plus a ``.done`` marker
written by rename after the data files, so a rank that died mid-write leaves no partial
checkpoint.  The job key is the job's sequence number in the process plus a digest of its plan: a
relaunched script submits the same jobs in the same order.  Tensors (device or host) are written
raw by the native part writer (io/writer.PartWriter: HBM -> pinned ring -> pwrite threads), in
PIECE-byte pieces round-robin over up to SPLIT_MAX data files so the writer threads work on
distinct inodes; the JSON layout records every piece's (file, offset, bytes), and a load reads
each piece straight into its slice of the rebuilt tensor (io/reader.read_to_device).  Host record
lists are pickles this framework wrote itself.  The default root of a relaunching launcher is a
launcher-owned directory under /dev/shm (host memory that outlives the rank processes).

Every save is checked against ``CheckpointBudgetBytes`` (context property; default 90% of the
checkpoint file system's free space when the job starts): a stage that would pass it is not
persisted (a ``persist_skipped`` job event; after a relaunch it simply runs again), and a save that
fails (full disk, an unpicklable record) is dropped the same way instead of failing the job.
"""
from __future__ import annotations

import hashlib
import json
import os
import pickle
import uuid

import torch

from ..gpu.table import DeviceTable, Ported, PortTables
from ..tools.replay import _shape_from, _shape_json

PIECE = 256 << 20            # bytes per written piece (round-robin over the data files)


def job_key(seq: int, plan) -> str:
    """Stable across processes and relaunches: the job's order in the script and its plan's
    structure (stage names, partition counts, edges, operator names; not lambda reprs or the
    generated names of temporary outputs, which differ between processes)."""
    shape = [(s.name, s.partitions, [(i.src, i.kind) for i in s.inputs], [o["op"] for o in s.ops])
             for s in plan.stages]
    d = hashlib.blake2b(repr(shape).encode(), digest_size=8).hexdigest()
    return f"job{seq:04d}-{d}"


def _table_tensors(t: DeviceTable, prefix: str = "") -> tuple[list, dict]:
    """[(key, contiguous tensor)] of a table (left where it is: device or host) + its layout."""
    out = [(prefix + "col:" + c, v[: t.n].contiguous()) for c, v in t.cols.items()]
    if t.rows is not None:
        out.append((prefix + "rows", t.rows[: t.n].contiguous()))
    if t.heap is not None:
        out.append((prefix + "heap", t.heap.contiguous()))
    for f_, h in t.strs.items():
        out.append((prefix + "str:" + f_, h.contiguous()))
    return out, dict(n=t.n, shape=_shape_json(t.shape), cols=list(t.cols))


def _table_from(tensors: dict, meta: dict, prefix: str = "") -> DeviceTable:
    g = lambda k: tensors.get(prefix + k)  # noqa: E731
    cols = {c: g("col:" + c) for c in meta["cols"]}
    strs = {k[len(prefix) + 4:]: v for k, v in tensors.items() if k.startswith(prefix + "str:")}
    return DeviceTable(meta["n"], _shape_from(meta["shape"]), cols, rows=g("rows"), heap=g("heap"), strs=strs)


def _dtype_name(dt: torch.dtype) -> str:
    return str(dt).split(".")[-1]


class StageCheckpoint:
    def __init__(self, root: str, key: str, budget: int | None = None):
        self.dir = os.path.join(root, key)
        os.makedirs(self.dir, exist_ok=True)
        if budget is None:
            st = os.statvfs(self.dir)
            budget = int(st.f_bavail * st.f_frsize * 0.9)
        self.budget = int(budget)
        self.used = 0

    def _base(self, sid: int, p: int) -> str:
        return os.path.join(self.dir, f"s{sid}", f"p{p}")

    def _files(self, base: str) -> list:
        d, name = os.path.split(base)
        try:
            return [os.path.join(d, f) for f in os.listdir(d) if f.startswith(name + ".")]
        except OSError:
            return []

    def drop(self, sid: int, p: int) -> None:
        base = self._base(sid, p)
        for f in [base + ".done"] + self._files(base):       # the marker first: never half a checkpoint
            try:
                os.remove(f)
            except OSError:
                pass

    def has(self, sid: int, p: int) -> bool:
        return os.path.exists(self._base(sid, p) + ".done")

    @staticmethod
    def persistable(value) -> bool:
        if value is None or isinstance(value, DeviceTable):
            return True
        if isinstance(value, Ported):
            return isinstance(value.table, DeviceTable)
        if isinstance(value, PortTables):
            return all(x is None or isinstance(x, (DeviceTable, list)) for x in value.tables)
        return isinstance(value, list)

    @staticmethod
    def _parts(value):
        """(meta, [(key, tensor)], host object or None) of a vertex output."""
        meta, tensors, obj = {}, [], None
        if value is None:
            meta["kind"] = "none"
        elif isinstance(value, DeviceTable):
            tensors, meta["table"] = _table_tensors(value)
            meta["kind"] = "table"
        elif isinstance(value, Ported):
            tensors, meta["table"] = _table_tensors(value.table)
            meta.update(kind="ported", offsets=list(value.offsets), order=value.order)
        elif isinstance(value, PortTables):
            meta.update(kind="port_tables", ports=[])
            objs = []
            for k, x in enumerate(value.tables):
                if isinstance(x, DeviceTable):
                    tk, mk = _table_tensors(x, prefix=f"{k}/")
                    tensors += tk
                    meta["ports"].append(dict(kind="table", table=mk))
                else:
                    meta["ports"].append(dict(kind="objects", index=len(objs)))
                    objs.append(x)
            obj = objs
        else:
            meta["kind"] = "objects"
            obj = value
        return meta, tensors, obj

    @staticmethod
    def nbytes(value) -> int:
        """Bytes a save of ``value`` writes: its tensors exactly, host records estimated at 32
        bytes each (they are pickled)."""
        if not StageCheckpoint.persistable(value):
            return 0
        _, tensors, obj = StageCheckpoint._parts(value)
        est = 0
        if obj is not None:
            est = 32 * sum(len(x) if isinstance(x, list) else 1 for x in (obj if isinstance(value, PortTables) else [obj]))
        return sum(t.numel() * t.element_size() for _, t in tensors) + est

    def save(self, sid: int, p: int, value) -> int:
        """Persist one vertex output -> bytes written (0: a kind this store does not hold; the
        stage then simply runs again after a relaunch).  Raises on I/O errors (the caller drops
        the partial checkpoint and records it)."""
        if not self.persistable(value):
            return 0
        base = self._base(sid, p)
        os.makedirs(os.path.dirname(base), exist_ok=True)
        tag = uuid.uuid4().hex[:8]
        meta, tensors, obj = self._parts(value)
        total = sum(t.numel() * t.element_size() for _, t in tensors)
        written = total
        layout = []
        if total:
            from ..io.writer import SPLIT_MAX, PartWriter
            k = max(1, min(SPLIT_MAX, -(-total // PIECE)))
            paths = [f"{base}.d{j}.{tag}" for j in range(k)]
            dev = next((t.device for _, t in tensors if t.is_cuda), None)
            foff, j = [0] * k, 0
            with PartWriter(paths, dev) as w:
                for key, t in tensors:
                    flat = t.reshape(-1).view(torch.uint8)
                    pieces = []
                    for a in range(0, flat.numel(), PIECE):
                        m = min(PIECE, flat.numel() - a)
                        f = j % k
                        w.write(flat[a: a + m], file=f)
                        pieces.append((f, foff[f], m))
                        foff[f] += m
                        j += 1
                    layout.append(dict(key=key, dtype=_dtype_name(t.dtype), shape=list(t.shape), pieces=pieces))
            for jj, f in enumerate(paths):
                os.replace(f, f"{base}.d{jj}")
        else:
            layout = [dict(key=key, dtype=_dtype_name(t.dtype), shape=list(t.shape), pieces=[]) for key, t in tensors]
        meta["tensors"] = layout
        if obj is not None:
            with open(f"{base}.pkl.{tag}", "wb") as f:
                pickle.dump(obj, f)
                written += f.tell()
            os.replace(f"{base}.pkl.{tag}", base + ".pkl")
        with open(f"{base}.json.{tag}", "w") as f:
            json.dump(meta, f)
        os.replace(f"{base}.json.{tag}", base + ".json")
        with open(f"{base}.done.{tag}", "w") as f:
            f.write("1")
        os.replace(f"{base}.done.{tag}", base + ".done")            # commit by rename
        self.used += written
        return max(written, 1)

    def load(self, sid: int, p: int, device):
        base = self._base(sid, p)
        with open(base + ".json") as f:
            meta = json.load(f)
        kind = meta["kind"]
        dev = torch.device(device)
        tensors = {}
        for ent in meta.get("tensors", []):
            t = torch.empty(ent["shape"], dtype=getattr(torch, ent["dtype"]), device=dev)
            flat = t.view(-1).view(torch.uint8)
            pos = 0
            for f, off, m in ent["pieces"]:
                path = f"{base}.d{f}"
                if dev.type == "cuda":
                    from ..io import reader as RD
                    RD.read_to_device(path, dev, offset=off, length=m, out=flat[pos: pos + m])
                else:
                    with open(path, "rb") as fh:
                        fh.seek(off)
                        fh.readinto(memoryview(flat[pos: pos + m].numpy()))
                pos += m
            tensors[ent["key"]] = t
        obj = None
        if os.path.exists(base + ".pkl"):
            with open(base + ".pkl", "rb") as f:           # written by this framework (save above)
                obj = pickle.load(f)
        if kind == "none":
            return None
        if kind == "table":
            return _table_from(tensors, meta["table"])
        if kind == "ported":
            return Ported(_table_from(tensors, meta["table"]), meta["offsets"], meta["order"])
        if kind == "port_tables":
            tabs = []
            for k, pm in enumerate(meta["ports"]):
                tabs.append(_table_from(tensors, pm["table"], prefix=f"{k}/") if pm["kind"] == "table"
                            else obj[pm["index"]])
            return PortTables(tabs)
        return obj


def from_env(ctx):
    """The checkpoint root when stage outputs are to be persisted: the context's
    PersistStageOutputs (a directory, or True for DRYAD_CHECKPOINT_DIR), or automatically under a
    launcher that relaunches lost gangs (DRYAD_GANG_RESTARTS > 0).  None: no persistence."""
    want = ctx._props.get("PersistStageOutputs")
    if want is False:
        return None
    if isinstance(want, str):
        return want
    root = os.environ.get("DRYAD_CHECKPOINT_DIR")
    if want or (root and int(os.environ.get("DRYAD_GANG_RESTARTS", "0") or 0) > 0):
        if not root:
            from .executor import dryad_home
            root = os.path.join(dryad_home(ctx), "checkpoints")
        return root
    return None


def gang_epoch() -> int:
    """How many times the launcher has relaunched this job's gang (0: the first start)."""
    return int(os.environ.get("DRYAD_GANG_EPOCH", "0") or 0)
